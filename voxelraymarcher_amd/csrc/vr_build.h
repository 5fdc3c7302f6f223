// vr_build.h -- the GPU scene builder (vr_build.hip), used by vr_host.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace vr {

// Device buffers of one scene (owned by the caller afterwards); layouts as in
// vr_internal.h, identical to the host builder's.
struct GpuScene {
    void* region_slot = nullptr; uint64_t region_slot_bytes = 0;
    void* vcs_mask = nullptr;    uint64_t vcs_mask_bytes = 0;
    void* vcs_vals = nullptr;    uint64_t vcs_vals_bytes = 0;
    void* ht_meta = nullptr;     uint64_t ht_meta_bytes = 0;
    void* ht_slots = nullptr;    uint64_t ht_slots_bytes = 0;
    uint32_t D = 1;
    int32_t min_coord = 0;
    uint32_t n_regions = 0;
    uint64_t n_voxels = 0;
};

// Build from device-resident voxels (xyz: 3n int32, rgb: n colours) on `stream`.
// 0 = OK; -1 invalid input, -2 HIP error, -5 build failure (message in err).
// On failure the buffers already allocated in `out` are the caller's to free.
int build_scene_gpu(int store, const int32_t* xyz, const uint32_t* rgb, uint64_t n, hipStream_t stream,
                    GpuScene& out, std::string& err);

}  // namespace vr
