// multi_gpu.h -- the CLI's multi-GPU frame: ONE process drives
// N devices of the node.  Per rank: hipSetDevice, its own replica of the scene, its own
// stream; the frame is dealt as the 2-D tile deal of include/vr.h (vr_render_tiles: every
// 16-row band cut into 16-column blocks, block j of band b -> rank (j + stride*b) % N), each
// rank packs its tiles to RGB8 (vr_pack_rgb8, writeColorToFramebuffer's 3 B per pixel), an
// RCCL gather over xGMI collects the equal-size tile buffers on device 0 (ncclCommInitAll,
// one ncclGather per rank inside one group), and device 0 undoes the deal
// (vr_assemble_tiles).  This is runRaymarchingKernel + writeResultingImageToDisk
// (main/Main.cu:105-174) per device; the reference itself renders on one device only
// (Main.cu:23,82-94).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "vr.h"

namespace vrx {

struct MultiGpuTiming {
    double frame_ms = 0;                 // host clock: first rank's launch -> frame assembled on device 0
    std::vector<float> rank_render_ms;   // per rank: its tile render (HIP events on its stream)
};

class MultiGpuFrame {
public:
    MultiGpuFrame() = default;
    MultiGpuFrame(const MultiGpuFrame&) = delete;
    MultiGpuFrame& operator=(const MultiGpuFrame&) = delete;
    ~MultiGpuFrame();

    // Devices 0..ngpus-1 (error if fewer are visible), the scene built on each, the RCCL
    // communicators and the buffers of a width x height frame.  Returns false with error().
    bool init(int ngpus, vr_store store, const std::vector<int32_t>& xyz, const std::vector<uint32_t>& rgb,
              uint32_t width, uint32_t height, uint32_t band_rows = 16, uint32_t tile_cols = 16);
    // One frame: every rank renders and packs its tiles, the gather to device 0, the assembly.
    // On return the RGB8 frame is in device 0's memory (frame_rgb()) and complete.
    bool render(vr_algo algo, const vr_camera& cam, const vr_lighting& lit, const float translation[3],
                uint32_t scale, MultiGpuTiming* timing = nullptr);
    // The assembled frame copied to host memory (width * height * 3 bytes).
    bool download(std::vector<uint8_t>& out);

    const vr_scene* scene(int rank) const { return ranks_[rank].scene; }
    int ngpus() const { return (int)ranks_.size(); }
    const std::string& error() const { return err_; }

private:
    struct Rank {
        int device = 0;
        vr_scene* scene = nullptr;
        void* stream = nullptr;        // hipStream_t
        void* comm = nullptr;          // ncclComm_t
        uint32_t* words = nullptr;     // this rank's tiles, packed 0x00RRGGBB
        uint8_t* rgb = nullptr;        // the same as RGB8 (the gather's send buffer)
        void* ev0 = nullptr;           // hipEvent_t around the render
        void* ev1 = nullptr;
    };
    bool fail(const std::string& msg);
    std::vector<Rank> ranks_;
    uint8_t* gathered_ = nullptr;      // device 0: N tile buffers of RGB8, rank order
    uint8_t* frame_ = nullptr;         // device 0: the assembled RGB8 frame
    uint32_t W_ = 0, H_ = 0, band_rows_ = 16, tile_cols_ = 16;
    uint64_t rank_words_ = 0;
    std::string err_;
};

}  // namespace vrx
