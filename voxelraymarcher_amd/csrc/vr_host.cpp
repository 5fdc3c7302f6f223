// vr_host.cpp -- host side of libvr.so: scene build (region bucketing, VCS
// and cuckoo images), device upload, the C ABI of include/vr.h, the
// synthetic grid generator and the .vox CSV reader/writer.
//
// Replaces, on the host: VoxelSceneCPU (geometry/VoxelSceneCPU.cuh:13-131),
// the VoxelClusterStore / CuckooHashTable constructors
// (storage/VoxelClusterStore.cuh:37-85, storage/CuckooHashTable.cuh:20-178),
// VoxelFile::readVoxelFile (geometry/VoxelFile.cuh:9-35), Camera::Camera
// (renderer/camera/Camera.cuh:11-23) and runRaymarchingKernel
// (main/Main.cu:105-163).  The nested unordered_maps of the reference become
// one sort of (region, key) records; pointers become 32-bit offsets.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <mutex>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstddef>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "vr.h"
#include "vr_build.h"
#include "vr_internal.h"

namespace {

thread_local std::string g_err = "";

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
int hip_fail(hipError_t e, const char* what) {
    return fail(VR_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// static_cast<int32_t>(float) with the CUDA semantics used on the device.
inline int32_t f2i(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return INT32_MAX;
    if (f <= -2147483648.0f) return INT32_MIN;
    return (int32_t)f;
}

// ---------------------------------------------------------------- camera math
struct f3 { float x, y, z; };
inline f3 add(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline f3 sub(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline f3 scl(float t, f3 a) { return {t * a.x, t * a.y, t * a.z}; }
inline f3 unit(f3 a) {
    float len = std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
    return {a.x / len, a.y / len, a.z / len};
}
inline f3 cross(f3 a, f3 b) {   // Vector3.cuh:154-159
    return {(a.y * b.z - a.z * b.y), (-(a.x * b.z - a.z * b.x)), (a.x * b.y - a.y * b.x)};
}

// ------------------------------------------------------------- cuckoo hashing
const uint32_t kPrimes[14] = {668265261u, 12289u, 24593u, 49157u, 98317u, 196613u, 393241u,
                              786433u, 1572869u, 3145739u, 6291469u, 12582917u, 25165843u, 50331653u};

inline uint32_t hash1(uint32_t k, uint32_t offset) {   // CuckooHashTable.cuh:181-190
    k = (k + 0x7ed55d16u) + (k << 12);
    k = (k ^ 0xc761c23cu) ^ (uint32_t)((int32_t)k >> 19);
    k = (k + 0x165667b1u) + (k << 5);
    k = (k + 0xd3a2646cu) ^ (k << 9);
    k = (k + 0xfd7046c5u) + (k << 3);
    k = (k ^ 0xb55a4f09u) ^ (uint32_t)((int32_t)k >> 16);
    return k + offset;
}
inline uint32_t hash2(uint32_t k, uint32_t prime) {    // CuckooHashTable.cuh:193-202
    k = (k ^ 61u) ^ (uint32_t)((int32_t)k >> 16);
    k = k + (k << 3);
    k = k ^ (uint32_t)((int32_t)k >> 4);
    k = k * prime;
    k = k ^ (uint32_t)((int32_t)k >> 15);
    return k;
}

// createCuckooHashTable (CuckooHashTable.cuh:97-178) into interleaved
// {key,value} slots: table 1 at slots[0..M), table 2 at slots[M..2M).
// The rehash draws a new prime/offset from a seeded generator instead of
// rand() (Random.cuh:14-18): lookups do not depend on the placement.
bool cuckoo_build(const uint32_t* keys, const uint32_t* vals, uint32_t n, uint32_t* M_out,
                  uint32_t* prime_out, uint32_t* offset_out, std::vector<uint32_t>& slots,
                  size_t base_words) {
    const uint32_t M = (uint32_t)((double)n * 1.25);   // numElements * 1.25 (:23)
    uint32_t prime = kPrimes[0], offset = 0;
    uint64_t rng = 0x9E3779B97F4A7C15ull ^ (uint64_t)n ^ ((uint64_t)keys[0] << 20);
    uint32_t* t = nullptr;
    for (int attempt = 0; attempt < 4096; ++attempt) {
        slots.resize(base_words + 4 * (size_t)M);
        t = slots.data() + base_words;
        for (uint32_t i = 0; i < 2 * M; ++i) { t[2 * i] = vr::kEmpty; t[2 * i + 1] = 0; }
        bool rehash = false;
        for (uint32_t i = 0; i < n && !rehash; ++i) {
            uint32_t code = keys[i], value = vals[i], bucket = 0, it = 0;
            for (;;) {
                if (it >= 300000u) { rehash = true; break; }
                uint32_t* slot = bucket == 0 ? t + 2 * (size_t)(hash1(code, offset) % M)
                                             : t + 2 * ((size_t)M + hash2(code, prime) % M);
                if (slot[0] == vr::kEmpty) { slot[0] = code; slot[1] = value; break; }
                std::swap(slot[0], code);
                std::swap(slot[1], value);
                bucket ^= 1u;
                ++it;
            }
        }
        if (!rehash) {
            *M_out = M; *prime_out = prime; *offset_out = offset;
            return true;
        }
        rng = rng * 6364136223846793005ull + 1442695040888963407ull;
        prime = kPrimes[(rng >> 33) % 14u];
        rng = rng * 6364136223846793005ull + 1442695040888963407ull;
        offset = (uint32_t)((rng >> 33) % 25u);
    }
    return false;
}

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

}  // namespace

std::atomic<uint64_t> g_scene_serial{0};
struct vr_scene {
    // a process-unique id (the learned orders' view key: a later scene may reuse a freed
    // scene's address)
    const uint64_t serial = ++g_scene_serial;
    int device = 0;
    vr_store store = VR_STORE_VCS;
    uint32_t D = 1;
    int32_t min_coord = 0;
    uint32_t n_regions = 0;
    uint64_t n_voxels = 0;
    DevBuf region_slot, vcs_mask, vcs_vals, ht_meta, ht_slots;
    DevBuf vcs_cbits;   // derived (not part of vr_scene_digest): cluster-existence bits per region
    DevBuf ht_filter;   // derived (not part of vr_scene_digest): cuckoo key-presence bits per region
    uint64_t device_bytes() const {
        return region_slot.bytes + vcs_mask.bytes + vcs_vals.bytes + ht_meta.bytes + ht_slots.bytes + vcs_cbits.bytes +
               ht_filter.bytes;
    }
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

void free_scene(vr_scene* s) {
    if (!s) return;
    DevBuf* bufs[] = {&s->region_slot, &s->vcs_mask, &s->vcs_vals, &s->ht_meta, &s->ht_slots, &s->vcs_cbits,
                      &s->ht_filter};
    for (DevBuf* b : bufs)
        if (b->p) (void)hipFree(b->p);
    delete s;
}

int upload(DevBuf& b, const void* src, size_t bytes) {
    b.bytes = bytes;
    if (bytes == 0) return VR_OK;
    hipError_t e = hipMalloc(&b.p, bytes);
    if (e != hipSuccess) return fail(VR_E_NOMEM, std::string("hipMalloc(") + std::to_string(bytes) + "): " + hipGetErrorString(e));
    e = hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpy H2D");
    return VR_OK;
}

// One record per inserted voxel: (region index, local key) sort key.
struct Rec {
    uint64_t k;       // region << 32 | key
    uint32_t val;
    uint32_t idx;     // insertion order (later wins)
};

int build_scene_host(int device, vr_store store, const int32_t* xyz, const uint32_t* rgb, size_t n, vr_scene** out) {
    if (!out) return fail(VR_E_INVALID, "out is NULL");
    *out = nullptr;
    if (store != VR_STORE_VCS && store != VR_STORE_HASHTABLE) return fail(VR_E_INVALID, "unknown store");
    if (n && (!xyz || !rgb)) return fail(VR_E_INVALID, "xyz/rgb NULL");
    if (n >= 0xFFFFFFFFull) return fail(VR_E_INVALID, "too many voxels");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(VR_E_HIP, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(VR_E_INVALID, "device index out of range");

    // VoxelSceneCPU::insertVoxel (VoxelSceneCPU.cuh:16-46)
    std::vector<int32_t> rc(3 * n);
    int32_t minc = 0, maxc = 0;
    for (size_t i = 0; i < n; ++i) {
        if (rgb[i] > 0xFFFFFFu)
            return fail(VR_E_INVALID, "voxel colour " + std::to_string(rgb[i]) + " at index " + std::to_string(i) +
                                          " exceeds 24-bit RGB");
        for (int a = 0; a < 3; ++a) {
            int32_t c = f2i(std::floor((float)xyz[3 * i + a] / 64.0f));   // :19-21
            rc[3 * i + a] = c;
            minc = std::min(minc, c);
            maxc = std::max(maxc, c);
        }
    }
    const int64_t D64 = (int64_t)maxc - (int64_t)minc + 1;
    if (D64 > 1024) return fail(VR_E_INVALID, "scene spans more than 1024 regions per axis");
    const uint32_t D = (uint32_t)D64;
    const uint64_t D3 = (uint64_t)D * D * D;

    std::vector<Rec> recs(n);
    for (size_t i = 0; i < n; ++i) {
        uint32_t l[3];
        for (int a = 0; a < 3; ++a) {
            int32_t c = xyz[3 * i + a];
            l[a] = (uint32_t)(((c % vr::kBlock) + vr::kBlock) % vr::kBlock);    // :24-26
        }
        uint64_t ax = (uint64_t)(rc[3 * i] - minc), ay = (uint64_t)(rc[3 * i + 1] - minc),
                 az = (uint64_t)(rc[3 * i + 2] - minc);
        uint64_t region = ax + ay * D + az * (uint64_t)D * D;
        uint32_t key = (l[0] << 20) | (l[1] << 10) | l[2];                     // generate3DPoint
        recs[i] = Rec{(region << 32) | key, rgb[i], (uint32_t)i};
    }
    std::vector<int32_t>().swap(rc);
    std::sort(recs.begin(), recs.end(), [](const Rec& a, const Rec& b) { return a.k < b.k || (a.k == b.k && a.idx < b.idx); });
    size_t m = 0;   // duplicates: the later insertion wins (map assignment, :46)
    for (size_t i = 0; i < n; ++i) {
        if (m && recs[m - 1].k == recs[i].k) recs[m - 1] = recs[i];
        else recs[m++] = recs[i];
    }
    recs.resize(m);

    std::vector<uint32_t> region_slot(D3, vr::kNone);
    std::vector<size_t> region_begin;
    for (size_t i = 0; i < m; ++i)
        if (i == 0 || (recs[i].k >> 32) != (recs[i - 1].k >> 32)) {
            region_slot[recs[i].k >> 32] = (uint32_t)region_begin.size();
            region_begin.push_back(i);
        }
    const uint32_t nr = (uint32_t)region_begin.size();
    region_begin.push_back(m);
    if (store == VR_STORE_VCS && nr > vr::kVcsMaxRegions)     // (cuckoo scenes have no region bound)
        return fail(VR_E_INVALID, "VCS scene with " + std::to_string(nr) + " occupied 64^3 regions (at most " +
                                      std::to_string(vr::kVcsMaxRegions) + ")");

    vr_scene* s = new vr_scene();
    s->device = device; s->store = store; s->D = D; s->min_coord = minc; s->n_regions = nr; s->n_voxels = m;
    DeviceGuard dg(device);
    int rc_up = upload(s->region_slot, region_slot.data(), region_slot.size() * 4);
    if (rc_up) { free_scene(s); return rc_up; }

    if (store == VR_STORE_VCS) {
        // VoxelClusterStore ctor (VoxelClusterStore.cuh:37-85): per region 512
        // cluster slots; a cluster's sorted keys become a 512-bit occupancy
        // mask over in-cluster indices (same order) with a running value index
        // per 32-bit word, its values follow in key order (vr_internal.h "VCS").
        if ((uint64_t)nr * 512u * 16u * sizeof(uint2) > (1ull << 40)) { free_scene(s); return fail(VR_E_BUILD, "VCS mask table too large"); }
        std::vector<uint2> mask((size_t)nr * 512 * 16, uint2{0u, vr::kNone});
        std::vector<uint32_t> vals;
        vals.reserve(m);
        for (uint32_t r = 0; r < nr; ++r) {
            size_t b = region_begin[r], e = region_begin[r + 1];
            uint32_t bits[512][16];
            uint32_t cnt[512] = {0};
            memset(bits, 0, sizeof bits);
            for (size_t i = b; i < e; ++i) {
                uint32_t key = (uint32_t)recs[i].k;
                uint32_t x = key >> 20, y = (key >> 10) & 0x3FFu, z = key & 0x3FFu;
                uint32_t c = ((x / 8u) << 6) | ((y / 8u) << 3) | (z / 8u);
                uint32_t q = ((x & 7u) << 6) | ((y & 7u) << 3) | (z & 7u);
                bits[c][q >> 5] |= 1u << (q & 31u);
                cnt[c]++;
            }
            // values: cluster by cluster, each in key order (keys arrive ascending
            // within a region, and one cluster's keys ascend with q)
            uint32_t start[512];
            uint32_t acc = (uint32_t)vals.size();
            for (uint32_t c = 0; c < 512; ++c) { start[c] = acc; acc += cnt[c]; }
            vals.resize(acc);
            uint32_t fill[512] = {0};
            for (size_t i = b; i < e; ++i) {
                uint32_t key = (uint32_t)recs[i].k;
                uint32_t x = key >> 20, y = (key >> 10) & 0x3FFu, z = key & 0x3FFu;
                uint32_t c = ((x / 8u) << 6) | ((y / 8u) << 3) | (z / 8u);
                vals[start[c] + fill[c]++] = recs[i].val;
            }
            for (uint32_t c = 0; c < 512; ++c) {
                if (!cnt[c]) continue;
                // slot order z3..5 | y3..5 | x3..5 (vr_device.h word_index)
                const uint32_t slot = (c >> 6) | (((c >> 3) & 7u) << 3) | ((c & 7u) << 6);
                uint2* w = &mask[((size_t)r * 512 + slot) * 16];
                uint32_t run = start[c];
                for (uint32_t j = 0; j < 16; ++j) {
                    w[j] = uint2{bits[c][j], run};
                    run += (uint32_t)__builtin_popcount(bits[c][j]);
                }
            }
        }
        if (mask.empty()) mask.assign(16, uint2{0u, vr::kNone});
        if (vals.empty()) vals.assign(1, 0u);
        if ((rc_up = upload(s->vcs_mask, mask.data(), mask.size() * sizeof(uint2))) ||
            (rc_up = upload(s->vcs_vals, vals.data(), vals.size() * 4))) {
            free_scene(s);
            return rc_up;
        }
    } else {
        // CuckooHashTable ctor (CuckooHashTable.cuh:20-49) per region.
        std::vector<uint32_t> meta((size_t)nr * 4);
        std::vector<uint32_t> slots;
        std::vector<uint32_t> keys, vals;
        for (uint32_t r = 0; r < nr; ++r) {
            size_t b = region_begin[r], e = region_begin[r + 1];
            keys.resize(e - b); vals.resize(e - b);
            for (size_t i = b; i < e; ++i) { keys[i - b] = (uint32_t)recs[i].k; vals[i - b] = recs[i].val; }
            size_t base_words = slots.size();
            uint32_t M = 0, prime = 0, offset = 0;
            if (!cuckoo_build(keys.data(), vals.data(), (uint32_t)(e - b), &M, &prime, &offset, slots, base_words)) {
                free_scene(s);
                return fail(VR_E_BUILD, "cuckoo hash table build failed for region " + std::to_string(r));
            }
            if (base_words / 2 >= 0xFFFFFFFFull) { free_scene(s); return fail(VR_E_BUILD, "hash slots exceed 32-bit offsets"); }
            meta[4 * r + 0] = (uint32_t)(base_words / 2);
            meta[4 * r + 1] = M;
            meta[4 * r + 2] = prime;
            meta[4 * r + 3] = offset;
        }
        if (slots.empty()) slots.assign(2, vr::kEmpty);
        if (meta.empty()) meta.assign(4, 0);
        if ((rc_up = upload(s->ht_meta, meta.data(), meta.size() * 4)) ||
            (rc_up = upload(s->ht_slots, slots.data(), slots.size() * 4))) {
            free_scene(s);
            return rc_up;
        }
    }
    *out = s;
    return VR_OK;
}

// Device build (vr_build.hip) from host or device voxel arrays.
int build_scene_device(int device, vr_store store, const int32_t* xyz, const uint32_t* rgb, size_t n, bool on_device,
                       hipStream_t stream, vr_scene** out) {
    DeviceGuard dg(device);
    const int32_t* dxyz = xyz;
    const uint32_t* drgb = rgb;
    void *tx = nullptr, *tc = nullptr;
    auto release = [&]() {
        if (tx) (void)hipFree(tx);
        if (tc) (void)hipFree(tc);
    };
    if (!on_device && n) {
        hipError_t e = hipMalloc(&tx, 3 * n * sizeof(int32_t));
        if (e == hipSuccess) e = hipMalloc(&tc, n * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMemcpyAsync(tx, xyz, 3 * n * sizeof(int32_t), hipMemcpyHostToDevice, stream);
        if (e == hipSuccess) e = hipMemcpyAsync(tc, rgb, n * sizeof(uint32_t), hipMemcpyHostToDevice, stream);
        if (e != hipSuccess) { release(); return hip_fail(e, "voxel upload"); }
        dxyz = (const int32_t*)tx;
        drgb = (const uint32_t*)tc;
    }
    vr::GpuScene g;
    std::string err;
    const int rc = vr::build_scene_gpu((int)store, dxyz, drgb, n, stream, g, err);
    release();
    vr_scene* s = new vr_scene();
    s->device = device; s->store = store; s->D = g.D; s->min_coord = g.min_coord;
    s->n_regions = g.n_regions; s->n_voxels = g.n_voxels;
    s->region_slot = DevBuf{g.region_slot, g.region_slot_bytes};
    s->vcs_mask = DevBuf{g.vcs_mask, g.vcs_mask_bytes};
    s->vcs_vals = DevBuf{g.vcs_vals, g.vcs_vals_bytes};
    s->ht_meta = DevBuf{g.ht_meta, g.ht_meta_bytes};
    s->ht_slots = DevBuf{g.ht_slots, g.ht_slots_bytes};
    if (rc) {
        free_scene(s);
        return fail(rc == -1 ? VR_E_INVALID : rc == -5 ? VR_E_BUILD : VR_E_HIP, "scene build: " + err);
    }
    *out = s;
    return VR_OK;
}

// The derived per-region key-presence bits of a cuckoo scene (vr_internal.h KScene::ht_filter),
// made on the device from the tables either builder wrote.
int add_hash_filter(vr_scene* s, hipStream_t stream) {
    DeviceGuard dg(s->device);
    const uint32_t nr = std::max(1u, s->n_regions);
    const size_t bytes = (size_t)nr * vr::kHashFilterWords * sizeof(uint32_t);
    hipError_t e = hipMalloc(&s->ht_filter.p, bytes);
    if (e != hipSuccess) {
        s->ht_filter.p = nullptr;
        return hip_fail(e, "hipMalloc(hash filter)");
    }
    s->ht_filter.bytes = bytes;
    e = hipMemsetAsync(s->ht_filter.p, 0, bytes, stream);
    if (e == hipSuccess && s->n_regions)
        e = vr::launch_hash_filter((const uint4*)s->ht_meta.p, (const uint2*)s->ht_slots.p, s->n_regions,
                                   (uint32_t*)s->ht_filter.p, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hip_fail(e, "hash filter");
    return VR_OK;
}

// The derived per-region cluster-existence bits of a VCS scene (vr_internal.h KScene),
// made on the device from the mask records either builder wrote.
int add_cluster_bits(vr_scene* s, hipStream_t stream) {
    if (s->store != VR_STORE_VCS) return add_hash_filter(s, stream);
    DeviceGuard dg(s->device);
    const uint32_t nr = std::max(1u, s->n_regions);
    const size_t bytes = (size_t)nr * 16u * sizeof(uint32_t);
    hipError_t e = hipMalloc(&s->vcs_cbits.p, bytes);
    if (e != hipSuccess) {
        s->vcs_cbits.p = nullptr;
        return hip_fail(e, "hipMalloc(cluster bits)");
    }
    s->vcs_cbits.bytes = bytes;
    e = hipMemsetAsync(s->vcs_cbits.p, 0, bytes, stream);
    if (e == hipSuccess && s->n_regions)
        e = vr::launch_cluster_bits((const uint2*)s->vcs_mask.p, s->n_regions, (uint32_t*)s->vcs_cbits.p, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hip_fail(e, "cluster bits");
    return VR_OK;
}

int build_scene_raw(int device, vr_store store, const int32_t* xyz, const uint32_t* rgb, size_t n, bool on_device,
                    vr_build mode, void* stream, vr_scene** out);

int build_scene(int device, vr_store store, const int32_t* xyz, const uint32_t* rgb, size_t n, bool on_device,
                vr_build mode, void* stream, vr_scene** out) {
    int rc = build_scene_raw(device, store, xyz, rgb, n, on_device, mode, stream, out);
    if (rc) return rc;
    rc = add_cluster_bits(*out, (hipStream_t)stream);
    if (rc) {
        DeviceGuard dg((*out)->device);
        free_scene(*out);
        *out = nullptr;
    }
    return rc;
}

int build_scene_raw(int device, vr_store store, const int32_t* xyz, const uint32_t* rgb, size_t n, bool on_device,
                    vr_build mode, void* stream, vr_scene** out) {
    if (!out) return fail(VR_E_INVALID, "out is NULL");
    *out = nullptr;
    if (store != VR_STORE_VCS && store != VR_STORE_HASHTABLE) return fail(VR_E_INVALID, "unknown store");
    if (n && (!xyz || !rgb)) return fail(VR_E_INVALID, "xyz/rgb NULL");
    if (n >= 0xFFFFFFFFull) return fail(VR_E_INVALID, "too many voxels");
    if (mode != VR_BUILD_AUTO && mode != VR_BUILD_DEVICE && mode != VR_BUILD_HOST) return fail(VR_E_INVALID, "unknown build mode");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(VR_E_HIP, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(VR_E_INVALID, "device index out of range");
    if (mode == VR_BUILD_HOST) {
        if (!on_device) return build_scene_host(device, store, xyz, rgb, n, out);
        DeviceGuard dg(device);
        std::vector<int32_t> hx(3 * n + 3);
        std::vector<uint32_t> hc(n + 1);
        if (n) {
            hipError_t e = hipMemcpy(hx.data(), xyz, 3 * n * sizeof(int32_t), hipMemcpyDeviceToHost);
            if (e == hipSuccess) e = hipMemcpy(hc.data(), rgb, n * sizeof(uint32_t), hipMemcpyDeviceToHost);
            if (e != hipSuccess) return hip_fail(e, "voxel download");
        }
        return build_scene_host(device, store, hx.data(), hc.data(), n, out);
    }
    return build_scene_device(device, store, xyz, rgb, n, on_device, (hipStream_t)stream, out);
}

vr::KScene kscene(const vr_scene* s) {
    vr::KScene k{};
    k.region_slot = (const uint32_t*)s->region_slot.p;
    k.vcs_mask = (const uint2*)s->vcs_mask.p;
    k.vcs_vals = (const uint32_t*)s->vcs_vals.p;
    k.vcs_cbits = (const uint32_t*)s->vcs_cbits.p;
    k.ht_meta = (const uint4*)s->ht_meta.p;
    k.ht_slots = (const uint2*)s->ht_slots.p;
    k.ht_filter = (const uint32_t*)s->ht_filter.p;
    k.D = s->D;
    k.min_coord = s->min_coord;
    k.n_regions = s->n_regions;
    return k;
}

int make_view(const vr_scene* s, const vr_camera* cam, const vr_lighting* lit, const float translation[3],
              uint32_t scale, uint32_t width, uint32_t height, vr::KView& v) {
    if (!s) return fail(VR_E_INVALID, "scene is NULL");
    if (!cam || !lit) return fail(VR_E_INVALID, "camera/lighting NULL");
    if (width == 0 || height == 0 || width > 65536 || height > 65536) return fail(VR_E_INVALID, "bad image size");
    memset(&v, 0, sizeof v);
    for (int i = 0; i < 3; ++i) {
        v.llc[i] = cam->lower_left[i]; v.hor[i] = cam->horizontal[i]; v.ver[i] = cam->vertical[i];
        v.org[i] = cam->origin[i];
        v.L[i] = lit->light_dir[i]; v.LC[i] = lit->light_color[i]; v.LP[i] = lit->light_pos[i];
        v.translation[i] = translation ? translation[i] : 0.0f;
    }
    v.L_fast = 1u;
    for (int i = 0; i < 3; ++i) {
        const float a = std::fabs(v.L[i]);
        v.Lr[i] = 1.0f / v.L[i];
        if (!(a >= 0x1p-64f && a <= 0x1p+20f)) v.L_fast = 0u;
    }
    {
        // the light's longest-axis frame, in the device's fp32 order (-ffp-contract=off)
        const float ax = std::fabs(v.L[0]), ay = std::fabs(v.L[1]), az = std::fabs(v.L[2]);
        const uint32_t order =
            (ax > ay && ax > az) ? (ay > az ? 0u : 1u) : (ay > az ? (ax > az ? 2u : 3u) : (ax > ay ? 4u : 5u));
        const float k = 1.0f / (order < 2u ? ax : (order < 4u ? ay : az));
        uint32_t cls = 0;
        bool unit = order == 5u && ax == ay && ay == az;
        for (int i = 0; i < 3; ++i) {
            v.Lw[i] = k * v.L[i];
            cls |= (uint32_t)(v.Lw[i] > 0.0f) << (2 * i) | (uint32_t)(v.Lw[i] < 0.0f) << (2 * i + 1);
            unit = unit && std::fabs(v.Lw[i]) == 1.0f;
        }
        v.L_order = order;
        v.L_cls = cls;
        v.L_unit = unit ? 1u : 0u;
        v.L_eq = (v.L[0] == v.L[1] && v.L[1] == v.L[2]) ? 1u : 0u;
    }
    v.scale_f = (float)scale;          // static_cast<float>(scale) (Ray.cuh:16)
    v.use_point_light = lit->use_point_light ? 1 : 0;
    v.use_shadows = lit->use_shadows ? 1 : 0;
    v.W = width;
    v.H = height;
    v.LW = width;
    return VR_OK;
}

// Per-device ring of device scratch slots that a launch borrows: the deferral
// list of the crawl pass (vr::kDeferWords uint32, zeroed once; the crawl pass
// resets it at its end).  A slot belongs to ONE launch at a time: the launch
// that takes it waits (on its own stream, hipStreamWaitEvent) for the event
// the slot's previous launch recorded after its last kernel, and records the
// slot's event again after its own.  The device's lock is held from taking the
// slot to recording the event, so two launches in flight -- on any streams,
// from any threads -- never share a slot however many slots there are (a wait
// on an event of the same stream or one that has completed costs nothing).
// Launches on different devices take different locks.

struct SlotRing {
    const char* name;
    size_t words;          // uint32 per slot
    uint32_t nslots;
    struct Dev {
        std::mutex mu;
        uint32_t* base = nullptr;
        std::vector<hipEvent_t> ev;
        std::vector<bool> used;
        uint32_t next = 0;
        // host-mapped: [0] the last crawl pass's record count (any slot); then per slot the
        // {launch id, record count} its last crawl pass reported (two words, 8-B aligned)
        uint32_t* stat_host = nullptr;
        uint32_t* stat_dev = nullptr;
        uint32_t launch_serial = 0;
        // per slot: the tile pass's work order (heaviest tile groups first) made from the
        // costs of the slot's last launch that recorded them, for a grid of gx x gy
        struct Order {
            uint32_t* cost = nullptr;      // kWavesPerTileGroup words per tile group
            uint32_t* order = nullptr;     // one word per tile group
            uint32_t cap = 0, gx = 0, gy = 0, age = 0;
            uint64_t key = 0;              // the view it was learned on (view_key)
            bool valid = false;
            // the lane order (vr_march.hip lane_pixel): per 16x16 block its pixels heaviest
            // first, for a grid of lgx x lgy, learned on view lkey
            uint8_t* perm = nullptr;       // vr::perm_bytes(lgx, lgy)
            size_t bcap = 0;
            uint32_t lgx = 0, lgy = 0, lage = 0;
            uint64_t lkey = 0;
            bool lvalid = false;
            bool relaned = false;          // the lane order changed after the work order's costs
            // the crawl pass: the slot's last launch that ran one (id, view), and whether a
            // completed one reported that this view defers nothing
            uint32_t cid = 0;
            uint64_t ckey = 0;
            bool czero = false;
        };
        std::vector<Order> ord;
        bool any = false;                  // the device's previous launch: its stream and slot
        hipStream_t last_stream = nullptr;
        uint32_t last_idx = 0;
        uint64_t last_key = 0;             // the view of the device's previous launch
        bool force_skip = false;           // vr_debug_skip_next_crawl (tests)
    } dev[64];
    SlotRing(const char* n, size_t w, uint32_t s) : name(n), words(w), nslots(s) {}
};
SlotRing g_defer_ring("defer ring", vr::kDeferWords, 16);

// First use of a device: the slots and their events.  On a
// failure everything made so far is released and the next launch tries again.
int ring_init(SlotRing& r, SlotRing::Dev& D) {
    void* q = nullptr;
    const size_t bytes = (size_t)r.nslots * r.words * sizeof(uint32_t);
    std::vector<hipEvent_t> made;
    auto undo = [&](hipError_t e, const char* what) {
        for (hipEvent_t x : made) (void)hipEventDestroy(x);
        if (q) (void)hipFree(q);
        return hip_fail(e, what);
    };
    hipError_t e = hipMalloc(&q, bytes);
    if (e != hipSuccess) { q = nullptr; return undo(e, "hipMalloc(slot ring)"); }
    e = hipMemset(q, 0, bytes);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) return undo(e, "hipMemset(slot ring)");
    std::vector<hipEvent_t> ev(r.nslots);
    for (uint32_t i = 0; i < r.nslots; ++i) {
        e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
        if (e != hipSuccess) return undo(e, "hipEventCreate(slot ring)");
        made.push_back(ev[i]);
    }
    void* h = nullptr;
    void* hd = nullptr;
    const size_t stat_words = 2u + 2u * (size_t)r.nslots;
    e = hipHostMalloc(&h, sizeof(uint32_t) * stat_words, hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) {
        for (size_t i = 0; i < stat_words; ++i) ((volatile uint32_t*)h)[i] = 0u;
        e = hipHostGetDevicePointer(&hd, h, 0);
        if (e != hipSuccess) (void)hipHostFree(h);
    }
    if (e != hipSuccess) return undo(e, "hipHostMalloc(crawl statistics)");
    D.ev = std::move(ev);
    D.used.assign(r.nslots, false);
    D.ord.assign(r.nslots, SlotRing::Dev::Order{});
    D.stat_host = (uint32_t*)h;
    D.stat_dev = (uint32_t*)hd;
    D.base = (uint32_t*)q;
    return VR_OK;
}

// The borrowed slot; the device's lock is held until release() (or destruction).
struct SlotLease {
    SlotRing* ring = nullptr;
    std::unique_lock<std::mutex> lk;
    int dev = -1;
    uint32_t idx = 0;
    uint32_t* p = nullptr;
    int acquire(SlotRing& r, int d, hipStream_t stream) {
        if (d < 0 || d >= 64) return fail(VR_E_INVALID, "device index too large");
        SlotRing::Dev& D = r.dev[d];
        lk = std::unique_lock<std::mutex>(D.mu);
        if (!D.base) {
            int rc = ring_init(r, D);
            if (rc) return rc;
        }
        ring = &r;
        dev = d;
        idx = D.next;
        D.next = (D.next + 1u) % r.nslots;
        if (D.used[idx]) {
            hipError_t e = hipStreamWaitEvent(stream, D.ev[idx], 0);
            if (e != hipSuccess) return hip_fail(e, "hipStreamWaitEvent(slot ring)");
        }
        p = D.base + r.words * idx;
        return VR_OK;
    }
    SlotRing::Dev& D() const { return ring->dev[dev]; }
    // after the launch's last kernel on `stream`
    int release(hipStream_t stream) {
        hipError_t e = hipEventRecord(D().ev[idx], stream);
        if (e != hipSuccess) return hip_fail(e, "hipEventRecord(slot ring)");
        D().used[idx] = true;
        lk.unlock();
        return VR_OK;
    }
};

// Heaviest-first work order and lane order: made once per slot and view -- a
// view's walk lengths do not change (scenes are immutable), so they are not remade unless
// VR_ORDER_REFRESH=N (experiments) asks for a remake every N uses of a slot.  VR_ORDER=0 /
// VR_LANE_ORDER=0 turn them off.
uint32_t order_refresh() {
    static const uint32_t r = [] {
        const char* e = std::getenv("VR_ORDER_REFRESH");
        const long v = e ? std::strtol(e, nullptr, 10) : 0;
        return (uint32_t)(v >= 1 ? v : 0);
    }();
    return r;
}
bool refresh_due(uint32_t& age) { return order_refresh() != 0 && ++age >= order_refresh(); }
// VR_CRAWL_RPW (A/B runs): crawl records per wave for every launch instead of 4 / 8.
uint32_t crawl_rpw_override() {
    static const uint32_t r = [] {
        const char* e = std::getenv("VR_CRAWL_RPW");
        const long v = e ? std::strtol(e, nullptr, 10) : 0;
        return (uint32_t)(v >= 1 && v <= 64 ? v : 0);
    }();
    return r;
}
// VR_CRAWL_RPW_IN_FLIGHT (A/B runs): crawl records per wave with frames in flight (default 32:
// fewer crawl waves for the other frames' tile passes to share the CUs with.  C5 per frame in
// flight is bimodal from run to run -- 0.541-0.543 ms in some processes, 0.561-0.567 in others --
// and the fast mode showed up in 6 of 20 runs at 32 or more and in none of 22 at 8 or 16; never slower;
// profiles/r06/ab/ab_C5_crawl_rpw.txt).
uint32_t crawl_rpw_in_flight() {
    static const uint32_t r = [] {
        const char* e = std::getenv("VR_CRAWL_RPW_IN_FLIGHT");
        const long v = e ? std::strtol(e, nullptr, 10) : 0;
        return (uint32_t)(v >= 1 && v <= 64 ? v : 32);
    }();
    return r;
}
// VR_INFLIGHT_WAVES=0 (A/B runs): frames in flight keep the lone-frame occupancy.
bool in_flight_occupancy() {
    static const bool on = [] {
        const char* e = std::getenv("VR_INFLIGHT_WAVES");
        return !(e && e[0] == '0');
    }();
    return on;
}
// VR_LANE_ORDER=0 (A/B runs): 8x8 tiles, no per-pixel lane order.
bool lane_order_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("VR_LANE_ORDER");
        return !(e && e[0] == '0');
    }();
    return on;
}
// VR_INFLIGHT_HEAVY=1 (A/B runs): AUTO dispatches heaviest first with frames in flight too.
bool inflight_heavy() {
    static const bool on = [] {
        const char* e = std::getenv("VR_INFLIGHT_HEAVY");
        return e && e[0] == '1';
    }();
    return on;
}
// VR_CRAWL_SKIP=0 (A/B runs): every launch runs its crawl pass.
bool crawl_skip_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("VR_CRAWL_SKIP");
        return !(e && e[0] == '0');
    }();
    return on;
}
bool order_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("VR_ORDER");
        return !(e && e[0] == '0');
    }();
    return on;
}

// The view a launch renders, for the learned orders and the crawl-pass skip: an FNV-1a hash
// of the scene (its per-process serial), the algorithm and every value field of the view --
// the KView prefix above `out`: camera (llc, hor, ver, org), lights (L, LC, LP and the
// host-made Lr, L_fast, Lw, L_order, L_cls, L_unit, L_eq), transform (translation, scale_f),
// use_point_light, use_shadows, frame size (W, H), the launch's rows (row0, band_rows, rank,
// nranks, local_rows, row_limit, band_minv) and its tile deal (LW, tile_cols, tile_minv,
// col_R, col_rank, col_stride).  make_view zeroes the struct, so its padding is 0.  These,
// with the compile-time tile budget (vr::kTileBudget), are every input of which pixels the
// tile pass defers (vr_internal.h KView: a field added after `out` fails a static_assert
// until reviewed).  The per-launch buffers (out and after) are not part of it.
uint64_t view_key(const vr_scene* s, vr_algo algo, const vr::KView& v) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void* p, size_t n) {
        const unsigned char* b = (const unsigned char*)p;
        for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    };
    const uint32_t a = (uint32_t)algo;
    mix(&s->serial, sizeof s->serial);
    mix(&a, sizeof a);
    mix(&v, offsetof(vr::KView, out));
    return h;
}

// The crawl-pass skip's key: the view, plus the per-launch knobs that change how the crawl
// pass resumes deferred pixels (the list's capacity, walk-from-the-start records).  Which
// pixels defer is a function of the view alone: the tile pass's budget is compile-time
// (vr::kTileBudget) and everything else it reads is in the view (vr_internal.h KView).
uint64_t crawl_key(uint64_t key, const vr::KView& v) {
    const uint32_t knobs[2] = {v.defer_cap, v.crawl_rewalk};
    const unsigned char* b = (const unsigned char*)knobs;
    for (size_t i = 0; i < sizeof knobs; ++i) key = (key ^ b[i]) * 1099511628211ull;
    return key;
}

// VR_HOST_PROF (measurement builds only, profiles/build_variant.sh -- -DVR_HOST_PROF): host
// clock stamps at the stages of each launch, fetched with vr_host_prof_fetch.
#ifdef VR_HOST_PROF
}  // namespace
static uint64_t g_hp[4096][8];
static uint32_t g_hp_n = 0;
static inline uint64_t hp_now() { return (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count(); }
extern "C" int vr_host_prof_fetch(uint64_t* out, int n) {
    const uint32_t k = g_hp_n < 4096u ? g_hp_n : 4096u;
    const uint32_t m = (uint32_t)n < k ? (uint32_t)n : k;
    for (uint32_t i = 0; i < m; ++i)
        for (int j = 0; j < 8; ++j) out[8 * i + j] = g_hp[(g_hp_n - m + i) % 4096u][j];
    return (int)m;
}
namespace {
#define VR_HP(i) hp_row[i] = hp_now()
#else
#define VR_HP(i) do { } while (0)
#endif
int launch(const vr_scene* s, vr_algo algo, uint32_t kernel, uint32_t schedule, uint32_t occupancy, vr::KView& v,
           void* stream) {
#ifdef VR_HOST_PROF
    uint64_t* hp_row = g_hp[g_hp_n++ % 4096u];
    for (int j = 0; j < 8; ++j) hp_row[j] = 0;
#endif
    VR_HP(0);
    if (algo != VR_ALGO_ORIGINAL && algo != VR_ALGO_LONGESTAXIS) return fail(VR_E_INVALID, "unknown algorithm");
    if (kernel != VR_KERNEL_AUTO && kernel != VR_KERNEL_TILE && kernel != VR_KERNEL_TILE_REWALK)
        return fail(VR_E_INVALID, "unknown kernel (2, the persistent kernel, was retired)");
    if (occupancy > VR_OCCUPANCY_IN_FLIGHT) return fail(VR_E_INVALID, "unknown occupancy");
    if (v.local_rows == 0 || v.LW == 0) return VR_OK;
    DeviceGuard dg(s->device);
    const bool count = v.bytes != nullptr;
    const hipStream_t st = (hipStream_t)stream;
    // A launch is not capturable into a graph: the slot ring's event wait/record and the
    // work order's host-side bookkeeping would be baked into it and not replay (no test
    // captures one), so capture is refused before anything is enqueued.
    {
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        const hipError_t e = hipStreamIsCapturing(st, &cap);
        if (e != hipSuccess) return hip_fail(e, "hipStreamIsCapturing");
        if (cap != hipStreamCaptureStatusNone)
            return fail(VR_E_INVALID, "vr_render* cannot be captured into a HIP graph (stream is capturing)");
    }
    v.crawl_rewalk = kernel == VR_KERNEL_TILE_REWALK ? 1u : 0u;
    // the deferral list of the crawl pass (cluster-skip crawls, walks over the tile budget)
    SlotLease lease;
    int rc = lease.acquire(g_defer_ring, s->device, st);
    if (rc) return rc;
    VR_HP(1);
    // An error after the slot was taken: the slot's event is recorded again on `st` first (a
    // stream-ordered free of its old buffers may already be queued there), then the error.
    auto bail = [&](hipError_t e, const char* what) {
        (void)lease.release(st);
        return hip_fail(e, what);
    };
    v.defer = lease.p;
    v.defer_cap = (v.defer_cap && v.defer_cap < vr::kDeferCap) ? v.defer_cap : vr::kDeferCap;
    v.defer_stat = lease.D().stat_dev;
    const uint32_t expect = *(volatile uint32_t*)lease.D().stat_host;   // an earlier launch's count (a hint)
    // The work order: this slot's order if it was made for this view, made (from this
    // launch's costs, after its passes) when missing and the view repeats.  It only permutes
    // the tile groups: any order renders the same pixels.
    uint32_t gx = 0, gy = 0;
    vr::march_grid(v, gx, gy);
    const uint32_t n = gx * gy;
    SlotRing::Dev& D = lease.D();
    SlotRing::Dev::Order& O = D.ord[lease.idx];
    bool remake = false;
    // (the lock orders launches: "previous" is well defined)
    const bool alone = !D.any || D.last_stream == st || hipEventQuery(D.ev[D.last_idx]) == hipSuccess;
    VR_HP(2);
    const bool heavy = schedule == VR_SCHEDULE_HEAVIEST_FIRST ||
                       (schedule == VR_SCHEDULE_AUTO && (alone || inflight_heavy()));
    // crawl records per wave: a lone frame ends with the crawl pass's longest chain (2 per
    // wave since round 4's shorter chains: C5 alone 0.767 -> 0.759 ms vs 4,
    // profiles/r04/crawl/scene_lds_ab.txt, rpw_multi_cluster.txt); with frames in flight the
    // pass's issue cycles are what count (32 per wave since round 6; crawl_rpw_in_flight)
    v.crawl_rpw = crawl_rpw_override() ? crawl_rpw_override() : (alone ? 2u : crawl_rpw_in_flight());
    D.any = true;
    D.last_stream = st;
    D.last_idx = lease.idx;
    // Orders are learned per view: one made for another view (e.g. the previous rank of a
    // one-GPU rank emulation, or a moved camera) would deal the wrong pixels together.  A
    // view whose previous launch on the device was the same view gets its orders made (on
    // each slot's first such launch); a view that changes every launch never does, and
    // renders as a first render does.
    const uint64_t key = view_key(s, algo, v);
    const bool repeat = D.last_key == key;
    VR_HP(3);
    D.last_key = key;
    if (heavy && order_enabled() && n != 0) {
        if (n > O.cap) {
            // Grow, stream-ordered: the slot's previous launch -- the last user of the old
            // buffers -- is fenced on this stream (SlotLease::acquire), so freeing them on
            // it needs no host synchronisation.  Every path frees what it allocated.
            hipError_t e = hipSuccess;
            if (O.cost) e = hipFreeAsync(O.cost, st);
            if (O.order) {
                const hipError_t e2 = hipFreeAsync(O.order, st);
                if (e == hipSuccess) e = e2;
            }
            O.cost = nullptr;        // (the work order's fields only: the lane order's are its own)
            O.order = nullptr;
            O.cap = 0;
            O.valid = false;
            if (e == hipSuccess) e = hipMallocAsync((void**)&O.cost, sizeof(uint32_t) * vr::kWavesPerTileGroup * (size_t)n, st);
            if (e == hipSuccess) e = hipMallocAsync((void**)&O.order, sizeof(uint32_t) * (size_t)n, st);
            if (e != hipSuccess) {
                if (O.cost) (void)hipFreeAsync(O.cost, st);
                if (O.order) (void)hipFreeAsync(O.order, st);
                O.cost = nullptr;
                O.order = nullptr;
                return bail(e, "work order buffers");
            }
            O.cap = n;
        }
        const bool match = O.valid && O.gx == gx && O.gy == gy && O.key == key;
        v.order = match ? O.order : nullptr;
        // (a work order made from costs walked under another lane order is remade: the lane
        // order moves the heavy pixels of a block into one of its two tile groups)
        remake = match ? (O.relaned || refresh_due(O.age)) : repeat;
        v.cost = remake ? O.cost : nullptr;
    }
    // The lane order, kept like the work order but for every schedule: this slot's if it was
    // made for this view, made from this launch's per-pixel walk lengths when missing and the
    // view repeats.  It permutes pixels within 16x16 blocks only: any permutation renders the
    // same pixels.
    bool relane = false;
    uint32_t* pcost = nullptr;        // (a relaning launch's per-pixel walk lengths: transient)
    const size_t npx = (size_t)v.LW * v.local_rows, nperm = vr::perm_bytes(gx, gy);
    if (lane_order_enabled() && n != 0) {
        if (nperm > O.bcap) {
            hipError_t e = O.perm ? hipFreeAsync(O.perm, st) : hipSuccess;
            O.perm = nullptr;
            O.bcap = 0;
            O.lvalid = false;
            if (e == hipSuccess) e = hipMallocAsync((void**)&O.perm, nperm, st);
            if (e != hipSuccess) {
                O.perm = nullptr;
                return bail(e, "lane order buffer");
            }
            O.bcap = nperm;
        }
        const bool match = O.lvalid && O.lgx == gx && O.lgy == gy && O.lkey == key;
        v.perm = match ? O.perm : nullptr;
        relane = match ? refresh_due(O.lage) : repeat;
        if (relane) {
            // 4 B per pixel, only between this launch's tile pass and its perm_kernel (freed
            // stream-ordered after it): the slots keep 1 B per pixel each, not 5
            const hipError_t e = hipMallocAsync((void**)&pcost, sizeof(uint32_t) * npx, st);
            if (e != hipSuccess) return bail(e, "lane order walk lengths");
        }
        v.pcost = pcost;
    }
    // The crawl pass is skipped for a view this slot has seen defer nothing: whether a walk
    // is deferred is a pure function of its ray, so a view defers the same pixels on every
    // launch.  Every record carries its launch's id and a crawl pass shades only its own,
    // so even a wrong skip cannot put another frame's pixels into a frame; the records it
    // leaves raise the count the next crawl pass of the slot reports, which ends the skipping.
    // (C2 lone launch: the 4-us empty crawl pass and a kernel boundary.)
    //   The safety net: every tile pass that defers a pixel writes {launch id, 1}
    // into the slot's report word (vr_march.hip deferral_report), skipped launches included.
    // While the slot skips, nothing else writes that word (its last crawl pass left
    // {id, 0}), so a nonzero count there means a skipped launch deferred: the skipping ends,
    // and the slot's next launch runs the crawl pass, which drops the stale records (they
    // carry another launch's id) and resets the list.  What the net cannot repair is the
    // frames of the skipped launches that deferred before the host saw the report (their
    // deferred pixels stay 0): that needs a deferral that is not a function of the crawl key
    // below, which the kernels do not have (vr_internal.h KView, "end of the view's
    // identity"); tests/test_gpu_slots.py forces one (vr_debug_skip_next_crawl) to test the net.
    VR_HP(4);
    bool crawl = true;
    {
        uint32_t lid = ++D.launch_serial;
        if (lid == 0u) lid = ++D.launch_serial;
        v.launch_id = lid;
        const uint64_t ckey = crawl_key(key, v);
        const uint64_t r = *reinterpret_cast<volatile uint64_t*>(D.stat_host + 2 + 2 * (size_t)lease.idx);
        if (O.ckey != ckey) {
            O.czero = false;
        } else if (O.czero) {
            if ((uint32_t)(r >> 32) != 0u) O.czero = false;   // a skipped launch deferred
        } else if (O.cid != 0u) {
            O.czero = (uint32_t)r == O.cid && (uint32_t)(r >> 32) == 0u;
        }
        if (D.force_skip) {                    // (vr_debug_skip_next_crawl: tests of the net)
            D.force_skip = false;
            O.czero = true;
            O.ckey = ckey;
        }
        crawl = !(O.czero && crawl_skip_enabled());
        v.slot_stat = D.stat_dev + 2 + 2 * (size_t)lease.idx;
        if (crawl) {
            O.cid = lid;
            O.ckey = ckey;
        }
    }
    // crawl pass grid from the records an earlier launch deferred (a hint: any grid renders
    // the same pixels)
    VR_HP(5);
    const vr::KScene ks = kscene(s);
    const uint32_t cwgs = vr::crawl_grid(expect, v.crawl_rpw);
    // the tile pass's occupancy variant (vr_occupancy): AUTO = the in-flight one while another
    // stream's launch is running
    const bool hi = occupancy == VR_OCCUPANCY_IN_FLIGHT ||
                    (occupancy == VR_OCCUPANCY_AUTO && !alone && in_flight_occupancy());
    VR_HP(6);
    hipError_t e = vr::launch_march((int)s->store, (int)algo, count, ks, v, st, cwgs, hi, crawl);
    VR_HP(7);
    // The lane order first: when the slot has work-order buffers for this grid, perm_kernel
    // also writes the waves' costs under the new lane order and the work order is remade from
    // them at once -- an order made from costs walked under another lane order puts the light
    // half of a block first as often as the heavy one (C2 lone launch 0.125 -> 0.185 ms with
    // it, 0.116 without, profiles/r05/lane_order/).
    bool with_costs = false;
    if (e == hipSuccess && relane) {
        with_costs = order_enabled() && O.cost && O.cap >= n;
        e = vr::launch_perm(pcost, v.LW, v.local_rows, gx, gy, O.perm, with_costs ? O.cost : nullptr, st);
        O.lvalid = e == hipSuccess;
        O.relaned = !with_costs;
        O.lgx = gx;
        O.lgy = gy;
        O.lkey = key;
        O.lage = 0;
    }
    if (e == hipSuccess && (remake || with_costs)) {
        // (on a side stream instead -- one more stream than the box's 4 hardware queues
        // serialised the two render streams: C2 0.1124 -> 0.1277 ms per frame in flight,
        // profiles/r03/ab_order_C2_C3.txt)
        e = vr::launch_order(O.cost, n, gx, O.order, st);
        if (std::getenv("VR_ORDER_CHECK")) {
            std::vector<uint32_t> h(n), c(2 * (size_t)n);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(h.data(), O.order, 4 * (size_t)n, hipMemcpyDeviceToHost);
            (void)hipMemcpy(c.data(), O.cost, 8 * (size_t)n, hipMemcpyDeviceToHost);
            std::vector<int> seen(n, 0);
            int bad = 0;
            for (uint32_t i = 0; i < n; ++i) {
                const uint32_t t = (h[i] >> 16) * gx + (h[i] & 0xFFFFu);
                if ((h[i] & 0xFFFFu) >= gx || t >= n || seen[t]++) ++bad;
            }
            fprintf(stderr, "[order] slot %u grid %ux%u n %u bad %d first %08x %08x cost0 %u %u\n", lease.idx, gx, gy, n,
                    bad, h[0], n > 1 ? h[1] : 0u, c[0], c[1]);
        }
        O.valid = e == hipSuccess;
        O.gx = gx;
        O.gy = gy;
        O.key = key;
        O.age = 0;
        O.relaned = false;
    }
    if (pcost) {
        const hipError_t ef = hipFreeAsync(pcost, st);
        if (e == hipSuccess) e = ef;
    }
    // (on a failed launch the slot is still fenced: a kernel of it may be queued)
    rc = lease.release(st);
    if (e != hipSuccess) return hip_fail(e, "ray-march launch");
    return rc;
}

// ------------------------------------------------------------- synthetic grid
inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
inline bool draw(uint64_t seed, uint64_t stream, uint64_t k, double p) {
    uint64_t h = splitmix64((seed << 34) | (stream << 32) | k);
    return (double)(h >> 40) * (1.0 / 16777216.0) < p;
}

// std::stoi as used by VoxelFile.cuh:18-21: skip leading whitespace, optional
// sign, at least one digit, stop at the first non-digit; out of int range or
// no digits throws in the reference -> VR_E_PARSE here.
bool stoi_like(const char* b, const char* e, int32_t* out) {
    while (b < e && (*b == ' ' || *b == '\t' || *b == '\n' || *b == '\v' || *b == '\f' || *b == '\r')) ++b;
    bool neg = false;
    if (b < e && (*b == '+' || *b == '-')) { neg = *b == '-'; ++b; }
    if (b >= e || *b < '0' || *b > '9') return false;
    int64_t v = 0;
    while (b < e && *b >= '0' && *b <= '9') {
        v = v * 10 + (*b - '0');
        if (v > 2147483648ll) return false;
        ++b;
    }
    if (neg) v = -v;
    if (v > 2147483647ll || v < -2147483648ll) return false;
    *out = (int32_t)v;
    return true;
}

// Whole-file read (the .vox parser splits the text across threads).
int read_file(const char* path, std::vector<char>& out) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return fail(VR_E_IO, std::string("cannot open ") + path + ": " + std::strerror(errno));
    char buf[1 << 16];
    size_t got;
    while ((got = std::fread(buf, 1, sizeof buf, f)) > 0) out.insert(out.end(), buf, buf + got);
    const bool err = std::ferror(f) != 0;
    std::fclose(f);
    if (err) return fail(VR_E_IO, std::string("read failed: ") + path);
    return VR_OK;
}

// VoxelFile::readVoxelFile (VoxelFile.cuh:11-35) for one line: comma-separated
// fields with empty fields skipped (find_first_not_of(",")), lines with <= 3
// fields ignored, each of the first four fields converted like std::stoi.
// Returns 1 = voxel, 0 = ignored line, -1 = std::stoi would throw.
int parse_vox_line(const char* p, const char* e, int32_t v[4]) {
    const char* fb[4] = {nullptr, nullptr, nullptr, nullptr};
    const char* fe[4] = {nullptr, nullptr, nullptr, nullptr};
    int nf = 0;
    while (p < e) {
        while (p < e && *p == ',') ++p;
        if (p >= e) break;
        const char* q = p;
        while (q < e && *q != ',') ++q;
        if (nf < 4) { fb[nf] = p; fe[nf] = q; }
        ++nf;
        p = q;
    }
    if (nf <= 3) return 0;                     // lineEntries.size() > 3 (VoxelFile.cuh:25)
    for (int i = 0; i < 4; ++i)
        if (!stoi_like(fb[i], fe[i], &v[i])) return -1;
    return 1;
}

struct VoxParse {
    std::vector<int32_t> xyz;
    std::vector<uint32_t> rgb;
};

// The text is cut at newlines into one chunk per worker; chunks are parsed in
// parallel and concatenated in file order (later duplicates must stay later).
// The first error in file order is reported with its line number.
int parse_vox_text(const char* path, const std::vector<char>& text, VoxParse& out) {
    const size_t len = text.size();
    const char* base = text.data();
    unsigned hw = std::thread::hardware_concurrency();
    size_t workers = std::max<size_t>(1, std::min<size_t>({(size_t)(hw ? hw : 1), (size_t)16, len / (1u << 20) + 1}));
    std::vector<size_t> cut(workers + 1, len);
    cut[0] = 0;
    for (size_t w = 1; w < workers; ++w) {
        size_t c = std::max(cut[w - 1], len * w / workers);
        while (c < len && base[c - 1] != '\n') ++c;
        cut[w] = c;
    }
    struct Part {
        VoxParse vp;
        size_t lines = 0;            // newline-terminated or final lines seen
        size_t bad_line = 0;         // 1-based within the chunk, 0 = none
    };
    std::vector<Part> parts(workers);
    auto run = [&](size_t w) {
        Part& pt = parts[w];
        const char* p = base + cut[w];
        const char* end = base + cut[w + 1];
        pt.vp.xyz.reserve((size_t)(end - p) / 8 * 3);
        pt.vp.rgb.reserve((size_t)(end - p) / 24);
        while (p < end) {
            const char* q = (const char*)std::memchr(p, '\n', (size_t)(end - p));
            const char* le = q ? q : end;
            ++pt.lines;
            int32_t v[4];
            const int r = parse_vox_line(p, le, v);
            if (r < 0) { pt.bad_line = pt.lines; return; }
            if (r > 0) {
                pt.vp.xyz.insert(pt.vp.xyz.end(), {v[0], v[1], v[2]});
                pt.vp.rgb.push_back((uint32_t)v[3]);
            }
            p = q ? q + 1 : end;
        }
    };
    if (workers == 1) {
        run(0);
    } else {
        std::vector<std::thread> th;
        for (size_t w = 0; w < workers; ++w) th.emplace_back(run, w);
        for (auto& t : th) t.join();
    }
    size_t line0 = 0, n = 0;
    for (size_t w = 0; w < workers; ++w) {
        if (parts[w].bad_line) {
            // lines before this chunk: every earlier chunk ends with a newline
            return fail(VR_E_PARSE, std::string(path) + ":" + std::to_string(line0 + parts[w].bad_line) +
                                        ": std::stoi would throw");
        }
        line0 += parts[w].lines;
        n += parts[w].vp.rgb.size();
    }
    out.xyz.reserve(3 * n);
    out.rgb.reserve(n);
    for (auto& pt : parts) {
        out.xyz.insert(out.xyz.end(), pt.vp.xyz.begin(), pt.vp.xyz.end());
        out.rgb.insert(out.rgb.end(), pt.vp.rgb.begin(), pt.vp.rgb.end());
    }
    return VR_OK;
}

// .vxb: the binary scene sidecar -- 32-byte header {"VRVXB001", u64 count,
// u64 reserved x2}, then int32 xyz[3 * count] and uint32 rgb[count], little
// endian, in insertion order (duplicates resolve exactly as in the CSV).
constexpr char kVxbMagic[9] = "VRVXB001";
struct VxbHeader {
    char magic[8];
    uint64_t count = 0;
    uint64_t reserved[2] = {0, 0};
};
static_assert(sizeof(VxbHeader) == 32, "vxb header");

int read_vxb_header(FILE* f, const char* path, VxbHeader& hd) {
    if (std::fread(&hd, sizeof hd, 1, f) != 1 || std::memcmp(hd.magic, kVxbMagic, 8) != 0)
        return fail(VR_E_PARSE, std::string(path) + ": not a .vxb scene (bad header)");
    if (hd.count >= 0xFFFFFFFFull) return fail(VR_E_PARSE, std::string(path) + ": .vxb voxel count too large");
    return VR_OK;
}

bool is_vxb(const char* path) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    char m[8];
    const bool yes = std::fread(m, 1, 8, f) == 8 && std::memcmp(m, kVxbMagic, 8) == 0;
    std::fclose(f);
    return yes;
}

}  // namespace

namespace vr {
int set_error(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace vr

extern "C" {

const char* vr_last_error(void) { return g_err.c_str(); }
const char* vr_version(void) { return "voxelraymarcher_amd 0.1 (gfx950)"; }

int vr_camera_make(const float eye[3], const float look_at[3], const float up[3], float fov_deg, float aspect,
                   vr_camera* out) {
    if (!eye || !look_at || !up || !out) return fail(VR_E_INVALID, "NULL argument");
    const float PI = 3.141592f;                                 // MathConstants.cuh:3
    float half_h = std::tan((fov_deg * PI / 180.f) / 2.0f);     // Camera.cuh:13
    float half_w = half_h * aspect;
    f3 o{eye[0], eye[1], eye[2]};
    f3 w = unit(sub(f3{look_at[0], look_at[1], look_at[2]}, o));
    f3 u = unit(cross(w, f3{up[0], up[1], up[2]}));
    f3 v = cross(u, w);
    f3 llc = add(sub(sub(o, scl(half_w, u)), scl(half_h, v)), w);   // :19
    f3 hor = scl(2 * half_w, u), ver = scl(2 * half_h, v);
    const f3* src[5] = {&o, &llc, &hor, &ver, &w};
    float* dst[5] = {out->origin, out->lower_left, out->horizontal, out->vertical, out->forward};
    for (int i = 0; i < 5; ++i) { dst[i][0] = src[i]->x; dst[i][1] = src[i]->y; dst[i][2] = src[i]->z; }
    return VR_OK;
}

int vr_lighting_default(vr_lighting* out) {
    if (!out) return fail(VR_E_INVALID, "NULL argument");
    f3 L = unit(f3{1.0f, 1.0f, 1.0f});                          // Main.cu:28
    out->light_dir[0] = L.x; out->light_dir[1] = L.y; out->light_dir[2] = L.z;
    for (int i = 0; i < 3; ++i) out->light_color[i] = 1.0f;    // :31
    out->light_pos[0] = 10.0f; out->light_pos[1] = 10.0f; out->light_pos[2] = -10.0f;   // :34
    out->use_point_light = 0;                                   // :37
    out->use_shadows = 1;                                       // :40
    return VR_OK;
}

int vr_lighting_set_direction(vr_lighting* lit, const float dir[3]) {
    if (!lit || !dir) return fail(VR_E_INVALID, "NULL argument");
    f3 L = unit(f3{dir[0], dir[1], dir[2]});                     // Main.cu:28 makeUnitVector
    if (!std::isfinite(L.x) || !std::isfinite(L.y) || !std::isfinite(L.z))
        return fail(VR_E_INVALID, "light direction must be a finite non-zero vector");
    lit->light_dir[0] = L.x; lit->light_dir[1] = L.y; lit->light_dir[2] = L.z;
    return VR_OK;
}

int vr_scene_create(int device, vr_store store, const int32_t* xyz, const uint32_t* rgb, size_t n, vr_scene** out) {
    return build_scene(device, store, xyz, rgb, n, false, VR_BUILD_AUTO, nullptr, out);
}

int vr_scene_create_ex(int device, vr_store store, const int32_t* xyz, const uint32_t* rgb, size_t n, int inputs_on_device,
                       vr_build build, void* stream, vr_scene** out) {
    return build_scene(device, store, xyz, rgb, n, inputs_on_device != 0, build, stream, out);
}

int vr_scene_digest(const vr_scene* s, uint64_t out[5]) {
    if (!s || !out) return fail(VR_E_INVALID, "NULL argument");
    DeviceGuard dg(s->device);
    const DevBuf* bufs[5] = {&s->region_slot, &s->vcs_mask, &s->vcs_vals, &s->ht_meta, &s->ht_slots};
    for (int i = 0; i < 5; ++i) {
        uint64_t h = 1469598103934665603ull ^ bufs[i]->bytes;     // FNV-1a over the buffer bytes
        if (bufs[i]->p && bufs[i]->bytes) {
            std::vector<unsigned char> host(bufs[i]->bytes);
            hipError_t e = hipMemcpy(host.data(), bufs[i]->p, bufs[i]->bytes, hipMemcpyDeviceToHost);
            if (e != hipSuccess) return hip_fail(e, "hipMemcpy D2H");
            for (unsigned char c : host) h = (h ^ c) * 1099511628211ull;
        }
        out[i] = h;
    }
    return VR_OK;
}

int vr_scene_load_vox(int device, vr_store store, const char* path, vr_scene** out) {
    if (!path) return fail(VR_E_INVALID, "NULL argument");
    if (is_vxb(path)) {
        size_t n = 0;
        int rc = vr_vxb_read(path, nullptr, nullptr, 0, &n);
        if (rc) return rc;
        std::vector<int32_t> xyz(3 * n + 3);
        std::vector<uint32_t> rgb(n + 1);
        rc = vr_vxb_read(path, xyz.data(), rgb.data(), n, &n);
        if (rc) return rc;
        return build_scene(device, store, xyz.data(), rgb.data(), n, false, VR_BUILD_AUTO, nullptr, out);
    }
    std::vector<char> text;                 // CSV: read and parse once
    int rc = read_file(path, text);
    if (rc) return rc;
    VoxParse vp;
    rc = parse_vox_text(path, text, vp);
    if (rc) return rc;
    std::vector<char>().swap(text);
    return build_scene(device, store, vp.xyz.data(), vp.rgb.data(), vp.rgb.size(), false, VR_BUILD_AUTO, nullptr, out);
}

int vr_scene_get_info(const vr_scene* s, vr_scene_info* out) {
    if (!s || !out) return fail(VR_E_INVALID, "NULL argument");
    out->diameter = s->D;
    out->min_coord = s->min_coord;
    out->region_count = s->n_regions;
    out->store = (uint32_t)s->store;
    out->voxel_count = s->n_voxels;
    out->device_bytes = s->device_bytes();
    out->device = s->device;
    return VR_OK;
}

void vr_scene_destroy(vr_scene* s) {
    if (!s) return;
    DeviceGuard dg(s->device);
    free_scene(s);
}

int vr_render_ex(const vr_scene* s, vr_algo algo, const vr_camera* cam, const vr_lighting* lit,
                 const float translation[3], uint32_t scale, uint32_t width, uint32_t height,
                 const vr_render_opts* opts, uint32_t* out_dev, void* stream) {
    if (!opts) return fail(VR_E_INVALID, "opts is NULL");
    // Versioned struct (vr.h): a caller built before struct_size existed passes `kernel`
    // (0..3) in the first word and is refused; fields past the caller's struct read as 0.
    // (checked first: only the caller's own struct_size bytes are ever read)
    if (opts->struct_size < VR_RENDER_OPTS_MIN_SIZE)
        return fail(VR_E_INVALID, "vr_render_opts.struct_size is " + std::to_string(opts->struct_size) +
                                      ": set it to sizeof(vr_render_opts) (vr_render_opts_init); a struct built "
                                      "against the layout without struct_size is not accepted");
    vr_render_opts o{};
    std::memcpy(&o, opts, std::min<size_t>(opts->struct_size, sizeof o));
    if (o.reserved != 0u) return fail(VR_E_INVALID, "vr_render_opts.reserved must be 0");
    vr::KView v;
    int rc = make_view(s, cam, lit, translation, scale, width, height, v);
    if (rc) return rc;
    if (!out_dev) return fail(VR_E_INVALID, "out_dev is NULL");
    const uint32_t row_end = o.row_end == 0xFFFFFFFFu ? height : o.row_end;
    if (o.row_begin > row_end || row_end > height) return fail(VR_E_INVALID, "bad row range");
    if (!o.nranks || o.rank >= o.nranks) return fail(VR_E_INVALID, "bad band partition");
    if (o.reserved2 != 0u) return fail(VR_E_INVALID, "vr_render_opts.reserved2 must be 0");
    const uint32_t rows = row_end - o.row_begin;
    const uint32_t band = o.band_rows ? o.band_rows : std::max(1u, rows);
    v.row0 = o.row_begin;
    v.row_limit = row_end;
    v.band_rows = band;
    v.band_minv = band == 1u ? 0xFFFFFFFFu : (uint32_t)((1ull << 32) / band);
    if (o.tile_cols == 0u) {
        v.rank = o.rank;
        v.nranks = o.nranks;
        v.local_rows = (uint32_t)(vr_band_buffer_words(width, rows, band, o.nranks) / width);
    } else {
        // 2-D tile deal: every band is this rank's; its columns are dealt (KView)
        if (o.tile_cols > width) return fail(VR_E_INVALID, "tile_cols larger than the frame width");
        v.rank = 0;
        v.nranks = 1;
        v.local_rows = (uint32_t)(((uint64_t)rows + band - 1) / band * band);
        const uint32_t nblk = (width + o.tile_cols - 1) / o.tile_cols;
        v.LW = (nblk + o.nranks - 1) / o.nranks * o.tile_cols;
        v.tile_cols = o.tile_cols;
        v.tile_minv = o.tile_cols == 1u ? 0xFFFFFFFFu : (uint32_t)((1ull << 32) / o.tile_cols);
        v.col_R = o.nranks;
        v.col_rank = o.rank;
        v.col_stride = (o.deal_stride ? o.deal_stride : vr_deal_stride_default(o.nranks)) % o.nranks;
        if (v.local_rows > 65535u || v.LW > 65535u) return fail(VR_E_INVALID, "tile buffer too large");
    }
    v.out = out_dev;
    v.bytes = (unsigned long long*)o.bytes_dev;
    v.stats = o.bytes_dev ? (unsigned long long*)o.stats_dev : nullptr;
    v.defer_cap = o.defer_cap;
    if (o.schedule > VR_SCHEDULE_HEAVIEST_FIRST) return fail(VR_E_INVALID, "unknown schedule");
    return launch(s, algo, o.kernel, o.schedule, o.occupancy, v, stream);
}

int vr_render_opts_init(vr_render_opts* opts) {
    if (!opts) return fail(VR_E_INVALID, "NULL argument");
    *opts = vr_render_opts{};
    opts->struct_size = (uint32_t)sizeof(vr_render_opts);
    opts->kernel = VR_KERNEL_AUTO;
    opts->row_begin = 0;
    opts->row_end = 0xFFFFFFFFu;
    opts->band_rows = 0;
    opts->rank = 0;
    opts->nranks = 1;
    opts->schedule = VR_SCHEDULE_AUTO;
    return VR_OK;
}

namespace {
vr_render_opts opts_rows(uint32_t row_begin, uint32_t row_end) {
    vr_render_opts o;
    vr_render_opts_init(&o);
    o.row_begin = row_begin;
    o.row_end = row_end;
    return o;
}
}  // namespace

int vr_render(const vr_scene* s, vr_algo algo, const vr_camera* cam, const vr_lighting* lit, const float translation[3],
              uint32_t scale, uint32_t width, uint32_t height, uint32_t row_begin, uint32_t row_end, uint32_t* out_dev,
              void* stream) {
    const vr_render_opts o = opts_rows(row_begin, row_end);
    return vr_render_ex(s, algo, cam, lit, translation, scale, width, height, &o, out_dev, stream);
}

uint64_t vr_band_buffer_words(uint32_t width, uint32_t height, uint32_t band_rows, uint32_t nranks) {
    if (!band_rows || !nranks) return 0;
    uint64_t nb = (height + (uint64_t)band_rows - 1) / band_rows;
    uint64_t per = (nb + nranks - 1) / nranks;
    return per * band_rows * (uint64_t)width;
}

uint32_t vr_deal_stride_default(uint32_t nranks) {
    return (nranks % 3u == 0u) ? 1u : 3u;
}

int vr_forget_orders(int device) {
    if (device < 0 || device >= 64) return fail(VR_E_INVALID, "device index out of range");
    SlotRing::Dev& D = g_defer_ring.dev[device];
    std::lock_guard<std::mutex> lk(D.mu);
    for (SlotRing::Dev::Order& O : D.ord) {         // (buffers kept)
        O.valid = O.lvalid = O.relaned = O.czero = false;
        O.cid = 0;
    }
    D.last_key = 0;
    return VR_OK;
}

int vr_debug_skip_next_crawl(int device) {
    if (device < 0 || device >= 64) return fail(VR_E_INVALID, "device index out of range");
    SlotRing::Dev& D = g_defer_ring.dev[device];
    std::lock_guard<std::mutex> lk(D.mu);
    D.force_skip = true;
    return VR_OK;
}

uint64_t vr_tile_buffer_words(uint32_t width, uint32_t height, uint32_t band_rows, uint32_t tile_cols, uint32_t nranks) {
    if (!nranks || !tile_cols || !width || !height) return 0;
    const uint64_t band = band_rows ? band_rows : height;
    const uint64_t rows = (height + band - 1) / band * band;
    const uint64_t nblk = ((uint64_t)width + tile_cols - 1) / tile_cols;
    return rows * ((nblk + nranks - 1) / nranks * tile_cols);
}

int vr_render_tiles(const vr_scene* s, vr_algo algo, const vr_camera* cam, const vr_lighting* lit,
                    const float translation[3], uint32_t scale, uint32_t width, uint32_t height, uint32_t band_rows,
                    uint32_t tile_cols, uint32_t rank, uint32_t nranks, uint32_t* out_dev, void* stream) {
    if (!band_rows || !tile_cols) return fail(VR_E_INVALID, "band_rows and tile_cols must be > 0");
    vr_render_opts o = opts_rows(0, height);
    o.band_rows = band_rows;
    o.tile_cols = tile_cols;
    o.rank = rank;
    o.nranks = nranks;
    return vr_render_ex(s, algo, cam, lit, translation, scale, width, height, &o, out_dev, stream);
}

int vr_assemble_tiles(const void* parts_dev, void* frame_dev, uint32_t elem_bytes, uint32_t width, uint32_t height,
                      uint32_t band_rows, uint32_t tile_cols, uint32_t nranks, uint32_t deal_stride, void* stream) {
    if (!parts_dev || !frame_dev) return fail(VR_E_INVALID, "NULL device buffer");
    if (elem_bytes < 1u || elem_bytes > 4u) return fail(VR_E_INVALID, "elem_bytes must be 1..4");
    if (!width || !height || !band_rows || !tile_cols || !nranks || tile_cols > width)
        return fail(VR_E_INVALID, "bad tile layout");
    vr::TileLayout t{};
    t.W = width;
    t.H = height;
    t.band_rows = band_rows;
    t.tile_cols = tile_cols;
    t.R = nranks;
    t.stride = (deal_stride ? deal_stride : vr_deal_stride_default(nranks)) % nranks;
    t.LW = (uint32_t)(vr_tile_buffer_words(width, band_rows, band_rows, tile_cols, nranks) / band_rows);
    t.rank_words = vr_tile_buffer_words(width, height, band_rows, tile_cols, nranks);
    hipError_t e = vr::launch_assemble_tiles(parts_dev, frame_dev, elem_bytes, t, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "assemble_tiles launch");
    return VR_OK;
}

int vr_render_bands(const vr_scene* s, vr_algo algo, const vr_camera* cam, const vr_lighting* lit,
                    const float translation[3], uint32_t scale, uint32_t width, uint32_t height, uint32_t band_rows,
                    uint32_t rank, uint32_t nranks, uint32_t* out_dev, void* stream) {
    if (!band_rows) return fail(VR_E_INVALID, "band_rows must be > 0");
    vr_render_opts o = opts_rows(0, height);
    o.band_rows = band_rows;
    o.rank = rank;
    o.nranks = nranks;
    return vr_render_ex(s, algo, cam, lit, translation, scale, width, height, &o, out_dev, stream);
}

int vr_render_count(const vr_scene* s, vr_algo algo, const vr_camera* cam, const vr_lighting* lit,
                    const float translation[3], uint32_t scale, uint32_t width, uint32_t height, uint32_t row_begin,
                    uint32_t row_end, uint32_t* out_dev, uint64_t* bytes_dev, void* stream) {
    if (!bytes_dev) return fail(VR_E_INVALID, "bytes_dev is NULL");
    vr_render_opts o = opts_rows(row_begin, row_end);
    o.bytes_dev = bytes_dev;
    return vr_render_ex(s, algo, cam, lit, translation, scale, width, height, &o, out_dev, stream);
}

int vr_pack_rgb8(const uint32_t* words_dev, uint8_t* rgb_dev, uint64_t n_pixels, void* stream) {
    if (n_pixels && (!words_dev || !rgb_dev)) return fail(VR_E_INVALID, "NULL device buffer");
    hipError_t e = vr::launch_pack_rgb8(words_dev, rgb_dev, n_pixels, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "pack_rgb8 launch");
    return VR_OK;
}

int vr_synth_generate(const vr_synth_params* p, int32_t* xyz, uint32_t* rgb, size_t capacity, size_t* n_out) {
    if (!p || !n_out) return fail(VR_E_INVALID, "NULL argument");
    if (p->n == 0 || p->n % 64 || p->n > 1024) return fail(VR_E_INVALID, "grid side must be a multiple of 64 in [64,1024]");
    if (xyz && !rgb) return fail(VR_E_INVALID, "rgb NULL");
    const uint32_t NR = p->n / 64, NC = p->n / 8;
    size_t cnt = 0;
    for (uint32_t rz = 0; rz < NR; ++rz)
        for (uint32_t ry = 0; ry < NR; ++ry)
            for (uint32_t rx = 0; rx < NR; ++rx) {
                if (!draw(p->seed, 0, rx + ry * NR + rz * NR * NR, p->p_region)) continue;
                for (uint32_t cz = rz * 8; cz < rz * 8 + 8; ++cz)
                    for (uint32_t cy = ry * 8; cy < ry * 8 + 8; ++cy)
                        for (uint32_t cx = rx * 8; cx < rx * 8 + 8; ++cx) {
                            if (!draw(p->seed, 1, cx + cy * NC + (uint64_t)cz * NC * NC, p->p_cluster)) continue;
                            for (uint32_t z = cz * 8; z < cz * 8 + 8; ++z)
                                for (uint32_t y = cy * 8; y < cy * 8 + 8; ++y)
                                    for (uint32_t x = cx * 8; x < cx * 8 + 8; ++x) {
                                        uint64_t key = ((uint64_t)x << 20) | (y << 10) | z;
                                        if (!draw(p->seed, 2, key, p->p_voxel)) continue;
                                        if (xyz) {
                                            if (cnt >= capacity) return fail(VR_E_INVALID, "capacity too small");
                                            xyz[3 * cnt] = (int32_t)x; xyz[3 * cnt + 1] = (int32_t)y; xyz[3 * cnt + 2] = (int32_t)z;
                                            rgb[cnt] = (uint32_t)(splitmix64((p->seed << 34) | (3ull << 32) | key) & 0xFFFFFFu);
                                        }
                                        ++cnt;
                                    }
                        }
            }
    *n_out = cnt;
    return VR_OK;
}

int vr_vox_read(const char* path, int32_t* xyz, uint32_t* rgb, size_t capacity, size_t* n_out) {
    if (!path || !n_out) return fail(VR_E_INVALID, "NULL argument");
    std::vector<char> text;
    int rc = read_file(path, text);
    if (rc) return rc;
    VoxParse vp;
    rc = parse_vox_text(path, text, vp);
    if (rc) return rc;
    const size_t n = vp.rgb.size();
    if (xyz) {
        if (!rgb) return fail(VR_E_INVALID, "rgb NULL");
        if (n > capacity) return fail(VR_E_INVALID, "capacity too small");
        std::memcpy(xyz, vp.xyz.data(), 3 * n * sizeof(int32_t));
        std::memcpy(rgb, vp.rgb.data(), n * sizeof(uint32_t));
    }
    *n_out = n;
    return VR_OK;
}

int vr_vxb_read(const char* path, int32_t* xyz, uint32_t* rgb, size_t capacity, size_t* n_out) {
    if (!path || !n_out) return fail(VR_E_INVALID, "NULL argument");
    FILE* f = std::fopen(path, "rb");
    if (!f) return fail(VR_E_IO, std::string("cannot open ") + path + ": " + std::strerror(errno));
    VxbHeader hd;
    int rc = read_vxb_header(f, path, hd);
    if (rc) { std::fclose(f); return rc; }
    if (xyz) {
        if (!rgb) { std::fclose(f); return fail(VR_E_INVALID, "rgb NULL"); }
        if (hd.count > capacity) { std::fclose(f); return fail(VR_E_INVALID, "capacity too small"); }
        if (std::fread(xyz, sizeof(int32_t), 3 * (size_t)hd.count, f) != 3 * (size_t)hd.count ||
            std::fread(rgb, sizeof(uint32_t), (size_t)hd.count, f) != (size_t)hd.count) {
            std::fclose(f);
            return fail(VR_E_PARSE, std::string(path) + ": truncated .vxb payload");
        }
    }
    std::fclose(f);
    *n_out = (size_t)hd.count;
    return VR_OK;
}

int vr_vxb_write(const char* path, const int32_t* xyz, const uint32_t* rgb, size_t n) {
    if (!path || (n && (!xyz || !rgb))) return fail(VR_E_INVALID, "NULL argument");
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(VR_E_IO, std::string("cannot open ") + path + ": " + std::strerror(errno));
    VxbHeader hd;
    std::memcpy(hd.magic, kVxbMagic, 8);
    hd.count = n;
    bool ok = std::fwrite(&hd, sizeof hd, 1, f) == 1 &&
              (n == 0 || (std::fwrite(xyz, sizeof(int32_t), 3 * n, f) == 3 * n &&
                          std::fwrite(rgb, sizeof(uint32_t), n, f) == n));
    if (std::fclose(f) != 0) ok = false;
    if (!ok) return fail(VR_E_IO, std::string("write failed: ") + path);
    return VR_OK;
}

int vr_scene_file_read(const char* path, int32_t* xyz, uint32_t* rgb, size_t capacity, size_t* n_out) {
    if (!path) return fail(VR_E_INVALID, "NULL argument");
    return is_vxb(path) ? vr_vxb_read(path, xyz, rgb, capacity, n_out) : vr_vox_read(path, xyz, rgb, capacity, n_out);
}

int vr_vox_write(const char* path, const int32_t* xyz, const uint32_t* rgb, size_t n) {
    if (!path || (n && (!xyz || !rgb))) return fail(VR_E_INVALID, "NULL argument");
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(VR_E_IO, std::string("cannot open ") + path + ": " + std::strerror(errno));
    for (size_t i = 0; i < n; ++i)
        std::fprintf(f, "%d,%d,%d,%d\n", xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], (int32_t)rgb[i]);
    if (std::fclose(f) != 0) return fail(VR_E_IO, std::string("write failed: ") + path);
    return VR_OK;
}

}  // extern "C"
