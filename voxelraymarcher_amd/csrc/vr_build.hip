// vr_build.hip -- the scene build on the GPU:
// VoxelSceneCPU::insertVoxel / generateVoxelScene (VoxelSceneCPU.cuh:16-93),
// the VoxelClusterStore image (VoxelClusterStore.cuh:37-85) and the
// CuckooHashTable images (CuckooHashTable.cuh:20-49, 97-178), producing the
// same device layout as the host builder in vr_host.cpp (vr_internal.h):
//
//   1. region coordinates, the min/max coordinate (minCoord/maxCoord start at 0)
//      and the first colour above 24 bits                       (reduction)
//   2. one 64-bit sort key per voxel: region | (cluster, in-cluster index) for
//      the VCS, region | x<<20|y<<10|z for the hash table           (map)
//   3. stable radix sort of (key, insertion index)                  (rocPRIM)
//   4. keep the LAST insertion of each key (unordered_map assignment, :46)
//   5. region slots in region order; VCS: colours in (region, cluster, key)
//      order and one 16-word mask record per present cluster (a thread per
//      cluster); cuckoo: per region the host's sequential insertion with the
//      same seeded rehash (one lane per region), so every key lands in the
//      same table as in the host build -- which the lookup's algorithmic byte
//      count (key found in table 1 or 2) depends on.
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <string>
#include <vector>

#include "vr_build.h"
#include "vr_device.h"

namespace vr {
namespace {

constexpr uint32_t kThreads = 256;

__global__ void k_minmax(const int32_t* __restrict__ xyz, const uint32_t* __restrict__ rgb, uint64_t n,
                         int32_t* mm, unsigned long long* bad) {
    int32_t lo = 0, hi = 0;                       // minCoord / maxCoord start at 0 (VoxelSceneCPU.cuh)
    unsigned long long first_bad = ~0ull;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        for (int a = 0; a < 3; ++a) {
            const int32_t c = f2i(floorf((float)xyz[3 * i + a] / 64.0f));   // :19-21
            lo = min(lo, c);
            hi = max(hi, c);
        }
        if (rgb[i] > 0xFFFFFFu && i < first_bad) first_bad = i;
    }
    for (int off = 32; off > 0; off >>= 1) {
        lo = min(lo, __shfl_down(lo, off, 64));
        hi = max(hi, __shfl_down(hi, off, 64));
        first_bad = min(first_bad, __shfl_down(first_bad, off, 64));
    }
    if ((threadIdx.x & 63u) == 0) {
        atomicMin(&mm[0], lo);
        atomicMax(&mm[1], hi);
        if (first_bad != ~0ull) atomicMin(bad, first_bad);
    }
}

// Sort key of voxel i and its insertion index.
__global__ void k_keys(const int32_t* __restrict__ xyz, uint64_t n, int32_t minc, uint32_t D, int store,
                       uint64_t* __restrict__ key, uint32_t* __restrict__ idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t l[3];
    uint64_t region = 0, mul = 1;
    for (int a = 0; a < 3; ++a) {
        const int32_t c = xyz[3 * i + a];
        const int32_t rc = f2i(floorf((float)c / 64.0f));
        l[a] = (uint32_t)(((c % kBlock) + kBlock) % kBlock);                // :24-26
        region += (uint64_t)(uint32_t)(rc - minc) * mul;
        mul *= D;
    }
    uint64_t k;
    if (store == STORE_VCS) {
        const uint32_t cid = ((l[0] >> 3) << 6) | ((l[1] >> 3) << 3) | (l[2] >> 3);
        const uint32_t q = ((l[0] & 7u) << 6) | ((l[1] & 7u) << 3) | (l[2] & 7u);
        k = (region << 18) | ((uint64_t)cid << 9) | q;
    } else {
        k = (region << 26) | ((l[0] << 20) | (l[1] << 10) | l[2]);          // generate3DPoint
    }
    key[i] = k;
    idx[i] = (uint32_t)i;
}

// 1 where this sorted entry is the last of its key (the winning insertion).
__global__ void k_flag_last(const uint64_t* __restrict__ key, uint64_t n, uint32_t* __restrict__ f) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) f[i] = (i + 1 == n || key[i] != key[i + 1]) ? 1u : 0u;
}

// 1 where key >> shift differs from the previous entry's (first of a group).
__global__ void k_flag_first(const uint64_t* __restrict__ key, uint64_t n, uint32_t shift, uint32_t* __restrict__ f) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) f[i] = (i == 0 || (key[i] >> shift) != (key[i - 1] >> shift)) ? 1u : 0u;
}

__global__ void k_compact(const uint64_t* __restrict__ key, const uint32_t* __restrict__ idx, const uint32_t* __restrict__ f,
                          const uint32_t* __restrict__ pos, uint64_t n, uint64_t* __restrict__ ukey, uint32_t* __restrict__ uidx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && f[i]) {
        ukey[pos[i]] = key[i];
        uidx[pos[i]] = idx[i];
    }
}

// Group starts: start[pos[i]] = i where f[i].
__global__ void k_starts(const uint32_t* __restrict__ f, const uint32_t* __restrict__ pos, uint64_t n, uint32_t* __restrict__ start) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && f[i]) start[pos[i]] = (uint32_t)i;
}

__global__ void k_fill_u32(uint32_t* __restrict__ p, uint64_t n, uint32_t v) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) p[i] = v;
}

__global__ void k_fill_u2(uint2* __restrict__ p, uint64_t n, uint2 v) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) p[i] = v;
}

// region_slot[region] = slot, for the first voxel of each region.
__global__ void k_region_slots(const uint64_t* __restrict__ ukey, const uint32_t* __restrict__ rstart, uint32_t nr,
                               uint32_t shift, uint32_t* __restrict__ region_slot) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < nr) region_slot[ukey[rstart[r]] >> shift] = r;
}

__global__ void k_gather_vals(const uint32_t* __restrict__ rgb, const uint32_t* __restrict__ uidx, uint64_t m,
                              uint32_t* __restrict__ vals) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) vals[j] = rgb[uidx[j]];
}

// One thread per present cluster: its 16 mask words {occupancy bits, value
// index of the word's first voxel}, in the record of slot perm(cid) of its region.
__global__ void k_cluster_records(const uint64_t* __restrict__ ukey, const uint32_t* __restrict__ cstart, uint32_t nc,
                                  uint64_t m, const uint32_t* __restrict__ rslot_of, uint2* __restrict__ mask) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nc) return;
    const uint32_t b = cstart[c];
    const uint32_t e = c + 1 < nc ? cstart[c + 1] : (uint32_t)m;
    const uint32_t r = rslot_of[b];
    const uint32_t cid = (uint32_t)(ukey[b] >> 9) & 511u;
    const uint32_t slot = (cid >> 6) | (((cid >> 3) & 7u) << 3) | ((cid & 7u) << 6);
    uint2* rec = mask + ((size_t)r * 512 + slot) * 16;
    uint32_t j = b, run = b;
    for (uint32_t w = 0; w < 16; ++w) {
        uint32_t bits = 0;
        while (j < e && (((uint32_t)ukey[j] & 511u) >> 5) == w) {
            bits |= 1u << ((uint32_t)ukey[j] & 31u);
            ++j;
        }
        rec[w] = make_uint2(bits, run);
        run += (uint32_t)__popc(bits);
    }
}

// Region slot of every unique voxel: (inclusive scan of region starts) - 1.
__global__ void k_minus_one(uint32_t* __restrict__ p, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] -= 1u;
}

// Per region: n_r, M_r = (u32)(n_r * 1.25) (CuckooHashTable.cuh:23) and 2 M_r slots.
__global__ void k_region_sizes(const uint32_t* __restrict__ rstart, uint32_t nr, uint64_t m, uint32_t* __restrict__ M,
                               uint32_t* __restrict__ slots2) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nr) return;
    const uint32_t b = rstart[r], e = r + 1 < nr ? rstart[r + 1] : (uint32_t)m;
    const uint32_t Mr = (uint32_t)((double)(e - b) * 1.25);
    M[r] = Mr;
    slots2[r] = 2u * Mr;
}

__constant__ uint32_t c_primes[14] = {668265261u, 12289u, 24593u, 49157u, 98317u, 196613u, 393241u,
                                      786433u, 1572869u, 3145739u, 6291469u, 12582917u, 25165843u, 50331653u};

// One wave per region: lane 0 inserts the region's keys in sorted order with
// the host builder's algorithm (bucket alternation, 300 000-step eviction
// limit, seeded prime/offset rehash, at most 4096 attempts); the wave clears
// the tables before each attempt.
__global__ void k_cuckoo(const uint64_t* __restrict__ ukey, const uint32_t* __restrict__ uidx, const uint32_t* __restrict__ rgb,
                         const uint32_t* __restrict__ rstart, uint32_t nr, uint64_t m, const uint32_t* __restrict__ M,
                         const uint32_t* __restrict__ base2, uint2* __restrict__ slots, uint4* __restrict__ meta,
                         uint32_t* __restrict__ failed) {
    const uint32_t r = blockIdx.x;
    if (r >= nr) return;
    const uint32_t lane = threadIdx.x;
    const uint32_t b = rstart[r], e = r + 1 < nr ? rstart[r + 1] : (uint32_t)m, n = e - b;
    const uint32_t Mr = M[r];
    uint2* t = slots + base2[r];
    __shared__ uint32_t s_prime, s_offset, s_done;
    if (lane == 0) {
        s_prime = c_primes[0];
        s_offset = 0;
        s_done = 0;
    }
    __syncthreads();
    const uint32_t key0 = (uint32_t)ukey[b] & 0x3FFFFFFu;
    uint64_t rng = 0x9E3779B97F4A7C15ull ^ (uint64_t)n ^ ((uint64_t)key0 << 20);
    for (int attempt = 0; attempt < 4096; ++attempt) {
        for (uint32_t i = lane; i < 2u * Mr; i += blockDim.x) t[i] = make_uint2(kEmpty, 0u);
        __threadfence_block();
        __syncthreads();
        if (lane == 0) {
            const uint32_t prime = s_prime, offset = s_offset;
            bool rehash = false;
            for (uint32_t i = b; i < e && !rehash; ++i) {
                uint32_t code = (uint32_t)ukey[i] & 0x3FFFFFFu, value = rgb[uidx[i]], bucket = 0, it = 0;
                for (;;) {
                    if (it >= 300000u) { rehash = true; break; }
                    uint2* slot = bucket == 0 ? t + hash1(code, offset) % Mr : t + Mr + hash2(code, prime) % Mr;
                    const uint2 old = *slot;
                    *slot = make_uint2(code, value);
                    if (old.x == kEmpty) break;
                    code = old.x;
                    value = old.y;
                    bucket ^= 1u;
                    ++it;
                }
            }
            if (!rehash) {
                meta[r] = make_uint4(base2[r], Mr, prime, offset);
                s_done = 1;
            } else {
                rng = rng * 6364136223846793005ull + 1442695040888963407ull;
                s_prime = c_primes[(rng >> 33) % 14u];
                rng = rng * 6364136223846793005ull + 1442695040888963407ull;
                s_offset = (uint32_t)((rng >> 33) % 25u);
            }
        }
        __syncthreads();
        if (s_done) return;
    }
    if (lane == 0) atomicAdd(failed, 1u);
}

inline dim3 blocks_for(uint64_t n) { return dim3((unsigned)std::max<uint64_t>(1, (n + kThreads - 1) / kThreads)); }

struct Scratch {
    std::vector<void*> ptrs;
    ~Scratch() { for (void* p : ptrs) (void)hipFree(p); }
    template <class T>
    hipError_t alloc(T** p, uint64_t count) {
        void* q = nullptr;
        hipError_t e = hipMalloc(&q, std::max<uint64_t>(count, 1) * sizeof(T));
        if (e == hipSuccess) { ptrs.push_back(q); *p = (T*)q; }
        return e;
    }
};

#define BUILD_CHECK(expr)                                                                   \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) {                                                             \
            err = std::string(#expr) + ": " + hipGetErrorString(e_);                        \
            return -2;                                                                      \
        }                                                                                   \
    } while (0)

template <class T>
int scan(bool inclusive, const T* in, T* out, uint64_t n, hipStream_t stream, std::string& err) {
    size_t bytes = 0;
    void* tmp = nullptr;
    if (inclusive) BUILD_CHECK(rocprim::inclusive_scan(nullptr, bytes, in, out, (size_t)n, rocprim::plus<T>(), stream));
    else BUILD_CHECK(rocprim::exclusive_scan(nullptr, bytes, in, out, T(0), (size_t)n, rocprim::plus<T>(), stream));
    BUILD_CHECK(hipMalloc(&tmp, std::max<size_t>(bytes, 1)));
    hipError_t e = inclusive ? rocprim::inclusive_scan(tmp, bytes, in, out, (size_t)n, rocprim::plus<T>(), stream)
                             : rocprim::exclusive_scan(tmp, bytes, in, out, T(0), (size_t)n, rocprim::plus<T>(), stream);
    (void)hipStreamSynchronize(stream);
    (void)hipFree(tmp);
    BUILD_CHECK(e);
    return 0;
}

template <class T>
T read_back(const T* p, hipStream_t stream) {
    T v{};
    (void)hipMemcpyAsync(&v, p, sizeof(T), hipMemcpyDeviceToHost, stream);
    (void)hipStreamSynchronize(stream);
    return v;
}

}  // namespace

int build_scene_gpu(int store, const int32_t* xyz, const uint32_t* rgb, uint64_t n, hipStream_t stream,
                    GpuScene& out, std::string& err) {
    out = GpuScene{};
    Scratch s;
    // 1. min / max region coordinate, first colour above 24 bits
    int32_t* mm;
    unsigned long long* bad;
    BUILD_CHECK(s.alloc(&mm, 2));
    BUILD_CHECK(s.alloc(&bad, 1));
    const int32_t mm0[2] = {0, 0};
    const unsigned long long bad0 = ~0ull;
    BUILD_CHECK(hipMemcpyAsync(mm, mm0, sizeof mm0, hipMemcpyHostToDevice, stream));
    BUILD_CHECK(hipMemcpyAsync(bad, &bad0, sizeof bad0, hipMemcpyHostToDevice, stream));
    if (n) {
        hipLaunchKernelGGL(k_minmax, dim3((unsigned)std::min<uint64_t>(2048, (n + kThreads - 1) / kThreads)), dim3(kThreads),
                           0, stream, xyz, rgb, n, mm, bad);
        BUILD_CHECK(hipGetLastError());
    }
    int32_t mmh[2];
    BUILD_CHECK(hipMemcpyAsync(mmh, mm, sizeof mmh, hipMemcpyDeviceToHost, stream));
    const unsigned long long badh = read_back(bad, stream);
    if (badh != ~0ull) {
        const uint32_t v = read_back(rgb + badh, stream);
        err = "voxel colour " + std::to_string(v) + " at index " + std::to_string(badh) + " exceeds 24-bit RGB";
        return -1;
    }
    const int64_t D64 = (int64_t)mmh[1] - (int64_t)mmh[0] + 1;
    if (D64 > 1024) {
        err = "scene spans more than 1024 regions per axis";
        return -1;
    }
    out.D = (uint32_t)D64;
    out.min_coord = mmh[0];
    const uint64_t D3 = (uint64_t)out.D * out.D * out.D;
    uint32_t rbits = 1;
    while (rbits < 64 && (D3 - 1) >> rbits) ++rbits;
    const uint32_t shift = store == STORE_VCS ? 18u : 26u;          // key >> shift = region
    // region table (all null) even for an empty scene
    BUILD_CHECK(hipMalloc(&out.region_slot, D3 * sizeof(uint32_t)));
    out.region_slot_bytes = D3 * sizeof(uint32_t);
    hipLaunchKernelGGL(k_fill_u32, dim3((unsigned)std::min<uint64_t>(4096, (D3 + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                       stream, (uint32_t*)out.region_slot, D3, kNone);
    BUILD_CHECK(hipGetLastError());

    uint64_t m = 0;
    uint64_t *key_a = nullptr, *key_b = nullptr, *ukey = nullptr;
    uint32_t *idx_a = nullptr, *idx_b = nullptr, *uidx = nullptr, *flag = nullptr, *pos = nullptr;
    uint32_t nr = 0;
    uint32_t *rstart = nullptr, *rslot_of = nullptr;
    if (n) {
        // 2-3. keys and a stable radix sort by key
        BUILD_CHECK(s.alloc(&key_a, n));
        BUILD_CHECK(s.alloc(&key_b, n));
        BUILD_CHECK(s.alloc(&idx_a, n));
        BUILD_CHECK(s.alloc(&idx_b, n));
        hipLaunchKernelGGL(k_keys, blocks_for(n), dim3(kThreads), 0, stream, xyz, n, out.min_coord, out.D, store, key_a, idx_a);
        BUILD_CHECK(hipGetLastError());
        size_t sort_bytes = 0;
        const unsigned end_bit = shift + rbits;
        BUILD_CHECK(rocprim::radix_sort_pairs(nullptr, sort_bytes, key_a, key_b, idx_a, idx_b, (size_t)n, 0, end_bit, stream));
        void* sort_tmp = nullptr;
        BUILD_CHECK(s.alloc((char**)&sort_tmp, sort_bytes));
        BUILD_CHECK(rocprim::radix_sort_pairs(sort_tmp, sort_bytes, key_a, key_b, idx_a, idx_b, (size_t)n, 0, end_bit, stream));
        // 4. keep the last insertion of every key
        BUILD_CHECK(s.alloc(&flag, n));
        BUILD_CHECK(s.alloc(&pos, n));
        hipLaunchKernelGGL(k_flag_last, blocks_for(n), dim3(kThreads), 0, stream, key_b, n, flag);
        BUILD_CHECK(hipGetLastError());
        if (int rc = scan(false, flag, pos, n, stream, err)) return rc;
        m = (uint64_t)read_back(pos + n - 1, stream) + read_back(flag + n - 1, stream);
        BUILD_CHECK(s.alloc(&ukey, m));
        BUILD_CHECK(s.alloc(&uidx, m));
        hipLaunchKernelGGL(k_compact, blocks_for(n), dim3(kThreads), 0, stream, key_b, idx_b, flag, pos, n, ukey, uidx);
        BUILD_CHECK(hipGetLastError());
        // 5. regions: starts, slots (region order), the slot of every voxel
        hipLaunchKernelGGL(k_flag_first, blocks_for(m), dim3(kThreads), 0, stream, ukey, m, shift, flag);
        BUILD_CHECK(hipGetLastError());
        if (int rc = scan(false, flag, pos, m, stream, err)) return rc;
        nr = read_back(pos + m - 1, stream) + read_back(flag + m - 1, stream);
        BUILD_CHECK(s.alloc(&rstart, nr));
        hipLaunchKernelGGL(k_starts, blocks_for(m), dim3(kThreads), 0, stream, flag, pos, m, rstart);
        hipLaunchKernelGGL(k_region_slots, blocks_for(nr), dim3(kThreads), 0, stream, ukey, rstart, nr, shift, (uint32_t*)out.region_slot);
        BUILD_CHECK(hipGetLastError());
        BUILD_CHECK(s.alloc(&rslot_of, m));
        if (int rc = scan(true, flag, rslot_of, m, stream, err)) return rc;
        hipLaunchKernelGGL(k_minus_one, blocks_for(m), dim3(kThreads), 0, stream, rslot_of, m);
        BUILD_CHECK(hipGetLastError());
    }
    out.n_regions = nr;
    out.n_voxels = m;
    if (store == STORE_VCS && nr > kVcsMaxRegions) {   // (cuckoo scenes have no region bound)
        err = "VCS scene with " + std::to_string(nr) + " occupied 64^3 regions (at most " +
              std::to_string(kVcsMaxRegions) + ")";
        return -1;
    }

    if (store == STORE_VCS) {
        const uint64_t words = std::max<uint64_t>((uint64_t)nr * 8192u, 16u);
        BUILD_CHECK(hipMalloc(&out.vcs_mask, words * sizeof(uint2)));
        out.vcs_mask_bytes = words * sizeof(uint2);
        hipLaunchKernelGGL(k_fill_u2, dim3((unsigned)std::min<uint64_t>(8192, (words + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                           stream, (uint2*)out.vcs_mask, words, make_uint2(0u, kNone));
        BUILD_CHECK(hipGetLastError());
        BUILD_CHECK(hipMalloc(&out.vcs_vals, std::max<uint64_t>(m, 1) * sizeof(uint32_t)));
        out.vcs_vals_bytes = std::max<uint64_t>(m, 1) * sizeof(uint32_t);
        if (m) {
            hipLaunchKernelGGL(k_gather_vals, blocks_for(m), dim3(kThreads), 0, stream, rgb, uidx, m, (uint32_t*)out.vcs_vals);
            // clusters: starts, then one thread per cluster writes its record
            hipLaunchKernelGGL(k_flag_first, blocks_for(m), dim3(kThreads), 0, stream, ukey, m, 9u, flag);
            BUILD_CHECK(hipGetLastError());
            if (int rc = scan(false, flag, pos, m, stream, err)) return rc;
            const uint32_t nc = read_back(pos + m - 1, stream) + read_back(flag + m - 1, stream);
            uint32_t* cstart;
            BUILD_CHECK(s.alloc(&cstart, nc));
            hipLaunchKernelGGL(k_starts, blocks_for(m), dim3(kThreads), 0, stream, flag, pos, m, cstart);
            hipLaunchKernelGGL(k_cluster_records, blocks_for(nc), dim3(kThreads), 0, stream, ukey, cstart, nc, m, rslot_of,
                               (uint2*)out.vcs_mask);
            BUILD_CHECK(hipGetLastError());
        } else {
            const uint32_t zero = 0;
            BUILD_CHECK(hipMemcpyAsync(out.vcs_vals, &zero, 4, hipMemcpyHostToDevice, stream));
        }
    } else {
        uint32_t *M = nullptr, *slots2 = nullptr, *base2 = nullptr, *failed = nullptr;
        uint64_t total = 2;
        if (nr) {
            BUILD_CHECK(s.alloc(&M, nr));
            BUILD_CHECK(s.alloc(&slots2, nr));
            BUILD_CHECK(s.alloc(&base2, nr));
            hipLaunchKernelGGL(k_region_sizes, blocks_for(nr), dim3(kThreads), 0, stream, rstart, nr, m, M, slots2);
            BUILD_CHECK(hipGetLastError());
            if (int rc = scan(false, slots2, base2, (uint64_t)nr, stream, err)) return rc;
            total = (uint64_t)read_back(base2 + nr - 1, stream) + read_back(slots2 + nr - 1, stream);
            if (total >= 0xFFFFFFFFull) { err = "hash slots exceed 32-bit offsets"; return -5; }
            total = std::max<uint64_t>(total, 2);
        }
        BUILD_CHECK(hipMalloc(&out.ht_slots, total * sizeof(uint2)));
        out.ht_slots_bytes = total * sizeof(uint2);
        hipLaunchKernelGGL(k_fill_u2, dim3((unsigned)std::min<uint64_t>(8192, (total + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                           stream, (uint2*)out.ht_slots, total, make_uint2(kEmpty, 0u));
        const uint64_t metas = std::max<uint32_t>(nr, 1);
        BUILD_CHECK(hipMalloc(&out.ht_meta, metas * sizeof(uint4)));
        out.ht_meta_bytes = metas * sizeof(uint4);
        BUILD_CHECK(hipMemsetAsync(out.ht_meta, 0, metas * sizeof(uint4), stream));
        if (nr) {
            BUILD_CHECK(s.alloc(&failed, 1));
            BUILD_CHECK(hipMemsetAsync(failed, 0, 4, stream));
            hipLaunchKernelGGL(k_cuckoo, dim3(nr), dim3(64), 0, stream, ukey, uidx, rgb, rstart, nr, m, M, base2,
                               (uint2*)out.ht_slots, (uint4*)out.ht_meta, failed);
            BUILD_CHECK(hipGetLastError());
            if (read_back(failed, stream)) { err = "cuckoo hash table build failed"; return -5; }
        }
    }
    BUILD_CHECK(hipStreamSynchronize(stream));
    return 0;
}

}  // namespace vr
