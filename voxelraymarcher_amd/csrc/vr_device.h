// vr_device.h -- device-side building blocks of the ray-march kernels
// (vr_march.hip: the tile pass, one lane per pixel, and the crawl pass):
// math with the reference's operation order, CUDA-semantics conversions,
// the storage lookups and the lighting.  FP policy: SURVEY.md 8(c).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vr_internal.h"

namespace vr {
namespace {

constexpr float kEps = 0.0001f;               // EPSILON (VoxelFunctions.cuh:19)
constexpr float kInf = __builtin_huge_valf();

enum { STORE_VCS = 0, STORE_HASH = 1 };
enum { ALGO_LONGEST = 0, ALGO_ORIGINAL = 1 };

struct f3 { float x, y, z; };
struct i3 { int32_t x, y, z; };

__device__ __forceinline__ f3 mk(float a, float b, float c) { return f3{a, b, c}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }   // Vector3.cuh:106
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }   // :112
__device__ __forceinline__ f3 mul(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }   // :118
__device__ __forceinline__ f3 scl(float t, f3 a) { return f3{t * a.x, t * a.y, t * a.z}; }      // :130,142
__device__ __forceinline__ float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }  // :148
__device__ __forceinline__ f3 unit(f3 a) {                                                         // :162, :79
    float len = sqrtf(a.x * a.x + a.y * a.y + a.z * a.z);
    return f3{a.x / len, a.y / len, a.z / len};
}
__device__ __forceinline__ f3 ld3(const float* p) { return f3{p[0], p[1], p[2]}; }

// Runtime axis select without private-memory arrays.
__device__ __forceinline__ float comp(f3 v, uint32_t a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }
__device__ __forceinline__ int32_t geti(i3 v, uint32_t a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }
__device__ __forceinline__ void seti(i3& v, uint32_t a, int32_t val) {
    v.x = a == 0 ? val : v.x;
    v.y = a == 1 ? val : v.y;
    v.z = a == 2 ? val : v.z;
}
__device__ __forceinline__ void setf(f3& v, uint32_t a, float val) {
    v.x = a == 0 ? val : v.x;
    v.y = a == 1 ? val : v.y;
    v.z = a == 2 ? val : v.z;
}

// static_cast<int32_t>(float) / static_cast<uint32_t>(float) with the CUDA
// device semantics (cvt.rzi.s32.f32 / cvt.rzi.u32.f32: truncate, saturate,
// NaN -> 0).  v_cvt_i32_f32 / v_cvt_u32_f32 implement exactly that on CDNA;
// emitting them directly keeps the conversion one branch-free instruction
// (a C cast is UB out of range and hipcc guards it with control flow).
__device__ __forceinline__ int32_t f2i(float f) {
    int32_t r;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(f));
    return r;
}
__device__ __forceinline__ uint32_t f2u(float f) {
    uint32_t r;
    asm("v_cvt_u32_f32 %0, %1" : "=v"(r) : "v"(f));
    return r;
}

// Correctly rounded n / d with the reciprocal hoisted out of a walk:
//   r = fma(fma(-d, r0, 1), r0, r0), r0 = v_rcp_f32(d)     (once per direction)
//   q = RN(n * r);  q' = fma(fma(-d, q, n), r, q) = RN(n / d)
// (one Markstein correction: mul + 2 fma per division).  For normal n, d whose
// intermediates stay normal every step scales exactly with the exponents, so
// the result depends only on the two significands -- r included:
// tools/div_proof.hip checks, on the device, that r(+-m 2^e) = +-r(m) 2^-e for
// every significand m and every e of the domain, and all 2^23 x 2^23
// significand pairs (n, d) against hipcc's IEEE division: 0 mismatches
// (profiles/r02/div_proof.json; the same holds with r = RN(1/d)).  The domain
// that keeps r, q and q' normal and the residual exact: 2^-64 <= |d| <= 2^20,
// 2^-90 <= |n| <= 2^20; tools/div_check.hip re-checks every numerator of it for
// a list of divisors.  Callers test div_fast_ok() (or the bounds it checks:
// inside a region walk |n| < 73 always) and fall back to `/`.
// (Round 1 ran hipcc's own sequence with the reciprocal half hoisted: mul + 4 fma.)
struct Rcp { float d, r; bool ok; };
__device__ __forceinline__ Rcp rcp_setup(float d) {
    const float r0 = __builtin_amdgcn_rcpf(d);
    const float r = __builtin_fmaf(__builtin_fmaf(-d, r0, 1.0f), r0, r0);
    const float a = fabsf(d);
    return Rcp{d, r, a >= 0x1p-64f && a <= 0x1p+20f};
}
__device__ __forceinline__ bool div_fast_ok(float n, const Rcp& c) {
    const float a = fabsf(n);
    return c.ok && a >= 0x1p-90f && a <= 0x1p+20f;
}
__device__ __forceinline__ float div_fast(float n, const Rcp& c) {
    const float q = n * c.r;
    return __builtin_fmaf(__builtin_fmaf(-c.d, q, n), c.r, q);
}
// px ? ceilf(o) + EPSILON : floorf(o) - EPSILON, branch-free: with s = +-1,
// s * (ceilf(s * o) + EPSILON) (floor(o) = -ceil(-o); negation and round-to-
// nearest commute, so both forms round identically).
__device__ __forceinline__ float next_plane(float o, float s, float eps) {
    return s * (ceilf(s * o) + eps);
}
// The same as one fma with se = s * EPSILON (exact): s * ceilf(s * o) is exact,
// so fma rounds s * c + s * eps once, = s * RN(c + eps) by the same symmetry.
__device__ __forceinline__ float next_plane_fma(float o, float s, float se) {
    return __builtin_fmaf(s, ceilf(s * o), se);
}

// (a << s) | b as one v_lshl_or_b32
__device__ __forceinline__ uint32_t lshl_or(uint32_t a, uint32_t sh, uint32_t b) {
    uint32_t r;
    asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "i"(sh), "v"(b));
    return r;
}
// m ? a : b per bit (m = 0 or ~0): one v_bfi_b32 (the compiler splits the
// and/or form into three operations).
__device__ __forceinline__ float bit_select(uint32_t m, float a, float b) {
    float r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}

// u32 `h % M` for a divisor fixed over a walk: minv = floor(2^32 / M) (2^32 - 1
// for M = 1) gives q' = mulhi(h, minv) in {q - 1, q}, so r' = h - q' M is in
// [0, 2M) and one wrap-around min finishes it.  Exact for every h and M >= 1.
struct FastMod { uint32_t M, minv; };
__device__ __forceinline__ FastMod fastmod_setup(uint32_t M) {
    uint32_t q = 0xFFFFFFFFu / M;                       // floor((2^32 - 1) / M)
    if (M != 1u && 0xFFFFFFFFu - q * M == M - 1u) ++q;  // M divides 2^32
    return FastMod{M, q};
}
__device__ __forceinline__ uint32_t fastmod(uint32_t h, FastMod f) {
    const uint32_t r = h - __umulhi(h, f.minv) * f.M;
    return min(r, r - f.M);
}

// CuckooHashTable::hashFunc1 / hashFunc2 (CuckooHashTable.cuh:181-202),
// int arithmetic with arithmetic right shifts.
__device__ __forceinline__ uint32_t hash1(uint32_t k, uint32_t offset) {
    k = (k + 0x7ed55d16u) + (k << 12);
    k = (k ^ 0xc761c23cu) ^ (uint32_t)((int32_t)k >> 19);
    k = (k + 0x165667b1u) + (k << 5);
    k = (k + 0xd3a2646cu) ^ (k << 9);
    k = (k + 0xfd7046c5u) + (k << 3);
    k = (k ^ 0xb55a4f09u) ^ (uint32_t)((int32_t)k >> 16);
    return k + offset;
}
__device__ __forceinline__ uint32_t hash2(uint32_t k, uint32_t prime) {
    k = (k ^ 61u) ^ (uint32_t)((int32_t)k >> 16);
    k = k + (k << 3);
    k = k ^ (uint32_t)((int32_t)k >> 4);
    k = k * prime;
    k = k ^ (uint32_t)((int32_t)k >> 15);
    return k;
}

// (float)c / 255.0f, correctly rounded (VoxelFunctions.cuh:71-73), for c in
// [0, 255]: div_fast with the correctly rounded reciprocal RN(1/255) (a
// compile-time constant), exact on this domain (tools/div_proof.hip; c = 0
// gives +0 as the division does).  Round 1 filled a 256-entry LDS table per
// workgroup: ~140 VALU per wave and a barrier at every kernel start.
__device__ __forceinline__ float div255(uint32_t c) {
    return div_fast((float)c, Rcp{255.0f, 1.0f / 255.0f, true});
}

// VCS: the mask word of the cluster holding the voxel, {occupancy bits,
// value index of the word's first voxel} or {0, kNone} (no cluster).
// Hashtable: unused ({0,0}: the space always exists).
typedef uint2 Blk;
__device__ __forceinline__ bool absent(Blk b) { return b.y == kNone; }

struct Hit {
    uint32_t col;       // the voxel's stored colour
    uint32_t nc;        // surface normal for the lighting: one component +-1, the others +0
                        // (every normal the walks make), as bits(+-1.0f) | axis -- one VGPR
                        // instead of three across the lighting (see normal_of)
    f3 so;              // hit location (region-local): lighting point and shadow-ray origin
    i3 region;          // currentRegion at the hit
    bool longest;       // isInShadowRayMarchVoxelSceneLongestAxis vs ...Original
};

// BUDGET: kTileBudget (tile pass: aborted = hand the pixel to the crawl pass)
// or kCrawlBudget (crawl pass: the hang guard).
template <int STORE, bool COUNT, uint32_t BUDGET>
struct Ctx {
    static constexpr uint32_t kBudget = BUDGET;
    const KScene& s;
    const KView& v;
    uint32_t iters = 0;
    bool aborted = false;
    uint32_t bytes = 0;
    uint32_t ff = 0;     // (COUNT) crawl iterations credited in closed form (crawl_run)
    uint32_t nl = 0;     // (COUNT) crawl-pass skip steps answered from the LDS cluster bits (counted, not loaded)
#ifdef VR_CRAWL_PROF
    uint32_t d_runs = 0, d_trips = 0;   // (diagnostic builds) crawl_run calls that applied steps, their loop trips
#endif

    __device__ Ctx(const KScene& s_, const KView& v_) : s(s_), v(v_) {}

    __device__ __forceinline__ void count(uint32_t b) {
        if (COUNT) bytes += b;
    }
    // n crawl iterations fast-forwarded: the existence read each of them stands for
    //  is credited, but the kernel never issues it
    __device__ __forceinline__ void count_ff(uint32_t n) {
#ifdef VR_CRAWL_PROF
        ++d_runs;
        ff += COUNT ? 0u : n;
#endif
        if (COUNT) {
            bytes += 4u * n;
            ff += n;
        }
    }
    __device__ __forceinline__ bool tick() {
        if (aborted) return false;
        if (++iters > BUDGET) { aborted = true; return false; }
        return true;
    }

    // VoxelScene::isRayInScene / getRegionStorageStructure (Renderer.cuh:29-44)
    __device__ __forceinline__ bool in_scene(i3 r) const {
        uint32_t mc = (uint32_t)s.min_coord;
        return ((uint32_t)r.x - mc) < s.D && ((uint32_t)r.y - mc) < s.D && ((uint32_t)r.z - mc) < s.D;
    }
    __device__ __forceinline__ uint32_t region_at(i3 r) {
        uint32_t mc = (uint32_t)s.min_coord;
        uint32_t ux = (uint32_t)r.x - mc, uy = (uint32_t)r.y - mc, uz = (uint32_t)r.z - mc;
        count(4);
        return s.region_slot[ux + uy * s.D + uz * s.D * s.D];
    }

    // the same slot read again, not counted (the walk that resumes a deferred
    // crawl already paid for it)
    __device__ __forceinline__ uint32_t region_at_nocount(i3 r) const {
        uint32_t mc = (uint32_t)s.min_coord;
        uint32_t ux = (uint32_t)r.x - mc, uy = (uint32_t)r.y - mc, uz = (uint32_t)r.z - mc;
        return s.region_slot[ux + uy * s.D + uz * s.D * s.D];
    }

    // `short` getVoxelClusterID (VoxelClusterStore.cuh:21-24); -1 = past the
    // reference's 512-entry directory (no cluster).
    __device__ __forceinline__ static int32_t cluster_id(int32_t x, int32_t y, int32_t z) {
        uint32_t c = (((uint32_t)x >> 3) << 6) | (((uint32_t)y >> 3) << 3) | ((uint32_t)z >> 3);
        int32_t cid = (int32_t)(int16_t)(uint16_t)c;
        return cid < 512 ? cid : -1;
    }
    // In-cluster voxel index ((x&7)<<6|(y&7)<<3|z&7): same order as the
    // reference's full keys x<<20|y<<10|z inside one cluster.
    __device__ __forceinline__ static uint32_t in_cluster(int32_t x, int32_t y, int32_t z) {
        return (((uint32_t)x & 7u) << 6) | (((uint32_t)y & 7u) << 3) | ((uint32_t)z & 7u);
    }
    // A region's 8192 mask words are stored at word index
    //   y2 | x0..x5 << 1 | y3..y5 << 7 | z3..z5 << 10   (vcs_word_index)
    // so a cluster's 16 words are contiguous (one 128-B record, in-cluster
    // word w = (x&7)<<1 | y2 as before) and the index of an in-region voxel
    // is a few bit operations.
    __device__ __forceinline__ static uint32_t slot_of(int32_t cid) {
        const uint32_t c = (uint32_t)cid;
        return (c >> 6) | (((c >> 3) & 7u) << 3) | ((c & 7u) << 6);
    }
    __device__ __forceinline__ const uint2* masks(uint32_t reg, int32_t cid) const {
        return s.vcs_mask + (size_t)reg * 8192u + (slot_of(cid) << 4);
    }
    // Word w of cluster slot `slot`'s record in region reg, addressed as a 32-bit byte offset
    // from the scene's (uniform) mask array, as the walks' own loads are: no 64-bit per-region
    // pointer is made (one that is, is loop-invariant, hoisted out of the walks and spilled).
    __device__ __forceinline__ Blk mword(uint32_t reg, uint32_t slot, uint32_t w) const {
        return *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(s.vcs_mask) +
                                               ((reg << 16) | (slot << 7) | (w << 3)));
    }
    __device__ __forceinline__ static uint32_t word_index(uint32_t x, uint32_t y, uint32_t z) {   // x,y,z < 64
        // v_bfe + 3 v_lshl_or; the two v_and (y & 0x38, z & 0x38) are shared
        // with the cluster-skip planes of the walk
        // (the instructions are pinned: left to itself the compiler re-associates
        // the shifts and masks into 8 operations)
        const uint32_t lo = lshl_or(x, 1u, __builtin_amdgcn_ubfe(y, 2u, 1u));
        const uint32_t hi = lshl_or(z & 0x38u, 3u, y & 0x38u);
        return lshl_or(hi, 4u, lo);
    }
    // Bit of an in-region voxel in its mask word, in the low 5 bits only
    // ((y&3)<<3 | z&7 there; v_bfe and shifts read just those): one v_bfi.
    __device__ __forceinline__ static uint32_t word_bit5(uint32_t y, uint32_t z) {
        uint32_t r;
        asm("v_bfi_b32 %0, 7, %1, %2" : "=v"(r) : "v"(z), "v"(y << 3));
        return r;
    }

    // doesVoxelSpaceExist (StorageStructure.cuh:29-32,49-52) ->
    // VoxelClusterStore::doesClusterExist (VoxelClusterStore.cuh:93-99).
    // VCS: one 8-B read of the mask word the later lookup of this voxel needs,
    // so existence and lookup share a single dependent load.
    __device__ __forceinline__ Blk exists(uint32_t reg, int32_t x, int32_t y, int32_t z) {
        if (STORE == STORE_HASH) return Blk{0u, 0u};
        count(4);
        return mask_word(reg, x, y, z);
    }
    // The read behind exists() without its byte count (for walks that request
    // it ahead and count it when the iteration that needs it runs).
    __device__ __forceinline__ Blk mask_word(uint32_t reg, int32_t x, int32_t y, int32_t z) const {
        const int32_t cid = cluster_id(x, y, z);
        if (cid < 0) return Blk{0u, kNone};
        return mword(reg, slot_of(cid), in_cluster(x, y, z) >> 5);
    }

    // Reference binary-search probes for a key of rank `rank` (number of keys
    // < q) among n sorted keys: key[mid] < q <=> mid < rank, key[mid] == q <=>
    // found && mid == rank (performBinarySearch, VoxelClusterStore.cuh:101-126).
    // Only the COUNT instantiations evaluate it (SURVEY 8(d) bytes); n and the
    // rank come from the cluster's first and last mask words.
    __device__ __forceinline__ void count_bsearch(const uint2* m, uint32_t idx, bool found) {
        if (!COUNT) return;
        const uint2 m0 = m[0], m15 = m[15];
        const uint32_t n = m15.y + __popc(m15.x) - m0.y, rank = idx - m0.y;
        int32_t low = 0, high = (int32_t)n - 1;
        uint32_t probes = 0;
        while (low <= high) {
            int32_t mid = low + ((high - low) >> 1);
            ++probes;
            if (found && (uint32_t)mid == rank) break;
            if ((uint32_t)mid < rank) low = mid + 1; else high = mid - 1;
        }
        count(4 + 4 * probes + (found ? 4 : 0));
    }

    // A coordinate outside [0,64) whose `short` cluster id still lands in the
    // directory (very large longest-axis grid coordinates): the reference
    // binary-searches the 32-bit key x<<20|y<<10|z (which wraps) among the
    // cluster's full keys.  Those are increasing in the in-cluster index, so the
    // number of keys below K is the population below the first index t whose
    // full key is >= K (found iff that key equals K and is present).  Exact, rare.
    __device__ __forceinline__ uint32_t lookup_aliased(uint32_t reg, int32_t x, int32_t y, int32_t z) {
        const int32_t cid = cluster_id(x, y, z);
        const uint32_t slot = slot_of(cid);
        const uint32_t K = ((uint32_t)x << 20) | ((uint32_t)y << 10) | (uint32_t)z;
        const uint32_t bx = ((uint32_t)cid >> 6) * 8u, by = (((uint32_t)cid >> 3) & 7u) * 8u, bz = ((uint32_t)cid & 7u) * 8u;
        auto full = [&](uint32_t q) { return ((bx + (q >> 6)) << 20) | ((by + ((q >> 3) & 7u)) << 10) | (bz + (q & 7u)); };
        uint32_t lo = 0, hi = 512;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (full(mid) < K) lo = mid + 1; else hi = mid;
        }
        if (lo == 512u) {
            if (COUNT) {
                const uint2 m15 = mword(reg, slot, 15u);
                count_bsearch(masks(reg, cid), m15.y + __popc(m15.x), false);
            }
            return kEmpty;
        }
        const uint2 w = mword(reg, slot, lo >> 5);
        const uint32_t bit = lo & 31u;
        const bool found = full(lo) == K && ((w.x >> bit) & 1u);
        const uint32_t idx = w.y + __popc(w.x & ((1u << bit) - 1u));
        if (COUNT) count_bsearch(masks(reg, cid), idx, found);
        return found ? s.vcs_vals[idx] : kEmpty;
    }

    // VoxelClusterStore::lookupVoxel / performBinarySearch (VoxelClusterStore.cuh:101-135):
    // the binary search's answer (is the key present, and its value) read off
    // the cluster's occupancy mask: bit q of the mask word `blk` fetched by
    // exists(), value index = word base + popcount of the lower bits.  No
    // further dependent load before the value itself.
    // CuckooHashTable::lookupVoxel (CuckooHashTable.cuh:59-76): both candidate
    // slots are requested together (the second read is counted only when the
    // reference would make it).
    __device__ __forceinline__ uint32_t lookup(uint32_t reg, Blk blk, int32_t x, int32_t y, int32_t z) {
        if (STORE == STORE_VCS) {
            if (((uint32_t)x | (uint32_t)y | (uint32_t)z) >= 64u) return lookup_aliased(reg, x, y, z);
            const uint32_t bit = in_cluster(x, y, z) & 31u;
            const bool found = (blk.x >> bit) & 1u;
            const uint32_t idx = blk.y + __popc(blk.x & ((1u << bit) - 1u));
            if (COUNT) count_bsearch(masks(reg, cluster_id(x, y, z)), idx, found);
            return found ? s.vcs_vals[idx] : kEmpty;
        } else {
            const uint32_t key = ((uint32_t)x << 20) | ((uint32_t)y << 10) | (uint32_t)z;   // generate3DPoint
            // the region's key-presence filter (KScene::ht_filter): a key the tables do not hold
            // costs the reference key1 + key2 and misses.  Tables hold local keys only (fields
            // x, y, z < 64), so a key with any other bit set -- a coordinate outside the
            // region, wrapped into the 32-bit key -- cannot be there.
            if ((key & ~0x03F0FC3Fu) != 0u) { count(8); return kEmpty; }
            {
                const uint32_t kx = (key >> 20) & 63u, ky = (key >> 10) & 63u, kz = key & 63u;
                const uint32_t fw = s.ht_filter[(size_t)reg * kHashFilterWords + word_index(kx, ky, kz)];
                if (!((fw >> (word_bit5(ky, kz) & 31u)) & 1u)) { count(8); return kEmpty; }
            }
            const uint4 m = s.ht_meta[reg];          // {base, M, prime, offset}
            const uint32_t s1 = hash1(key, m.w) % m.y;
            const uint32_t s2 = hash2(key, m.z) % m.y;
            const uint2 e1 = s.ht_slots[m.x + s1];
            const uint2 e2 = s.ht_slots[m.x + m.y + s2];
            count(4);
            if (e1.x == key) { count(4); return e1.y; }
            count(4);
            if (e2.x == key) { count(4); return e2.y; }
            return kEmpty;
        }
    }

    // applyLighting / applyDirectionalLightingToColor / applyPointLightingToColor
    // (Renderer.cuh:57-86,249-258), colour packing (VoxelFunctions.cuh:69-83).
    __device__ __forceinline__ uint32_t lighting(uint32_t col, uint32_t nc, f3 rwp, f3 ro) const {
        const f3 n = normal_of(nc);
        f3 LC = ld3(v.LC);
        // convertRGBIntegerColorToVector: c / 255.0f per channel, correctly rounded
        // (div255); colours are < 2^24 so R = col >> 16 <= 255.
        f3 c = mk(div255(col >> 16), div255((col >> 8) & 0xFFu), div255(col & 0xFFu));
        f3 r;
        if (v.use_point_light) {
            f3 p2l = sub(ld3(v.LP), add(rwp, ro));
            float dist = sqrtf(p2l.x * p2l.x + p2l.y * p2l.y + p2l.z * p2l.z);
            f3 ldir = unit(p2l);
            float att = 1.0f / (1.0f + 0.045f * dist + 0.0075f * (dist * dist));
            float diff = fmaxf(dot3(n, ldir), 0.0f);
            r = mul(scl(att, scl(diff, LC)), c);
        } else {
            float diff = fmaxf(dot3(n, ld3(v.L)), 0.0f);
            r = mul(c, scl(diff, LC));
        }
        uint32_t R = f2u(r.x * 255.0f), G = f2u(r.y * 255.0f), B = f2u(r.z * 255.0f);
        return (R << 16) | (G << 8) | B;
    }

    // copysignf(1.0f, -x), computed where it is used: the volatile barrier keeps
    // the compiler from hoisting the three signs out of the walk loops, where they
    // were spilled to scratch for every pixel (three VGPRs over the 7-wave budget).
    __device__ __forceinline__ static float neg_sign_one(float x) {
        uint32_t u = __float_as_uint(x);
        asm volatile("" : "+v"(u));
        return __uint_as_float((u & 0x80000000u) ^ 0xBF800000u);
    }

    // getNormalFromTValues (Renderer.cuh:237-247)
    __device__ __forceinline__ static uint32_t normal_from_t(float tX, float tY, float tZ, float tMin, f3 d) {
        if (tX == tMin) return ncode(0u, neg_sign_one(d.x));
        if (tY == tMin) return ncode(1u, neg_sign_one(d.y));
        return ncode(2u, neg_sign_one(d.z));
    }
    // Hit::nc: the normal whose component `axis` is `one` (+-1.0f, low mantissa bits 0)
    // and whose other components are +0.0f
    __device__ __forceinline__ static uint32_t ncode(uint32_t axis, float one) {
        return __float_as_uint(one) | axis;
    }
    __device__ __forceinline__ static f3 normal_of(uint32_t nc) {
        const float one = __uint_as_float(nc & ~3u);
        const uint32_t a = nc & 3u;
        return mk(a == 0u ? one : 0.0f, a == 1u ? one : 0.0f, a == 2u ? one : 0.0f);
    }

    __device__ __forceinline__ static bool in_region(f3 o) {               // Renderer.cuh:93-98
        return o.x >= 0.0f && o.x < 64.0f && o.y >= 0.0f && o.y < 64.0f && o.z >= 0.0f && o.z < 64.0f;
    }
    // The same predicate on the float encodings: after x + 0.0f (which turns
    // -0 into +0 and keeps NaN), x in [0, 64) <=> bits(x) < bits(64.0f).
    __device__ __forceinline__ static bool in_region_bits(f3 o) {
        const uint32_t a = __float_as_uint(o.x + 0.0f), b = __float_as_uint(o.y + 0.0f), c = __float_as_uint(o.z + 0.0f);
        return max(max(a, b), c) < 0x42800000u;
    }
    // For coordinates that are not -0: a walk position is canonicalised (x + 0)
    // once, and o + p only gives a zero by exact cancellation, which rounds to
    // +0 -- so positions stepped from it are never -0 either.
    __device__ __forceinline__ static bool in_region_bits_nz(f3 o) {
        return max(max(__float_as_uint(o.x), __float_as_uint(o.y)), __float_as_uint(o.z)) < 0x42800000u;
    }
    // Loop-state equality for the never-finishes test (crawl pass): the same
    // bits, or both NaN (every later use treats NaNs alike).
    __device__ __forceinline__ static bool same_f(float a, float b) {
        return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
    }
    __device__ __forceinline__ static bool same_pos(i3 ca, f3 a, i3 cb, f3 b) {
        return ca.x == cb.x && ca.y == cb.y && ca.z == cb.z && same_f(a.x, b.x) && same_f(a.y, b.y) &&
               same_f(a.z, b.z);
    }
    // Brent's cycle detection over a loop's state (cr, o) (crawl pass): a snapshot is taken at
    // rounds 1, 2, 4, 8, ... and every later state is compared with it, so a loop whose state
    // repeats -- after any prefix, with any period -- is found within about twice (prefix +
    // period) rounds.  Every round of the reference's region, null-region and entry-clip loops
    // is a function of this state alone, so a repeat means the reference never returns; the
    // pixel is then declared non-terminating.  (Round 4 compared each round with
    // the one before only, which finds period-1 repeats: fixed points.)
    struct Cycle {
        i3 c;
        f3 o;
        uint32_t lam, pow;
    };
    __device__ __forceinline__ static Cycle cycle_start(i3 c, f3 o) { return Cycle{c, o, 0u, 1u}; }
    __device__ __forceinline__ static bool cycle_step(Cycle& y, i3 c, f3 o) {
        if (same_pos(c, o, y.c, y.o)) return true;
        if (++y.lam == y.pow) {
            y.c = c;
            y.o = o;
            y.pow <<= 1;
            y.lam = 0u;
        }
        return false;
    }
    __device__ __forceinline__ static bool grid_in_region(int32_t a, int32_t b, int32_t c) {   // :436-439
        return (uint32_t)a < 64u && (uint32_t)b < 64u && (uint32_t)c < 64u;
    }

    // Region advance (e.g. Renderer.cuh:421-429).
    __device__ __forceinline__ static void advance_region(i3& cr, f3& o) {
        int32_t dx = f2i(floorf(o.x / 64.0f)), dy = f2i(floorf(o.y / 64.0f)), dz = f2i(floorf(o.z / 64.0f));
        cr.x += dx; cr.y += dy; cr.z += dz;
        o = sub(o, mk((float)(dx * kBlock), (float)(dy * kBlock), (float)(dz * kBlock)));
    }

    // Null-region skip body (Renderer.cuh:386-409; guarded form :187-210).
    template <bool GUARDED>
    __device__ __forceinline__ bool skip_null(i3& cr, f3& o, f3 d, uint32_t& reg) {
        return skip_null_rt(cr, o, d, reg, GUARDED);
    }
    __device__ __forceinline__ bool skip_null_rt(i3& cr, f3& o, f3 d, uint32_t& reg, const bool GUARDED) {
        float nx = d.x > 0.0f ? 64.0f + kEps : 0.0f - kEps;
        float ny = d.y > 0.0f ? 64.0f + kEps : 0.0f - kEps;
        float nz = d.z > 0.0f ? 64.0f + kEps : 0.0f - kEps;
        const float tX = (GUARDED && d.x == 0.0f) ? kInf : (nx - o.x) / d.x;
        const float tY = (GUARDED && d.y == 0.0f) ? kInf : (ny - o.y) / d.y;
        const float tZ = (GUARDED && d.z == 0.0f) ? kInf : (nz - o.z) / d.z;
        float tMin = fminf(tX, fminf(tY, tZ));
        o = add(o, scl(tMin, d));
        advance_region(cr, o);
        if (!in_scene(cr)) return false;
        reg = region_at(cr);
        return true;
    }

};

}  // namespace
}  // namespace vr
