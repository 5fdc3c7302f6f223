// vr_device.h -- device-side building blocks shared by the ray-march kernels
// (vr_march.hip: one lane per pixel; vr_persist.hip: persistent state machine):
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

typedef uint2 Blk;    // VCS directory entry {block offset (16-B units), n}
__device__ __forceinline__ bool absent(Blk b) { return b.x == kNone; }

struct Hit {
    uint32_t col;       // the voxel's stored colour
    f3 n;               // surface normal for the lighting
    f3 so;              // hit location (region-local): lighting point and shadow-ray origin
    i3 region;          // currentRegion at the hit
    bool longest;       // isInShadowRayMarchVoxelSceneLongestAxis vs ...Original
};

template <int STORE, bool COUNT>
struct Ctx {
    const KScene& s;
    const KView& v;
    uint32_t iters = 0;
    bool aborted = false;
    uint32_t bytes = 0;

    __device__ Ctx(const KScene& s_, const KView& v_) : s(s_), v(v_) {}

    __device__ __forceinline__ void count(uint32_t b) {
        if (COUNT) bytes += b;
    }
    __device__ __forceinline__ bool tick() {
        if (aborted) return false;
        if (++iters > kIterBudget) { aborted = true; return false; }
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

    // doesVoxelSpaceExist (StorageStructure.cuh:29-32,49-52) ->
    // VoxelClusterStore::doesClusterExist (VoxelClusterStore.cuh:93-99).
    // Returns the directory entry {block offset, n} (VCS) or {0,0} (hashtable:
    // the space always exists); absent() = no cluster.
    __device__ __forceinline__ Blk exists(uint32_t reg, int32_t x, int32_t y, int32_t z) {
        if (STORE == STORE_HASH) return Blk{0u, 0u};
        count(4);
        uint32_t c = (((uint32_t)x >> 3) << 6) | (((uint32_t)y >> 3) << 3) | ((uint32_t)z >> 3);
        int32_t cid = (int32_t)(int16_t)(uint16_t)c;      // `short` getVoxelClusterID
        if (cid < 0 || cid >= 512) return Blk{kNone, 0u}; // past the reference's directory
        return s.vcs_dir[reg * 512u + (uint32_t)cid];
    }

    // Reference binary-search probes for a key of rank `rank` (number of keys
    // < q) among n sorted keys: key[mid] < q <=> mid < rank, key[mid] == q <=>
    // found && mid == rank (performBinarySearch, VoxelClusterStore.cuh:101-126).
    // Only the COUNT instantiations evaluate it (SURVEY 8(d) bytes).
    __device__ __forceinline__ void count_bsearch(uint32_t n, uint32_t rank, bool found) {
        if (!COUNT) return;
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
    // directory (longest-axis walks can probe one): the reference binary-searches
    // the full key x<<20|y<<10|z, which no key of the block can equal.  Rare;
    // run the reference search verbatim over the block's keys widened back to
    // full keys, so the probe count (COUNT) is exact too.
    __device__ uint32_t lookup_aliased(const uint4* b, VcsGeom gm, uint32_t n, int32_t x,
                                                                 int32_t y, int32_t z) {
        const uint32_t ux = (uint32_t)x, uy = (uint32_t)y, uz = (uint32_t)z;
        const uint32_t K = (ux << 20) | (uy << 10) | uz;
        const uint32_t c = (((ux >> 3) << 6) | ((uy >> 3) << 3) | (uz >> 3)) & 0x1FFu;
        const uint32_t bx = (c >> 6) * 8u, by = ((c >> 3) & 7u) * 8u, bz = (c & 7u) * 8u;
        const uint16_t* k16 = reinterpret_cast<const uint16_t*>(b + gm.u_keys);
        count(4);
        int32_t low = 0, high = (int32_t)n - 1;
        while (low <= high) {
            int32_t mid = low + ((high - low) >> 1);
            const uint32_t c9 = k16[mid];
            const uint32_t full = ((bx + (c9 >> 6)) << 20) | ((by + ((c9 >> 3) & 7u)) << 10) | (bz + (c9 & 7u));
            count(4);
            if (full == K) { count(4); return reinterpret_cast<const uint32_t*>(b + gm.u_vals)[mid]; }
            if (full < K) low = mid + 1; else high = mid - 1;
        }
        return kEmpty;
    }

    // Number of the 8 16-bit keys of a node that are < q.
    __device__ __forceinline__ static uint32_t count_lt(uint4 nd, uint32_t q) {
        uint32_t c = 0;
        c += (nd.x & 0xFFFFu) < q; c += (nd.x >> 16) < q;
        c += (nd.y & 0xFFFFu) < q; c += (nd.y >> 16) < q;
        c += (nd.z & 0xFFFFu) < q; c += (nd.z >> 16) < q;
        c += (nd.w & 0xFFFFu) < q; c += (nd.w >> 16) < q;
        return c;
    }
    __device__ __forceinline__ static uint32_t key_at(uint4 nd, uint32_t j) {
        uint32_t w = j < 4u ? (j < 2u ? nd.x : nd.y) : (j < 6u ? nd.z : nd.w);
        return (j & 1u) ? (w >> 16) : (w & 0xFFFFu);
    }

    // VoxelClusterStore::lookupVoxel / performBinarySearch (VoxelClusterStore.cuh:101-135):
    // the same search over the cluster's sorted keys, widened to one 16-B node
    // of 8 keys per level (9-ary): 1 node load for n <= 8, 2 for n <= 64, 3 for
    // n <= 512 instead of 1 + ~log2(n) dependent word loads.  Identical result.
    // CuckooHashTable::lookupVoxel (CuckooHashTable.cuh:59-76).
    __device__ __forceinline__ uint32_t lookup(uint32_t reg, Blk blk, int32_t x, int32_t y, int32_t z) {
        if (STORE == STORE_VCS) {
            const uint32_t n = blk.y;
            const VcsGeom gm = vcs_geom(n);
            const uint4* b = s.vcs_pool + blk.x;
            if (((uint32_t)x | (uint32_t)y | (uint32_t)z) >= 64u) return lookup_aliased(b, gm, n, x, y, z);
            const uint32_t q = (((uint32_t)x & 7u) << 6) | (((uint32_t)y & 7u) << 3) | ((uint32_t)z & 7u);
            uint32_t grp = 0, chunk = 0;
            if (gm.groups > 1u) {
                grp = count_lt(b[0], q);
                if (grp >= gm.groups) { count_bsearch(n, n, false); return kEmpty; }
            }
            if (gm.chunks > 1u) {
                const uint32_t cl = count_lt(b[gm.u_f1 + grp], q);
                const uint32_t in_grp = min(8u, gm.chunks - 8u * grp);
                if (cl >= in_grp) { count_bsearch(n, n, false); return kEmpty; }
                chunk = 8u * grp + cl;
            }
            const uint4 leaf = b[gm.u_keys + chunk];
            const uint32_t r = count_lt(leaf, q);
            const bool found = r < 8u && key_at(leaf, r) == q;
            count_bsearch(n, min(8u * chunk + r, n), found);
            if (!found) return kEmpty;
            return reinterpret_cast<const uint32_t*>(b + gm.u_vals)[8u * chunk + r];
        } else {
            const uint32_t key = ((uint32_t)x << 20) | ((uint32_t)y << 10) | (uint32_t)z;   // generate3DPoint
            uint4 m = s.ht_meta[reg];          // {base, M, prime, offset}
            uint32_t s1 = hash1(key, m.w) % m.y;
            count(4);
            uint2 e = s.ht_slots[m.x + s1];
            if (e.x == key) { count(4); return e.y; }
            uint32_t s2 = hash2(key, m.z) % m.y;
            count(4);
            e = s.ht_slots[m.x + m.y + s2];
            if (e.x == key) { count(4); return e.y; }
            return kEmpty;
        }
    }

    // applyLighting / applyDirectionalLightingToColor / applyPointLightingToColor
    // (Renderer.cuh:57-86,249-258), colour packing (VoxelFunctions.cuh:69-83).
    __device__ __forceinline__ uint32_t lighting(uint32_t col, f3 n, f3 rwp, f3 ro) const {
        f3 LC = ld3(v.LC);
        f3 c = mk((float)(col >> 16) / 255.0f, (float)((col >> 8) & 0xFFu) / 255.0f, (float)(col & 0xFFu) / 255.0f);
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

    // getNormalFromTValues (Renderer.cuh:237-247)
    __device__ __forceinline__ static f3 normal_from_t(float tX, float tY, float tZ, float tMin, f3 d) {
        if (tX == tMin) return mk(copysignf(1.0f, -d.x), 0.0f, 0.0f);
        if (tY == tMin) return mk(0.0f, copysignf(1.0f, -d.y), 0.0f);
        return mk(0.0f, 0.0f, copysignf(1.0f, -d.z));
    }

    __device__ __forceinline__ static bool in_region(f3 o) {               // Renderer.cuh:93-98
        return o.x >= 0.0f && o.x < 64.0f && o.y >= 0.0f && o.y < 64.0f && o.z >= 0.0f && o.z < 64.0f;
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
        float nx = d.x > 0.0f ? 64.0f + kEps : 0.0f - kEps;
        float ny = d.y > 0.0f ? 64.0f + kEps : 0.0f - kEps;
        float nz = d.z > 0.0f ? 64.0f + kEps : 0.0f - kEps;
        float tX, tY, tZ;
        if (GUARDED) {
            tX = d.x != 0.0f ? (nx - o.x) / d.x : kInf;
            tY = d.y != 0.0f ? (ny - o.y) / d.y : kInf;
            tZ = d.z != 0.0f ? (nz - o.z) / d.z : kInf;
        } else {
            tX = (nx - o.x) / d.x;
            tY = (ny - o.y) / d.y;
            tZ = (nz - o.z) / d.z;
        }
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
