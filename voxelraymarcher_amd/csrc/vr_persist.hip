// vr_persist.hip -- persistent, flattened ray-march kernel for gfx950.
//
// Why: rays of one 8x8 tile diverge (tile max/mean work ~2.1x on C2, see
// DESIGN.md), hit pixels walk a second (shadow) ray, and wave64 issues every
// loop iteration for all 64 lanes.  Here each lane runs a small state machine
// in which ONE loop iteration = ONE voxel probe of whatever the lane is doing:
//   P_REGION  region-table read + null-region skips + the walk's first step
//   P_DDA     one iteration of rayMarchVoxelGrid / shadowRayMarchVoxelGrid
//             (Renderer.cuh:282-332 / :122-168)
//   P_LA      one axis step of rayMarchVoxelGridLongestAxis (:787-909 / :522-625)
//   P_JUMP    one iteration of performVoxelSpaceJump (:705-729 / :449-473)
// Primary and shadow rays run through the same code (a per-lane flag picks
// the guarded divisions of the shadow walk), and a lane whose pixel is done
// fetches the next pixel from a global counter (wave-aggregated atomic), so
// waves stay full until the frame is drained.  Pixels are handed out in 8x8
// tile order so the lanes of a wave stay spatially coherent.
//
// Every loop iteration of the reference maps to exactly one state-machine
// step with the same iteration-budget tick and the same memory reads, so the
// pixels AND the algorithmic byte count equal the oracle's bit for bit.
#include "vr_device.h"

namespace vr {
namespace {

enum : uint32_t { P_REGION = 0, P_DDA = 1, P_LA = 2, P_JUMP = 3 };

template <int STORE, int ALGO, bool COUNT>
struct Machine : Ctx<STORE, COUNT> {
    using C = Ctx<STORE, COUNT>;
    using C::s; using C::v; using C::tick; using C::exists; using C::lookup; using C::lighting;
    using C::normal_from_t; using C::in_region; using C::grid_in_region; using C::advance_region;
    using C::in_scene; using C::region_at;

    // per-lane walk state
    f3 o, d;                 // region-local origin (the reference's localRay / originalRay) and direction
    i3 cr;                   // currentRegion
    uint32_t reg = kNone;
    float tX = 0.0f, tY = 0.0f, tZ = 0.0f, tMin = 0.0f;   // DDA t values (stale-normal semantics) / jump t values
    // longest-axis state (dead code for ALGO_ORIGINAL)
    f3 old_o, ray_o, ds;
    i3 g, ad;
    uint32_t L = 0, M = 0, S = 0;
    uint32_t queue = 0, qlen = 0;    // pending axis steps of the current LA iteration
    bool mid_floor = false, need_adv = false;
    // pixel state
    uint32_t lit = 0, result = 0, phase = P_REGION;
    bool shadow = false, shadow_la = false;

    __device__ Machine(const KScene& s_, const KView& v_) : C(s_, v_) {}

    __device__ __forceinline__ bool la() const { return shadow ? shadow_la : (ALGO == ALGO_LONGEST); }
    __device__ __forceinline__ static float gdiv(float n, float o_, float d_, bool guard) {
        float t = (n - o_) / d_;
        return (guard && d_ == 0.0f) ? kInf : t;
    }
    __device__ __forceinline__ f3 rwp() const {   // regionWorldPosition (Renderer.cuh:413)
        return add(ld3(v.translation), mk((float)(cr.x * kBlock), (float)(cr.y * kBlock), (float)(cr.z * kBlock)));
    }
    __device__ __forceinline__ int finish(uint32_t col) {
        result = col;
        return 1;
    }
    __device__ __forceinline__ int walk_miss() { return finish(shadow ? lit : 0u); }
    __device__ __forceinline__ int start_shadow(f3 so, bool la_walk) {
        if (!v.use_shadows) return finish(lit);      // isInShadow... returns false (Renderer.cuh:176-179)
        shadow = true;
        shadow_la = la_walk;
        o = so;
        d = ld3(v.L);
        phase = P_REGION;
        return 0;
    }

    // calculateWorldRay + entry clip of rayMarchVoxelScene (Renderer.cuh:1013-1022, 340-378).
    // Returns 1 if the pixel is already final (result set).
    __device__ int begin_pixel(uint32_t x, uint32_t y) {
        this->iters = 0;
        this->aborted = false;
        shadow = false;
        shadow_la = false;
        lit = 0;
        float u = ((float)x + 0.5f) / (float)v.W;
        float vv = ((float)(v.H - y) + 0.5f) / (float)v.H;
        f3 ro = add(add(ld3(v.llc), scl(u, ld3(v.hor))), scl(vv, ld3(v.ver)));
        f3 rd = unit(sub(ro, ld3(v.org)));
        f3 so = scl(v.scale_f, sub(ro, ld3(v.translation)));
        d = rd;
        cr = i3{f2i(floorf(so.x / 64.0f)), f2i(floorf(so.y / 64.0f)), f2i(floorf(so.z / 64.0f))};
        while (!in_scene(cr)) {
            if (!tick()) return finish(0);
            int32_t hi = (int32_t)(s.D + (uint32_t)s.min_coord), lo = s.min_coord;
            int32_t nx = d.x < 0.0f ? hi : lo, ny = d.y < 0.0f ? hi : lo, nz = d.z < 0.0f ? hi : lo;
            float eX = ((float)(nx * kBlock) - so.x) / d.x;
            float eY = ((float)(ny * kBlock) - so.y) / d.y;
            float eZ = ((float)(nz * kBlock) - so.z) / d.z;
            if (eX <= 0.0f) eX = kInf;
            if (eY <= 0.0f) eY = kInf;
            if (eZ <= 0.0f) eZ = kInf;
            float eMin = fminf(eX, fminf(eY, eZ));
            if (eMin == kInf) return finish(0);
            so = add(so, scl(eMin + kEps, d));
            cr = i3{f2i(floorf(so.x / 64.0f)), f2i(floorf(so.y / 64.0f)), f2i(floorf(so.z / 64.0f))};
        }
        o = sub(so, mk((float)(cr.x * kBlock), (float)(cr.y * kBlock), (float)(cr.z * kBlock)));
        phase = P_REGION;
        return 0;
    }

    // First step of rayMarchVoxelGrid (:263-280) / shadowRayMarchVoxelGrid (:103-120).
    __device__ __forceinline__ void grid_init() {
        const bool gd = shadow;
        float nX = d.x > 0.0f ? ceilf(o.x) + kEps : floorf(o.x) - kEps;
        float nY = d.y > 0.0f ? ceilf(o.y) + kEps : floorf(o.y) - kEps;
        float nZ = d.z > 0.0f ? ceilf(o.z) + kEps : floorf(o.z) - kEps;
        tX = gdiv(nX, o.x, d.x, gd);
        tY = gdiv(nY, o.y, d.y, gd);
        tZ = gdiv(nZ, o.z, d.z, gd);
        tMin = fminf(tX, fminf(tY, tZ));
        o = add(o, scl(tMin + kEps, d));
        phase = P_DDA;
    }

    // Prologue of rayMarchVoxelGridLongestAxis (:762-784) incl. Ray::convertRayToLongestAxisDirection.
    __device__ __forceinline__ void la_init() {
        float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z), k;
        if (ax > ay && ax > az) {
            L = 0; M = ay > az ? 1 : 2; S = ay > az ? 2 : 1; k = 1.0f / ax;
        } else if (ay > az) {
            L = 1; M = ax > az ? 0 : 2; S = ax > az ? 2 : 0; k = 1.0f / ay;
        } else {
            L = 2; M = ax > ay ? 0 : 1; S = ax > ay ? 1 : 0; k = 1.0f / az;
        }
        ds = scl(k, d);
        old_o = o;
        g = i3{f2i(o.x), f2i(o.y), f2i(o.z)};
        ad = i3{0, 0, 0};
        int32_t adL = comp(d, L) < 0.0f ? -1 : 1;
        seti(ad, L, adL);
        float gL = (float)geti(g, L), oL = comp(o, L);
        float t = adL > 0 ? (gL + kEps + 1.0f - oL) / (float)adL : (gL - kEps - oL) / (float)adL;
        ray_o = add(old_o, scl(t, ds));
        seti(ad, M, f2i(comp(ray_o, M)) - geti(g, M));
        seti(ad, S, f2i(comp(ray_o, S)) - geti(g, S));
        mid_floor = comp(ds, M) < 0.0f;
        qlen = 0;
        need_adv = false;
        phase = P_LA;
    }

    // P_REGION: top of the region loop (:381-410 / :182-211 / :641-670 / :957-986).
    __device__ int region_step() {
        if (!in_scene(cr)) return walk_miss();
        if (!tick()) return finish(0);
        reg = region_at(cr);
        while (reg == kNone) {
            if (!tick()) return finish(0);
            const bool gd = shadow && !shadow_la;   // only isInShadowOriginalRayMarch guards (:191-193)
            float nx = d.x > 0.0f ? 64.0f + kEps : 0.0f - kEps;
            float ny = d.y > 0.0f ? 64.0f + kEps : 0.0f - kEps;
            float nz = d.z > 0.0f ? 64.0f + kEps : 0.0f - kEps;
            float sx = gdiv(nx, o.x, d.x, gd), sy = gdiv(ny, o.y, d.y, gd), sz = gdiv(nz, o.z, d.z, gd);
            float sMin = fminf(sx, fminf(sy, sz));
            o = add(o, scl(sMin, d));
            advance_region(cr, o);
            if (!in_scene(cr)) return walk_miss();
            reg = region_at(cr);
        }
        if (ALGO == ALGO_LONGEST && la()) la_init();
        else grid_init();
        return 0;
    }

    // P_DDA: one iteration of the original DDA loop; the cluster skip
    // (:290-306) and the voxel step (:318-331) share one select-driven step
    // (see vr_march.hip grid_original).
    __device__ int dda_step() {
        if (!in_region(o)) {              // loop exit -> back in the region loop (:421-429)
            advance_region(cr, o);
            phase = P_REGION;
            return 0;
        }
        if (!tick()) return finish(0);
        const bool gd = shadow;
        const int32_t vx = f2i(o.x), vy = f2i(o.y), vz = f2i(o.z);
        const Blk blk = exists(reg, vx, vy, vz);
        const bool skip = absent(blk);
        if (!skip) {
            const uint32_t col = lookup(reg, blk, vx, vy, vz);
            if (col != kEmpty) {
                if (shadow) return finish(0);
                lit = lighting(col, normal_from_t(tX, tY, tZ, tMin, d), rwp(), o);
                return start_shadow(o, false);
            }
        }
        const bool px = d.x > 0.0f, py = d.y > 0.0f, pz = d.z > 0.0f;
        const float nX = skip ? (float)(px ? ((vx / 8) + 1) * 8 : (vx / 8) * 8) : (px ? ceilf(o.x) + kEps : floorf(o.x) - kEps);
        const float nY = skip ? (float)(py ? ((vy / 8) + 1) * 8 : (vy / 8) * 8) : (py ? ceilf(o.y) + kEps : floorf(o.y) - kEps);
        const float nZ = skip ? (float)(pz ? ((vz / 8) + 1) * 8 : (vz / 8) * 8) : (pz ? ceilf(o.z) + kEps : floorf(o.z) - kEps);
        const float sX = gdiv(nX, o.x, d.x, gd), sY = gdiv(nY, o.y, d.y, gd), sZ = gdiv(nZ, o.z, d.z, gd);
        const float sMin = fminf(sX, fminf(sY, sZ));
        if (!skip) { tX = sX; tY = sY; tZ = sZ; tMin = sMin; }
        o = add(o, scl(sMin + kEps, d));
        return 0;
    }

    // P_LA: one axis step of the longest-axis loop.
    __device__ int la_step() {
        if (qlen == 0) {
            if (need_adv) {               // end of a completed iteration (:903-908)
                old_o = ray_o;
                ray_o = add(ray_o, ds);
                seti(ad, M, f2i(comp(ray_o, M)) - geti(g, M));
                seti(ad, S, f2i(comp(ray_o, S)) - geti(g, S));
                need_adv = false;
            }
            if (!grid_in_region(geti(g, L) + geti(ad, L), geti(g, M) + geti(ad, M), geti(g, S) + geti(ad, S))) {
                o = old_o;                // :911-914 -> original DDA for the rest of the region
                grid_init();
                return 0;
            }
            if (!tick()) return finish(0);
            int32_t adM = geti(ad, M), adS = geti(ad, S);
            if (adS != 0 && adM != 0) {   // :792-805
                float om = comp(old_o, M);
                float t1 = ((mid_floor ? floorf(om) : ceilf(om)) - om) / comp(ds, M);
                float sp = comp(old_o, S) + comp(ds, S) * t1;
                int32_t sd = f2i(floorf(sp)) - geti(g, S);
                uint32_t a0 = sd != 0 ? S : M, a1 = sd != 0 ? M : S;
                queue = a0 | (a1 << 2) | (L << 4);
                qlen = 3;
            } else if (adM != 0) {
                queue = M | (L << 2);
                qlen = 2;
            } else if (adS != 0) {
                queue = S | (L << 2);
                qlen = 2;
            } else {
                queue = L;
                qlen = 1;
            }
        }
        const uint32_t axis = queue & 3u;
        queue >>= 2;
        --qlen;
        seti(g, axis, geti(g, axis) + geti(ad, axis));
        Blk blk = exists(reg, g.x, g.y, g.z);
        if (absent(blk)) {               // -> performVoxelSpaceJump
            tX = tY = tZ = tMin = 0.0f;
            qlen = 0;
            phase = P_JUMP;
            return 0;
        }
        uint32_t col = lookup(reg, blk, g.x, g.y, g.z);
        if (col != kEmpty) {
            if (shadow) return finish(0);
            f3 n = mk(0.0f, 0.0f, 0.0f);
            setf(n, axis, copysignf(1.0f, -comp(ds, axis)));
            f3 hit;
            if (axis == L) {
                hit = ray_o;              // :897-900
            } else {                      // getLocalHitLocation (:753-758)
                float oa = comp(old_o, axis), da = comp(ds, axis);
                float t = da > 0.0f ? (ceilf(oa) - oa) / da : (floorf(oa) - oa) / da;
                hit = add(old_o, scl(t, ds));
            }
            lit = lighting(col, n, rwp(), hit);
            return start_shadow(hit, true);
        }
        if (qlen == 0) need_adv = true;
        return 0;
    }

    // P_JUMP: one iteration of performVoxelSpaceJump's `while (!doesVoxelSpaceExist)`.
    __device__ int jump_step() {
        Blk blk = exists(reg, g.x, g.y, g.z);
        if (absent(blk)) {
            if (!tick()) return finish(0);
            int32_t nx = ds.x > 0.0f ? ((g.x / 8) + 1) * 8 : (g.x / 8) * 8;
            int32_t ny = ds.y > 0.0f ? ((g.y / 8) + 1) * 8 : (g.y / 8) * 8;
            int32_t nz = ds.z > 0.0f ? ((g.z / 8) + 1) * 8 : (g.z / 8) * 8;
            tX = ((float)nx - old_o.x) / ds.x;
            tY = ((float)ny - old_o.y) / ds.y;
            tZ = ((float)nz - old_o.z) / ds.z;
            tMin = fminf(tX, fminf(tY, tZ)) + kEps;
            old_o = add(old_o, scl(tMin, ds));
            g = i3{f2i(floorf(old_o.x)), f2i(floorf(old_o.y)), f2i(floorf(old_o.z))};
            if (!grid_in_region(g.x, g.y, g.z)) {   // left the region: EMPTY_VAL, originalRay = oldRay.o
                o = old_o;
                advance_region(cr, o);
                phase = P_REGION;
            }
            return 0;
        }
        uint32_t col = lookup(reg, blk, g.x, g.y, g.z);
        if (col != kEmpty) {
            if (shadow) return finish(0);
            lit = lighting(col, normal_from_t(tX, tY, tZ, tMin, ds), rwp(), old_o);
            return start_shadow(old_o, true);
        }
        float oL = comp(old_o, L), dL = comp(ds, L);
        float tNext = dL > 0.0f ? (ceilf(oL) - oL) / dL : (floorf(oL) - oL) / dL;
        ray_o = add(old_o, scl(tNext + kEps, ds));
        seti(ad, M, f2i(comp(ray_o, M)) - geti(g, M));
        seti(ad, S, f2i(comp(ray_o, S)) - geti(g, S));
        phase = P_LA;                     // CONTINUE_VAL: next iteration, no advance
        qlen = 0;
        need_adv = false;
        return 0;
    }

    __device__ __forceinline__ int step() {
        if (phase == P_DDA) return dda_step();
        if (ALGO == ALGO_LONGEST) {
            if (phase == P_LA) return la_step();
            if (phase == P_JUMP) return jump_step();
        }
        return region_step();
    }
};

// Work distribution: the frame's 8x8 tiles are split into kShards contiguous
// stripes; workgroup b starts on stripe b % 8 (workgroups b and b+8 share an
// XCD under round-robin placement -- speed only, never correctness) and
// steals from the other stripes when its own is drained.  A wave fetches one
// whole tile (64 pixels) per atomic into a wave-local pool; lanes whose
// pixel is done take the next pixel of the pool.  queue[kHeadStride * s] is
// stripe s's head (zeroed by the host before the launch).
constexpr uint32_t kShards = 8;
constexpr uint32_t kHeadStride = 64;     // one head per 256-B line

template <int STORE, int ALGO, bool COUNT>
__global__ __launch_bounds__(256) void persist_kernel(KScene s, KView v, uint32_t* __restrict__ queue) {
    Machine<STORE, ALGO, COUNT> m(s, v);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t tiles_x = (v.W + 7u) / 8u;
    const uint32_t ntiles = tiles_x * ((v.local_rows + 7u) / 8u);
    const uint32_t home = blockIdx.x % kShards;
    bool has = false, wave_live = true;
    uint32_t out_idx = 0;
    uint32_t pool_next = 0, pool_end = 0;      // wave-uniform pixel range
    uint32_t shard = home;
    // Wave-level scheduling: every iteration runs exactly ONE kind of step for
    // the lanes in that state (refill, region, DDA, LA, jump), so a wave never
    // pays for several divergent code blocks in one iteration.  Idle lanes are
    // refilled in batches of >= kRefillBatch (or when nothing else is left).
    constexpr uint32_t kRefillBatch = 16;
    for (;;) {
        const uint64_t m_has = __ballot(has);
        const uint64_t m_need = __ballot(wave_live && !has);
        if (!m_has && !m_need) break;
        uint32_t kind;                                    // wave-uniform
        if (m_need && (!m_has || (uint32_t)__popcll(m_need) >= kRefillBatch)) {
            kind = 0xFFu;
        } else {
            uint32_t best = P_DDA, nbest = (uint32_t)__popcll(__ballot(has && m.phase == P_DDA));
            const uint32_t nreg = (uint32_t)__popcll(__ballot(has && m.phase == P_REGION));
            if (nreg > nbest) { best = P_REGION; nbest = nreg; }
            if (ALGO == ALGO_LONGEST) {
                const uint32_t nla = (uint32_t)__popcll(__ballot(has && m.phase == P_LA));
                if (nla > nbest) { best = P_LA; nbest = nla; }
                const uint32_t nj = (uint32_t)__popcll(__ballot(has && m.phase == P_JUMP));
                if (nj > nbest) { best = P_JUMP; nbest = nj; }
            }
            kind = best;
        }
        if (kind == 0xFFu) {
            for (;;) {   // refill lanes without a pixel
                const bool need = wave_live && !has;
                const uint64_t mask = __ballot(need);
                if (mask == 0) break;
                if (pool_next == pool_end) {
                    uint32_t got = 0xFFFFFFFFu;
                    if (lane == 0) {
                        for (uint32_t k = 0; k < kShards; ++k) {
                            const uint32_t sh = (shard + k) % kShards;
                            const uint32_t t0 = (uint32_t)(((uint64_t)ntiles * sh) / kShards);
                            const uint32_t t1 = (uint32_t)(((uint64_t)ntiles * (sh + 1)) / kShards);
                            uint32_t* head = queue + kHeadStride * sh;
                            if (__hip_atomic_load(head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= t1 - t0) continue;
                            const uint32_t t = t0 + atomicAdd(head, 1u);
                            if (t < t1) { got = t; shard = sh; break; }
                        }
                    }
                    got = __builtin_amdgcn_readfirstlane(got);
                    shard = __builtin_amdgcn_readfirstlane(shard);
                    if (got == 0xFFFFFFFFu) { wave_live = false; break; }
                    pool_next = got * 64u;
                    pool_end = pool_next + 64u;
                }
                const uint32_t avail = pool_end - pool_next;
                const uint32_t rank = (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
                if (need && rank < avail) {
                    const uint32_t idx = pool_next + rank;
                    const uint32_t t = idx >> 6, w = idx & 63u;
                    const uint32_t x = (t % tiles_x) * 8u + (w & 7u), l = (t / tiles_x) * 8u + (w >> 3);
                    if (x < v.W && l < v.local_rows) {
                        out_idx = l * v.W + x;
                        const uint32_t band = l / v.band_rows;
                        const uint32_t y = v.row0 + (band * v.nranks + v.rank) * v.band_rows + (l - band * v.band_rows);
                        if (y >= v.row_limit) {
                            v.out[out_idx] = 0u;
                        } else if (m.begin_pixel(x, y)) {
                            v.out[out_idx] = m.aborted ? 0u : m.result;
                            m.count(4);
                        } else {
                            has = true;
                        }
                    }
                }
                const uint32_t n = (uint32_t)__popcll(mask);
                pool_next += n < avail ? n : avail;
            }
            continue;
        }
        if (has && m.phase == kind) {
            int r;
            if (kind == P_DDA) r = m.dda_step();
            else if (ALGO == ALGO_LONGEST && kind == P_LA) r = m.la_step();
            else if (ALGO == ALGO_LONGEST && kind == P_JUMP) r = m.jump_step();
            else r = m.region_step();
            if (r) {
                v.out[out_idx] = m.aborted ? 0u : m.result;
                m.count(4);
                has = false;
            }
        }
    }
    if (COUNT) {
        unsigned long long b = m.bytes;
        for (int off = 32; off > 0; off >>= 1) b += __shfl_down(b, off, 64);
        if (lane == 0 && b) atomicAdd(v.bytes, b);
    }
}

template <int STORE, int ALGO, bool COUNT>
hipError_t launch_one(const KScene& s, const KView& v, uint32_t* queue, hipStream_t stream) {
    static int blocks_per_cu[64] = {0};
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return hipErrorNoDevice;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    if (!blocks_per_cu[dev]) {
        int nb = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, persist_kernel<STORE, ALGO, COUNT>, 256, 0);
        if (e != hipSuccess) return e;
        hipDeviceProp_t prop;
        e = hipGetDeviceProperties(&prop, dev);
        if (e != hipSuccess) return e;
        cus[dev] = prop.multiProcessorCount;
        blocks_per_cu[dev] = nb > 0 ? nb : 1;
    }
    const uint64_t tiles = (uint64_t)((v.W + 7u) / 8u) * ((v.local_rows + 7u) / 8u);
    uint64_t grid = (uint64_t)blocks_per_cu[dev] * (uint64_t)cus[dev];
    const uint64_t need = (tiles + 3u) / 4u;      // 4 waves per block, >= 1 tile each
    if (grid > need) grid = need;
    if (grid == 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(queue, 0, kShards * kHeadStride * sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((persist_kernel<STORE, ALGO, COUNT>), dim3((unsigned)grid), dim3(256), 0, stream, s, v, queue);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_persist(int store, int algo, bool count, const KScene& s, const KView& v, uint32_t* queue,
                          hipStream_t stream) {
    if (store == STORE_VCS) {
        if (algo == ALGO_ORIGINAL)
            return count ? launch_one<STORE_VCS, ALGO_ORIGINAL, true>(s, v, queue, stream)
                         : launch_one<STORE_VCS, ALGO_ORIGINAL, false>(s, v, queue, stream);
        return count ? launch_one<STORE_VCS, ALGO_LONGEST, true>(s, v, queue, stream)
                     : launch_one<STORE_VCS, ALGO_LONGEST, false>(s, v, queue, stream);
    }
    if (algo == ALGO_ORIGINAL)
        return count ? launch_one<STORE_HASH, ALGO_ORIGINAL, true>(s, v, queue, stream)
                     : launch_one<STORE_HASH, ALGO_ORIGINAL, false>(s, v, queue, stream);
    return count ? launch_one<STORE_HASH, ALGO_LONGEST, true>(s, v, queue, stream)
                 : launch_one<STORE_HASH, ALGO_LONGEST, false>(s, v, queue, stream);
}

}  // namespace vr
