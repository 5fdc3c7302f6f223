// vr_march.hip -- the per-pixel voxel ray march for gfx950 (CDNA4).
//
// One lane per pixel; one wave64 = one 8x8 pixel tile (the reference's 8x8
// CUDA block, Main.cu:109-111, but as a single wavefront so the tile's rays
// walk the same clusters together), two waves (tiles side by side) per
// 128-thread workgroup (kTilesX/kTilesY below).  Templated on {store, algorithm, count}: no virtual calls, no
// function pointers (the reference's StorageStructure vtable,
// StorageStructure.cuh:12-56, and nextXFunc pointers, Renderer.cuh:263-265,
// become compile-time branches).
//
// Arithmetic follows the reference expression by expression (file:line in
// each function) under the FP policy of SURVEY.md 8(c): -ffp-contract=off,
// correctly rounded '/' and sqrtf, fminf/fmaxf, truncating saturating
// float->int with NaN -> 0, wrapping int arithmetic (-fwrapv).  The
// shadow ray of a hit is evaluated after the primary walk returns instead of
// from inside it (Renderer.cuh:315,737,821,...): the shadow result depends
// only on (hit origin, region, shadow algorithm), so the pixel is identical.
#include "vr_device.h"

#include <algorithm>
#include <type_traits>

// VR_DIAG (profiling builds only, profiles/wave_counts.py): wave-level execution
// counters -- one atomic per wave per counted event, from the wave's first
// active lane.  Never part of the library build.
#ifdef VR_CRAWL_PROF
// per crawl record of the last crawl pass (profiles/crawl_prof.py): {shader cycles, plain
// loop iterations (bit 31: walked from the start), crawl_run calls that applied steps, their
// loop trips, start and end (s_memrealtime, 100 MHz), 0, 0}
__device__ unsigned int g_vr_crawl_prof[16384 * 8];
#endif
#ifdef VR_DIAG
__device__ unsigned long long g_vr_diag[32];
#define VR_DIAG_COUNT(k)                                                              \
    do {                                                                             \
        if (__lane_id() == (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec())) \
            atomicAdd(&g_vr_diag[(k)], 1ull);                                        \
    } while (0)
#define VR_DIAG_COUNT_IF(c, k)                                  \
    do {                                                       \
        if (__builtin_amdgcn_ballot_w64(c) != 0) VR_DIAG_COUNT(k); \
    } while (0)
#else
#define VR_DIAG_COUNT(k) do { } while (0)
#define VR_DIAG_COUNT_IF(c, k) do { } while (0)
#endif

namespace vr {
namespace {

// Exact fast-forward of a cluster-skip crawl (rayMarchVoxelGrid's skip branch,
// Renderer.cuh:290-306, with tMin = +-0).  An iteration started in an absent
// cluster, found t = 0 on an axis whose skip plane is the position itself and
// moved to `on` = o + RN(EPSILON * d) componentwise.  While the positions stay
// in that cluster and, per axis, in one binade, every further iteration is the
// same skip: t = 0 on the same (unmoved) axis -- every other t is >= 0 -- and
// o_i <- RN(o_i + c_i), c_i = RN(EPSILON * d_i), i.e. o_i += delta_i, a fixed
// multiple of the binade's ulp (for a tie c_i / ulp = k + 1/2 only from an even
// mantissa, where every step lands on an even mantissa again).  Returns the number
// m of such iterations (0 = none, at most `room`) and the per-axis deltas; the
// caller credits m loop iterations and m existence reads.
struct Crawl { uint32_t m; float dx, dy, dz; };
// One axis: returns false to decline; else sets its delta, ORs in whether it is
// pinned on its skip plane, and lowers m to a number of iterations its binade and
// the cluster certainly allow (the float quotients are shrunk by 2^-20, so m may
// come out a little low -- the walk then simply runs those iterations -- never high).
__device__ __forceinline__ float crawl_floor(float num, float den) {
    return floorf(num * __builtin_amdgcn_rcpf(den) * (1.0f - 0x1p-20f));
}
__device__ __forceinline__ bool crawl_axis(float x, float dir, int32_t v, bool pos, float& delta, bool& pinned,
                                           float& m) {
    const float c = kEps * dir, nx = x + c;
    const float cl = (float)(v & ~7);                                           // cluster [cl, cl + 8)
    if (nx == x) {
        delta = 0.0f;
        pinned |= !pos && cl == x;
        return true;
    }
    if (!(x >= 0x1p-100f)) return false;     // zero / tiny coordinate: no binade arithmetic
    const uint32_t bits = __float_as_uint(x), be = bits >> 23;                  // x > 0: biased exponent
    const float lo = __uint_as_float(be << 23), hi = __uint_as_float((be + 1u) << 23);
    if (!(nx >= lo && nx < hi)) return false;
    const float x1 = __uint_as_float(bits + 1u), x2 = __uint_as_float(bits + 2u);
    delta = nx - x;                           // exact (same binade)
    if (!(x2 < hi)) return false;
    if ((x1 + c) - x1 != delta) {
        // c / ulp = k + 1/2: ties-to-even makes every result's mantissa even, so
        // from an even mantissa the step is constant (checked on the next even one).
        if ((bits & 1u) || (x2 + c) - x2 != delta) return false;
    }
    // positions x + t*delta: t = 0..m inside [lo, hi), t = 0..m-1 inside [cl, cl + 8)
    m = delta > 0.0f ? fminf(m, fminf(crawl_floor(hi - x, delta), crawl_floor(cl + 8.0f - x, delta)))
                     : fminf(m, fminf(crawl_floor(x - lo, -delta), crawl_floor(x - cl, -delta)));
    return true;
}
__device__ __forceinline__ Crawl crawl_steps(f3 on, f3 d, int32_t vx, int32_t vy, int32_t vz,
                                             bool px, bool py, bool pz, uint32_t room) {
    Crawl r{0u, 0.0f, 0.0f, 0.0f};
    if (((f2i(on.x) ^ vx) | (f2i(on.y) ^ vy) | (f2i(on.z) ^ vz)) & ~7) return r;   // left the cluster
    if (!(on.x >= 0.0f && on.y >= 0.0f && on.z >= 0.0f)) return r;
    bool pinned = false;
    float m = (float)room;
    f3 dl{0.0f, 0.0f, 0.0f};
    // (crawl kernel only: its register budget is not the tile pass's, so the axes are
    // unrolled -- VR_CRAWL_ROLLED keeps the rolled loop for A/B)
#ifdef VR_CRAWL_ROLLED
#pragma unroll 1
#else
#pragma unroll
#endif
    for (uint32_t a = 0; a < 3u; ++a) {
        float delta;
        if (!crawl_axis(comp(on, a), comp(d, a), a == 0 ? vx : (a == 1 ? vy : vz), a == 0 ? px : (a == 1 ? py : pz),
                        delta, pinned, m))
            return r;
        setf(dl, a, delta);
    }
    r.m = (pinned && m > 0.0f) ? (uint32_t)m : 0u;
    r.dx = dl.x; r.dy = dl.y; r.dz = dl.z;
    return r;
}

// A whole crawl (crawl pass): from `o` -- the position a crawl iteration stepped to from
// voxel q -- apply every further crawl iteration: runs of identical steps in one binade
// at once (crawl_steps), and the steps between runs (across a binade edge, a tie from an
// odd mantissa) one by one, exactly as the walk computes them, o_i + RN(EPSILON * d_i).
// Returns their number (0: not a crawl); at most `room`.  Pure arithmetic: a crawl of
// 10^5..10^6 iterations costs a few dozen loop trips instead of as many dependent mask
// loads.
//   lbm == null (performVoxelSpaceJump's crawls): only the iterations whose results stay
// in q's cluster; the step that leaves it is left to the walk (the jump's hit normal
// reads its t values).
//   lbm (the original DDA's crawls, whose skip steps feed no normal: Renderer.cuh:297-301,
// SURVEY Q8): the region's cluster-existence bits.  A crawl does not end at its cluster's
// face: an iteration that starts in an ABSENT cluster with the pinned axis still on its
// plane (it never moves; the next cluster on the other axes shares that plane) is again a
// skip with t = +-0 -- the same step.  So the crossing step is taken here as well, and
// the crawl goes on through every absent cluster the ray meets in the region; it stops
// after the step into a present cluster or out of the region (the walk resumes there).
// Without this, each face crossing returned to the walk loop, which re-armed crawl
// detection only after 8 single-step iterations: ~10-35 crossings per C5 record.
__device__ __forceinline__ uint32_t crawl_run(f3& o, f3 d, int32_t qx, int32_t qy, int32_t qz, bool px, bool py,
                                              bool pz, uint32_t room, const uint32_t* lbm = nullptr,
                                              uint32_t* trips = nullptr) {
    const f3 c{kEps * d.x, kEps * d.y, kEps * d.z};
    int32_t lx = qx & ~7, ly = qy & ~7, lz = qz & ~7;
    // an axis pinned on its cluster plane: direction negative, on the plane, unmoved by its step
    const bool pinned = (!px && (float)lx == o.x && o.x + c.x == o.x) ||
                        (!py && (float)ly == o.y && o.y + c.y == o.y) ||
                        (!pz && (float)lz == o.z && o.z + c.z == o.z);
    if (!pinned) return 0u;
    auto inside = [&](f3 p) {   // in the cluster [l, l + 8) on every axis (p >= 0: trunc = floor)
        return p.x >= (float)lx && p.x < (float)(lx + 8) && p.y >= (float)ly && p.y < (float)(ly + 8) &&
               p.z >= (float)lz && p.z < (float)(lz + 8);
    };
    // p left the current cluster: go on crawling in p's cluster when it is in the region and absent
    auto absent_next = [&](f3 p) -> bool {
        if (!lbm || !(p.x >= 0.0f && p.x < 64.0f && p.y >= 0.0f && p.y < 64.0f && p.z >= 0.0f && p.z < 64.0f))
            return false;
        const int32_t ax = f2i(p.x), ay = f2i(p.y), az = f2i(p.z);
        const uint32_t slot = (uint32_t)(((az >> 3) << 6) | ((ay >> 3) << 3) | (ax >> 3));
        if ((lbm[slot >> 5] >> (slot & 31u)) & 1u) return false;
        qx = ax; qy = ay; qz = az;
        lx = ax & ~7; ly = ay & ~7; lz = az & ~7;
        return true;
    };
    if (!inside(o) && !absent_next(o)) return 0u;   // the crawl iteration itself left the cluster
    uint32_t n = 0;
#pragma unroll 1
    for (uint32_t trip = 0; trip < 65536u && n < room; ++trip) {
        if (trips) ++*trips;
        const Crawl cw = crawl_steps(o, d, qx, qy, qz, px, py, pz, room - n);
        if (cw.m != 0u) {
            const float fm = (float)cw.m;       // exact: m * delta_i stays inside the binade
            o = f3{o.x + fm * cw.dx, o.y + fm * cw.dy, o.z + fm * cw.dz};
            n += cw.m;
            if (n >= room) break;
        }
        const f3 o1{o.x + c.x, o.y + c.y, o.z + c.z};
        if (!inside(o1)) {
            if (!lbm) break;
            o = o1;                             // the crossing step (a skip in an absent cluster)
            ++n;
            if (!absent_next(o1)) break;
            continue;
        }
        o = o1;
        ++n;
    }
    return n;
}

// Direction-sign specialisation of the VCS loop: S = +1 / -1 a sign every lane
// of the wave shares, 0 = per lane.  plane_v is px ? ceilf(o) + EPSILON :
// floorf(o) - EPSILON (next_plane_fma's value); plane_c8 the cluster-skip offset.
template <int S> struct Sgn { static constexpr int value = S; };
template <int S>
__device__ __forceinline__ float plane_v(float o, float g, float ge) {
    if constexpr (S > 0) return ceilf(o) + kEps;
    else if constexpr (S < 0) return floorf(o) - kEps;
    else return next_plane_fma(o, g, ge);
}
template <int S>
__device__ __forceinline__ int32_t plane_c8(int32_t c8) {
    if constexpr (S > 0) return 8;
    else if constexpr (S < 0) return 0;
    else return c8;
}

// A crawl iteration has t = 0, so it stepped o_i <- RN(o_i + c_i), c_i =
// RN(EPSILON d_i); its voxel is q_i = trunc(old o_i), old o_i >= 0 (it was in
// the region).  The old coordinate lies within ulp(on)/2 + ulp(e)/2 of
// e = RN(on - c) (< 1.5 ulp(e) for e >= 1), so it is one of the floats at most 4
// steps from e that step to `on`: q is found when all of those truncate alike.
__device__ __forceinline__ bool crawl_voxel(float on, float c, int32_t& q) {
    const float e = on - c;
    if (e + 0x1p-20f < 1.0f) { q = 0; return true; }          // every candidate in [0, 1)
    int32_t found = -1;
    bool ok = true;
#pragma unroll 1
    for (int32_t k = -4; k <= 4; ++k) {
        const float x = __uint_as_float(__float_as_uint(e) + (uint32_t)k);
        if (!(x >= 0.0f) || x + c != on) continue;
        const int32_t t = f2i(x);
        ok &= found < 0 || t == found;
        found = t;
    }
    q = found;
    return ok && found >= 0;
}

// Tile pass workgroup: kTilesX x kTilesY waves, one 8x8 pixel tile each.  Two
// tiles side by side (128 threads) measured faster than 2 x 2 (256): a
// workgroup's slot is held until its slowest wave ends, so smaller ones pack the
// CUs more tightly (per frame in flight: C2 0.151 -> 0.1415 ms, C3 0.420 -> 0.385,
// C4 0.101 -> 0.096; one tile per workgroup: C2 0.1423, C3 0.377, C4 0.0955).
#ifndef VR_TILES_X
#define VR_TILES_X 2
#endif
#ifndef VR_TILES_Y
#define VR_TILES_Y 1
#endif
constexpr uint32_t kTilesX = VR_TILES_X, kTilesY = VR_TILES_Y;
// VR_UNIFORM_SKIP: the cluster-skip planes and their selects are computed only in
// wave-iterations where some lane stands in an absent cluster (one uniform branch on
// the ballot).  In C2, 61 % of the primary and 60 % of the shadow wave-iterations
// have no skipping lane (VR_DIAG counters 22-25, profiles/r02/wave_counts_C2_skip.txt):
// those run 51 VALU instead of 61.  C2 0.1172 -> 0.1113 ms per frame in flight,
// identical pixels; C5 (sparse: mostly skips) 0.688 -> 0.697 (profiles/r02/ab_uniform_skip_*.txt).
// A three-way form (voxel planes only when some lane does not skip, so they wait for the
// load) measured slower: C2 0.1112 -> 0.1147, C5 0.688 -> 0.694 (ab_uniform_skip3_*.txt).
#ifndef VR_UNIFORM_SKIP
#define VR_UNIFORM_SKIP 1
#endif
#ifndef VR_LONG_TAIL_GENERIC
#define VR_LONG_TAIL_GENERIC false
#endif
// VR_LONG_TAIL_EQ: the original-DDA tail of a longest-axis shadow walk takes the
// one-division loop when the light's components are equal (as the original
// algorithm's shadow walks do).  Measured neutral on C3 (0.2722 vs 0.2736 ms alone,
// profiles/r03/ab_la_signs_unit_C3.txt): off, the tail stays one loop.
#ifndef VR_LONG_TAIL_EQ
#define VR_LONG_TAIL_EQ 0
#endif

// The iteration count of a tile-pass walk that wrote a crawl record (see the deferral
// in grid_original_rt): the pixel is the crawl pass's already.
constexpr uint32_t kDeferredIters = 0xFFFFFFFFu;

// A tile-pass lane that defers its pixel tells the host, through the launch slot's
// host-mapped report word (KView::slot_stat): {launch id, 1}.  On a launch that runs its
// crawl pass the pass overwrites it with its own count.  On a launch whose crawl pass the
// host skipped -- believing the view defers nothing -- it is the only writer, and the host
// stops skipping when it sees it (vr_host.cpp launch): the next launch of the slot runs the
// crawl pass, which drops the stale records and resets the list.  (Rare: one 8-B store.)
__device__ __forceinline__ void deferral_report(const KView& v) {
    if (v.slot_stat) *reinterpret_cast<uint2*>(v.slot_stat) = uint2{v.launch_id, 1u};
}

// The tile group (column, row of kTilesX x kTilesY tiles) this tile-pass workgroup
// renders: the work order's entry (heaviest first, KView::order), or its grid position
// (a uniform load: SGPRs).
__device__ __forceinline__ void tile_group(const KView& v, uint32_t& bx, uint32_t& by) {
    bx = blockIdx.x;
    by = blockIdx.y;
    if (v.order) {
        const uint32_t t = v.order[blockIdx.y * gridDim.x + blockIdx.x];
        bx = t & 0xFFFFu;
        by = t >> 16;
    }
}

// The pixel (local column x, local row l) of this tile-pass lane.  Without a lane order
// (KView::perm null) wave w of tile group (bx, by) is the 8x8 tile (2 bx + w, by).  With one,
// the tile groups of a kLaneBlock x kLaneBlock pixel block share its pixels: they are dealt
// to the block's waves heaviest first (perm_kernel, from the walk lengths an earlier launch
// of the view recorded), so a wave's lanes walk about equally far and finish together --
// 16x16 blocks, C2: 24 % fewer wave-iterations for the same per-lane work (the oracle's
// per-pixel counts, profiles/r05/lane_sort_sim.py, lane_order/).  Slot q of a block is wave
// w of its tile group (bx mod kLbX, by mod kLbY) in row-major order, q = 2 (tile group) + w;
// lane i of slot q renders pixel perm[block * kLanePixels + 64 q + i] = (row * kLaneBlock +
// column) of the block.  Blocks cut by the grid's edge keep the 8x8 tiles.
#ifndef VR_LANE_BLOCK
#define VR_LANE_BLOCK 16
#endif
constexpr uint32_t kLaneBlock = VR_LANE_BLOCK;
static_assert(kLaneBlock == 16 || kLaneBlock == 32, "lane block: 16 or 32 pixels");
constexpr uint32_t kLanePixels = kLaneBlock * kLaneBlock;
constexpr uint32_t kLbX = kLaneBlock / (8u * kTilesX), kLbY = kLaneBlock / (8u * kTilesY);
using PermT = std::conditional<kLaneBlock == 16, uint8_t, uint16_t>::type;
constexpr bool kLaneOrder = kTilesX == 2 && kTilesY == 1;   // (other tile shapes ignore perm)
__device__ __forceinline__ void lane_pixel(const KView& v, uint32_t& x, uint32_t& l) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t bx, by;
    tile_group(v, bx, by);
    const uint32_t BX = bx / kLbX, BY = by / kLbY;
    if (kLaneOrder && v.perm && (BX + 1u) * kLbX <= gridDim.x && (BY + 1u) * kLbY <= gridDim.y) {
        const uint32_t q = ((by % kLbY) * kLbX + bx % kLbX) * kTilesX + wave;
        const uint32_t blk = BY * ((gridDim.x + kLbX - 1u) / kLbX) + BX;
        const uint32_t p = reinterpret_cast<const PermT*>(v.perm)[(size_t)blk * kLanePixels + q * 64u + lane];
        x = BX * kLaneBlock + p % kLaneBlock;
        l = BY * kLaneBlock + p / kLaneBlock;
    } else {
        x = (bx * kTilesX + wave % kTilesX) * 8u + (lane & 7u);
        l = (by * kTilesY + wave / kTilesX) * 8u + (lane >> 3);
    }
}

// The tile pass's pixels by thread, (l << 16 | x), written once by march_kernel: a deferral
// deep in the walk reads its pixel back with one LDS load instead of keeping it live or
// recomputing it from the work and lane orders (two dependent global loads).
__device__ __forceinline__ uint32_t* tile_pixels() {
    __shared__ uint32_t p[64u * kTilesX * kTilesY];
    return p;
}

// The primary walk's length per tile-pass thread, for a launch that records the lane order's
// walk lengths (KView::pcost): shade writes it between the walks, march_kernel reads it back.
__device__ __forceinline__ uint32_t* tile_prim() {
    __shared__ uint32_t p[64u * kTilesX * kTilesY];
    return p;
}

// CRAWL: fast-forward cluster-skip crawls (the deferred-ray pass); otherwise a
// crawling ray reserves an entry in the launch's deferral list and unwinds.
// kExact (the crawl pass): every walk runs to its end here, and a loop round that
// leaves its state unchanged is detected as a walk that never finishes.  Otherwise
// (the tile pass) a walk past kTileBudget iterations is handed to the crawl pass.
// (Making the cuckoo store's tile pass exact instead -- it has no cluster skips, so
// no crawls, and could do without a crawl pass -- keeps the round-state snapshot live
// through its walk loop: C4 0.085 -> 0.109 ms per frame, profiles/r03/ab_exact_cuckoo.txt.)
template <int STORE, bool CRAWL>
struct ExactWalk { static constexpr bool value = CRAWL; };
template <int STORE, bool COUNT, bool CRAWL>
struct Walker : Ctx<STORE, COUNT, ExactWalk<STORE, CRAWL>::value ? kCrawlBudget : kTileBudget> {
    using C = Ctx<STORE, COUNT, ExactWalk<STORE, CRAWL>::value ? kCrawlBudget : kTileBudget>;
    static constexpr bool kExact = ExactWalk<STORE, CRAWL>::value;
    static constexpr uint32_t kBudget = C::kBudget;
    using C::s; using C::v; using C::aborted; using C::tick; using C::exists; using C::lookup;
    using C::lighting; using C::normal_from_t; using C::in_region; using C::grid_in_region;
    using C::advance_region; using C::in_scene; using C::region_at; using C::skip_null; using C::bytes;
    __device__ Walker(const KScene& s_, const KView& v_) : C(s_, v_) {}
    // Per-ray reciprocals for the entry clip and each region walk's initial step
    // (div_fast instead of IEEE division): cuckoo C4 -2.5 %, but the VCS walks'
    // kernel runs at its 72-VGPR limit and the longer-lived values cost spills
    // there (C2 +1.6 %, C3 +4 %), so VCS keeps the plain divisions.
    static constexpr bool kFastSetup = STORE == STORE_HASH;
    // VR_LONG_REMAT (the VCS longest-axis tile pass): see primary_regions
#ifndef VR_LONG_REMAT
#define VR_LONG_REMAT 1
#endif
    static constexpr bool kRematDir = VR_LONG_REMAT && STORE == STORE_VCS && !CRAWL;
    // what a deferred crawl must know to be resumed (see the deferral below):
    // bit 1 = the shadow walk is the longest-axis one; the lit colour of the hit
    uint32_t ctx = 0, lit_saved = 0;
    // Crawl pass (VCS): this lane's LDS copy of the cluster-existence bits of region
    // bm_reg (KScene::vcs_cbits, 16 words), or null.  A crawl record's remaining walk
    // -- up to ~280 iterations, mostly cluster skips through C5's empty clusters, each
    // a dependent mask load from MALL/HBM -- then loads a mask word only in present
    // clusters: a skip step reads one LDS word instead.
    uint32_t* lbm = nullptr;
    uint32_t bm_reg = kNone;

    // rayMarchVoxelGrid (Renderer.cuh:260-336) and, SHADOW, shadowRayMarchVoxelGrid (:100-172).
    // The cluster-skip step (:290-306) and the voxel step (:318-331) share one
    // code path: both are o += (min_i (target_i - o_i) / d_i + EPSILON) * d with
    // target = the cluster plane (int, no EPSILON) or ceilf/floorf(o) +- EPSILON;
    // only the voxel step refreshes the t values the hit normal reads (the skip
    // branch's are block-scoped).  One set of IEEE divisions per
    // iteration instead of two divergent ones.  Lighting is applied by the
    // caller after the walk (Hit carries colour, normal and position).
    // EQ (shadow walks only): the direction's components are equal (the
    // default light, normalize(1,1,1), Main.cu:28).  Then every t_i = a_i / d
    // shares one divisor, and correctly rounded division is monotone in the
    // numerator, so min_i RN(a_i / d) = RN(min_i a_i / d) (max_i for d < 0):
    // one division per iteration instead of three, and (t + EPSILON) * d_i is
    // one product.  Bit-identical; shadow walks read no per-axis t values.
    template <bool SHADOW, bool EQ = false>
    __device__ __forceinline__ bool grid_original(f3& o, f3 d, uint32_t reg, i3 cr, Hit& h,
                                                  const uint32_t* rs = nullptr, const Rcp* rc = nullptr) {
        return grid_original_rt(o, d, reg, cr, h, SHADOW, SHADOW && EQ, rs, rc);
    }
    // The same with the shadow flag a per-lane value (fused primary + shadow
    // walk); the template form above constant-folds it.
    // rs (crawl pass only): a deferral record -- resume the walk at its crawl.
    // rc: the ray's reciprocals rcp_setup(d.x), (d.y), (d.z), made once per ray
    // (nullptr: made here).
    // generic: one loop for every sign pattern (the longest-axis walks' rare
    // original-DDA tails: less code and register demand in that kernel)
    __device__ __forceinline__ bool grid_original_rt(f3& o, f3 d, uint32_t reg, i3 cr, Hit& h, const bool SHADOW,
                                                     const bool EQ, const uint32_t* rs = nullptr,
                                                     const Rcp* rc = nullptr, const bool generic = false) {
        const bool resume = CRAWL && rs != nullptr;
        VR_DIAG_COUNT(SHADOW ? 9 : 8);                 // grid_original calls
        const bool px = d.x > 0.0f, py = d.y > 0.0f, pz = d.z > 0.0f;
        const bool zx = SHADOW && d.x == 0.0f, zy = SHADOW && d.y == 0.0f, zz = SHADOW && d.z == 0.0f;
        float tX, tY, tZ;
        if (resume) {                             // o is the stepped position of the crawl
            tX = __uint_as_float(rs[11]); tY = __uint_as_float(rs[12]); tZ = __uint_as_float(rs[13]);
        } else if (!CRAWL) {
            // The initial step (Renderer.cuh:269-280; shadow :106-117) with the ray's
            // hoisted reciprocals (or the walk's own, which its loop shares): |n| <= 1 +
            // EPSILON here, so the fast division's domain is the direction's plus
            // |n| >= 2^-90 (see div_fast).
            const bool use_rc = rc && (kFastSetup || SHADOW);
            const Rcp r0x = use_rc ? rc[0] : rcp_setup(d.x), r0y = use_rc ? rc[1] : rcp_setup(d.y),
                      r0z = use_rc ? rc[2] : rcp_setup(d.z);
            const float sx = px ? 1.0f : -1.0f, sy = py ? 1.0f : -1.0f, sz = pz ? 1.0f : -1.0f;
            const float ax = next_plane_fma(o.x, sx, sx * kEps) - o.x, ay = next_plane_fma(o.y, sy, sy * kEps) - o.y,
                        az = next_plane_fma(o.z, sz, sz * kEps) - o.z;
            const bool fast = r0x.ok && r0y.ok && r0z.ok && !zx && !zy && !zz &&
                              fminf(fabsf(ax), fminf(fabsf(ay), fabsf(az))) >= 0x1p-90f;
            tX = div_fast(ax, r0x); tY = div_fast(ay, r0y); tZ = div_fast(az, r0z);
            if (__builtin_expect(__builtin_amdgcn_ballot_w64(!fast) != 0, 0)) {
                tX = fast ? tX : (zx ? kInf : ax / d.x);
                tY = fast ? tY : (zy ? kInf : ay / d.y);
                tZ = fast ? tZ : (zz ? kInf : az / d.z);
            }
            o = add(o, scl(fminf(tX, fminf(tY, tZ)) + kEps, d));
        } else {
            const float nX = px ? ceilf(o.x) + kEps : floorf(o.x) - kEps;
            const float nY = py ? ceilf(o.y) + kEps : floorf(o.y) - kEps;
            const float nZ = pz ? ceilf(o.z) + kEps : floorf(o.z) - kEps;
            tX = zx ? kInf : (nX - o.x) / d.x;
            tY = zy ? kInf : (nY - o.y) / d.y;
            tZ = zz ? kInf : (nZ - o.z) / d.z;
            o = add(o, scl(fminf(tX, fminf(tY, tZ)) + kEps, d));
        }
        uint32_t col = kEmpty;
        if constexpr (STORE == STORE_VCS) {
            // Inside the region every voxel coordinate is in [0, 64): the mask
            // word index is a few bit operations and the lookup needs no
            // range check (Ctx::lookup's general form handles the rest).
            const uint2* mreg = s.vcs_mask + (size_t)reg * 8192u;
            // the region's mask words as a 32-bit byte offset from the scene's (uniform)
            // mask array: the loads take the SGPR-base form (one VGPR, no 64-bit add)
            const uint32_t moff = reg << 16;
            // (crawl pass) the region's cluster-existence bits in LDS: the workgroup's copy of
            // the scene's, or this lane's slot, refilled when the walk enters another region
            const uint32_t* bits = nullptr;
            if constexpr (CRAWL) {
                if (lbm) {
                    if (reg != bm_reg) {
                        const uint4* src = reinterpret_cast<const uint4*>(s.vcs_cbits + (size_t)reg * 16u);
                        const uint4 b0 = src[0], b1 = src[1], b2 = src[2], b3 = src[3];
                        uint4* dst = reinterpret_cast<uint4*>(lbm);
                        dst[0] = b0; dst[1] = b1; dst[2] = b2; dst[3] = b3;
                        bm_reg = reg;
                    }
                    bits = lbm;
                }
            }
            // Straight-line body with one exit: the hit test, the region test of
            // the stepped position and the iteration budget are folded into a
            // single condition; the step of the hit iteration is computed and
            // discarded (the reference breaks before it).  tick() semantics are
            // kept: iteration k of the pixel runs iff k <= kBudget.
            o = add(o, f3{0.0f, 0.0f, 0.0f});      // -0 -> +0 (in_region_bits_nz below)
            if (!this->in_region_bits_nz(o)) return false;
            if (aborted || this->iters >= kBudget) { aborted = true; return false; }
            bool found = false, inside = true, crawl = false;
            // crawl exits (see crawl_steps): from this iteration count on (crawl pass);
            // tile pass: until a deferral failed
            uint32_t crawl_after = 0;
            bool crawl_off = false;
            uint32_t vi = 0;
            int32_t qx = 0, qy = 0, qz = 0;   // crawl pass: voxel of the iteration that exited to crawl
            Blk blk{0u, kNone};
            uint32_t bit = 0;
            bool resume_now = resume;
            for (;;) {
                // Per-walk constants, (re)made here in the crawl pass so they are
                // dead across the crawl code below (the barrier keeps them from
                // being hoisted).
                f3 dl = d;
                if (CRAWL) asm("" : "+v"(dl.x), "+v"(dl.y), "+v"(dl.z));
                // Hoisted reciprocals (div_fast) and +-1 plane signs for the loop
                // (rcp_setup(-d) = -rcp_setup(d) bit for bit: tools/div_proof.hip).
                Rcp rx, ry, rz;
                if (rc && !CRAWL && (kFastSetup || SHADOW)) {
                    rx = EQ ? Rcp{fabsf(dl.x), fabsf(rc[0].r), rc[0].ok} : rc[0];
                    ry = rc[1];
                    rz = rc[2];
                } else {
                    rx = rcp_setup(EQ ? fabsf(dl.x) : dl.x); ry = rcp_setup(dl.y); rz = rcp_setup(dl.z);
                }
                const float gx = px ? 1.0f : -1.0f, gy = py ? 1.0f : -1.0f, gz = pz ? 1.0f : -1.0f;
                const float ex = gx * kEps, ey = gy * kEps, ez = gz * kEps;
                const int32_t cx8 = px ? 8 : 0, cy8 = py ? 8 : 0, cz8 = pz ? 8 : 0;
                // A guarded zero direction component (shadow ray) keeps the lane on the
                // slow branch, which applies the guard: the fast path needs no selects.
                const bool walk_ok = rx.ok && ry.ok && rz.ok && !zx && !zy && !zz;
                // one compare per iteration: min |n| >= lim (lim = +inf sends the lane
                // to the slow branch every iteration; |n| < 73 inside a region)
                const float nlim = walk_ok ? 0x1p-90f : kInf;
                if (resume_now) {
                    // the deferred crawl: its iteration left an absent cluster (blk) at
                    // voxel q with o stepped; the post-loop test below re-finds the crawl
                    resume_now = false;
                    blk = Blk{0u, kNone};
                    bit = 0;
                    qx = (int32_t)rs[15]; qy = (int32_t)rs[16]; qz = (int32_t)rs[17];
                } else {
                    // The loop, specialised for a wave whose lanes share the signs of the
                    // direction (nearly every primary tile; every shadow walk): the planes
                    // then need no sign multiplications (see plane_v / plane_c8).
                    auto walk = [&](auto SXc, auto SYc, auto SZc) {
                        constexpr int SX = decltype(SXc)::value, SY = decltype(SYc)::value, SZ = decltype(SZc)::value;
                        // All three components positive (every lane of this pass, and every
                        // lane's reciprocals in div_fast's domain: checked before this loop is
                        // chosen): then no numerator is ever tiny or zero -- a voxel plane lies
                        // >= ~EPSILON/2 beyond o, a cluster plane (v & ~7) + 8 > o by >= ulp(64)
                        // -- so the division needs no fallback, and no crawl (t = 0) can occur.
                        // (Sgn<2>: positive, and the caller checked the reciprocals)
                        constexpr bool kPos = SX == 2 && SY == 2 && SZ == 2;
                        // The iteration count as the budget test reads it, biased so that
                        // it reaches bits(64.0f) exactly when iters exceeds kBudget:
                        // one add per iteration.
                        uint32_t ic = this->iters + (0x42800000u - kBudget);
                        // Every lane's direction in div_fast's domain (nearly every walk): then
                        // only a cluster-skip plane can give a numerator outside it -- a voxel
                        // plane (ceilf(o) + EPSILON, floorf(o) - EPSILON) lies >= ~EPSILON/2 from
                        // o -- so the domain check runs only in wave-iterations where some lane
                        // skips (a scalar branch; -2 VALU per iteration without a skip).
                        const bool okw = __builtin_amdgcn_ballot_w64(!walk_ok) == 0;
                        VR_DIAG_COUNT((SHADOW ? 4 : 0) + (SX == 0 ? 1 : 0));   // walk entries
                        for (;;) {
                            VR_DIAG_COUNT((SHADOW ? 6 : 2) + (SX == 0 ? 1 : 0));   // loop iterations
                            const int32_t vx = f2i(o.x), vy = f2i(o.y), vz = f2i(o.z);
                            this->count(4);
                            const uint32_t wi = this->word_index((uint32_t)vx, (uint32_t)vy, (uint32_t)vz);
                            if constexpr (CRAWL) {
                                // (crawl pass) cluster slot wi >> 4 absent per the LDS bits: no load
                                const bool pres = !bits || ((bits[wi >> 9] >> ((wi >> 4) & 31u)) & 1u);
                                if (COUNT && !pres) ++this->nl;   // counted above, never loaded
                                blk = Blk{0u, kNone};
                                if (pres)
                                    blk = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(s.vcs_mask) +
                                                                          (moff | (wi << 3)));
                            } else {
                                blk = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(s.vcs_mask) +
                                                                      (moff | (wi << 3)));
                            }
                            __builtin_amdgcn_sched_barrier(0);   // issue the load before the planes
                            // both candidate planes, computed while the mask word is in
                            // flight and materialised (with the whole 8-B word: one load)
#if VR_UNIFORM_SKIP
                            float vX = plane_v<SX>(o.x, gx, ex), vY = plane_v<SY>(o.y, gy, ey), vZ = plane_v<SZ>(o.z, gz, ez);
                            asm("" : "+v"(vX), "+v"(vY), "+v"(vZ), "+v"(blk.x), "+v"(blk.y));
                            const bool skip = absent(blk);
                            float nX = vX, nY = vY, nZ = vZ;
                            const bool any_skip = __builtin_amdgcn_ballot_w64(skip) != 0;
                            if (any_skip) {
                                float cX = (float)((vx & 0x38) + plane_c8<SX>(cx8)), cY = (float)((vy & 0x38) + plane_c8<SY>(cy8)),
                                      cZ = (float)((vz & 0x38) + plane_c8<SZ>(cz8));
                                nX = skip ? cX : vX; nY = skip ? cY : vY; nZ = skip ? cZ : vZ;
                                asm volatile("" : "+v"(nX), "+v"(nY), "+v"(nZ));
                            }
#else
                            float vX = plane_v<SX>(o.x, gx, ex), vY = plane_v<SY>(o.y, gy, ey), vZ = plane_v<SZ>(o.z, gz, ez);
                            // (in the region v < 64, so v & ~7 == v & 0x38, the form word_index shares)
                            float cX = (float)((vx & 0x38) + plane_c8<SX>(cx8)), cY = (float)((vy & 0x38) + plane_c8<SY>(cy8)),
                                  cZ = (float)((vz & 0x38) + plane_c8<SZ>(cz8));
                            asm("" : "+v"(vX), "+v"(vY), "+v"(vZ), "+v"(cX), "+v"(cY), "+v"(cZ), "+v"(blk.x), "+v"(blk.y));
                            const bool skip = absent(blk);
                            const bool any_skip = __builtin_amdgcn_ballot_w64(skip) != 0;
#endif
                            const bool chk = !kPos && (!okw || any_skip);   // (uniform)
#ifdef VR_DIAG
                            {   // wave-iterations where no active lane / every active lane skips a cluster
                                const uint64_t bs = __builtin_amdgcn_ballot_w64(skip);
                                if (bs == 0) VR_DIAG_COUNT(SHADOW ? 24 : 22);
                                else if (bs == __builtin_amdgcn_read_exec()) VR_DIAG_COUNT(SHADOW ? 25 : 23);
                            }
#endif
                            bit = this->word_bit5((uint32_t)vy, (uint32_t)vz);
                            // 0 or ~0 (an absent cluster's words have no bits set)
                            const uint32_t fm = (uint32_t)__builtin_amdgcn_sbfe((int32_t)blk.x, bit, 1u);
                            found = fm != 0u;
                            vi = blk.y + __popc(blk.x & ((1u << (bit & 31u)) - 1u));
                            if (COUNT && !skip) this->count_bsearch(mreg + (wi & ~15u), vi, found);
#if !VR_UNIFORM_SKIP
                            const float nX = skip ? cX : vX;
                            const float nY = skip ? cY : vY;
                            const float nZ = skip ? cZ : vZ;
#endif
                            const float ax = nX - o.x, ay = nY - o.y, az = nZ - o.z;
                            float sMin;
                            crawl = false;
                            if (EQ) {
                                // |a_i| / |d| = a_i / d up to the sign of a zero (t = -0 for
                                // a = +0, d < 0), which neither the step nor the crawl test sees
                                const float am = fminf(fabsf(ax), fminf(fabsf(ay), fabsf(az)));
                                sMin = div_fast(am, rx);
                                if (chk) {
                                    const bool bad = !(am >= nlim);
                                    if (__builtin_expect(__builtin_amdgcn_ballot_w64(bad) != 0, 0)) {
                                        sMin = bad ? am / fabsf(d.x) : sMin;
                                        crawl = bad & walk_ok & skip & (sMin == 0.0f) &
                                                (CRAWL ? ic + 1u - (0x42800000u - kBudget) >= crawl_after : !crawl_off);
                                        if (CRAWL && crawl) { qx = vx; qy = vy; qz = vz; }
                                    }
                                }
                            } else {
                                float sX = div_fast(ax, rx), sY = div_fast(ay, ry), sZ = div_fast(az, rz);
                                if (chk) {
                                    const bool bad = !(fminf(fabsf(ax), fminf(fabsf(ay), fabsf(az))) >= nlim);
                                    if (__builtin_expect(__builtin_amdgcn_ballot_w64(bad) != 0, 0)) {
                                        sX = bad ? (zx ? kInf : ax / d.x) : sX;
                                        sY = bad ? (zy ? kInf : ay / d.y) : sY;
                                        sZ = bad ? (zz ? kInf : az / d.z) : sZ;
                                        // a skip step with t = 0 (its plane axis has n = 0, so it is
                                        // always on this branch): the ray creeps through an empty cluster
                                        crawl = bad & walk_ok & skip & (fminf(sX, fminf(sY, sZ)) == 0.0f) &
                                                (CRAWL ? ic + 1u - (0x42800000u - kBudget) >= crawl_after : !crawl_off);
                                        if (CRAWL && crawl) { qx = vx; qy = vy; qz = vz; }
                                    }
                                }
                                sMin = fminf(sX, fminf(sY, sZ));
                                const bool vox = !skip && !found;        // a voxel step: its t values feed the normal
                                tX = vox ? sX : tX; tY = vox ? sY : tY; tZ = vox ? sZ : tZ;   // (tMin: min of the three, at the use)
                            }
                            // A hit keeps o unstepped: its step length becomes (-EPSILON) + EPSILON
                            // = +0 exactly, and o + (+0 * d) = o (o is never -0, d is finite in here).
                            const float ts = bit_select(fm, -kEps, sMin) + kEps;
                            o = EQ ? add(o, f3{ts * d.x, ts * d.x, ts * d.x}) : add(o, scl(ts, d));
                            // One unsigned compare for hit, region exit (in_region_bits_nz of the
                            // stepped position) and the budget (iters >= kBudget):
                            // (the add as asm: loop strength reduction otherwise keeps two counters)
                            asm("v_add_u32 %0, 1, %0" : "+v"(ic));
                            const uint32_t ev = max(max(max(max(__float_as_uint(o.x), __float_as_uint(o.y)), __float_as_uint(o.z)),
                                                        ic), fm);
                            if (ev >= 0x42800000u || crawl) break;
                        }
                        this->iters = ic - (0x42800000u - kBudget);
                    };
                    const uint32_t sg = (px ? 1u : 0u) | (py ? 2u : 0u) | (pz ? 4u : 0u);
                    using N = Sgn<-1>;
                    using P = Sgn<1>;
                    if (CRAWL || generic) {
                        walk(Sgn<0>{}, Sgn<0>{}, Sgn<0>{});
                    } else {
                        // One pass of the loop specialised for each sign pattern present in
                        // the wave (nearly always one; a tile straddling a plane where a
                        // direction component changes sign runs two or more, one after the
                        // other).  A generic, per-lane-sign loop in this kernel needed ~81
                        // VGPRs against the specialised loops' ~72 (7 waves/SIMD).  (An
                        // equal-component shadow direction has pattern 0 or 7.)
                        bool todo = true;
                        while (todo) {
                            const uint32_t pat = __builtin_amdgcn_readfirstlane(sg);
                            if (sg == pat) {
                                todo = false;
                                switch (pat) {
                                case 0: walk(N{}, N{}, N{}); break;
                                case 7:
                                    if (__builtin_amdgcn_ballot_w64(!walk_ok) == 0) walk(Sgn<2>{}, Sgn<2>{}, Sgn<2>{});
                                    else walk(P{}, P{}, P{});
                                    break;
                                case 1: if (!EQ) walk(P{}, N{}, N{}); break;
                                case 2: if (!EQ) walk(N{}, P{}, N{}); break;
                                case 3: if (!EQ) walk(P{}, P{}, N{}); break;
                                case 4: if (!EQ) walk(N{}, N{}, P{}); break;
                                case 5: if (!EQ) walk(P{}, N{}, P{}); break;
                                default: if (!EQ) walk(N{}, P{}, P{}); break;
                                }
                            }
                        }
                    }
                }
                // Why the lane left, recomputed from values the loop keeps in VGPRs
                // anyway (a flag read after a divergent loop is carried through it as
                // a lane mask, at three scalar ops per flag per iteration; the barrier
                // keeps the compiler from reusing the in-loop flags): a hit leaves o
                // unstepped (inside), and a crawl is the one remaining exit.
                asm("" : "+v"(blk.x), "+v"(blk.y), "+v"(bit), "+v"(o.x), "+v"(o.y), "+v"(o.z), "+v"(this->iters));
                found = !absent(blk) & (__builtin_amdgcn_ubfe(blk.x, bit, 1u) != 0u);
                inside = found || this->in_region_bits_nz(o);
                crawl = !found && inside && this->iters < kBudget;
                if (!crawl || !inside || this->iters >= kBudget) break;
                if constexpr (!CRAWL) {
                    // Defer only a real crawl: an axis on its own skip plane that
                    // EPSILON * d cannot move (it did not: o is the stepped position),
                    // so t = 0 again and again.  A one-off t = 0 step walks on here.
                    // (o on its plane (v & ~7) <=> o / 8 is an integer; o * 0.125 is exact)
                    const bool kx = !px && truncf(o.x * 0.125f) == o.x * 0.125f && o.x + kEps * d.x == o.x;
                    const bool ky = !py && truncf(o.y * 0.125f) == o.y * 0.125f && o.y + kEps * d.y == o.y;
                    const bool kz = !pz && truncf(o.z * 0.125f) == o.z * 0.125f && o.z + kEps * d.z == o.z;
                    // Defer the whole pixel to the crawl pass if a list entry is
                    // free (unwinds like an abort); otherwise walk on plainly.
                    if ((kx || ky || kz) && v.defer) {
                        const uint32_t idx = atomicAdd(v.defer, 1u);
                        deferral_report(v);
                        if (idx < v.defer_cap) {
                            // (the tile pass writes this pixel as 0; the crawl pass,
                            // which runs after it, overwrites it and counts its bytes)
                            uint32_t* r = v.defer + 4 + (size_t)idx * kDeferRecWords;
                            r[0] = tile_pixels()[threadIdx.x];   // (l << 16 | x), from LDS: not kept live through the walk
                            r[1] = (SHADOW ? 1u : 0u) | this->ctx;
                            r[2] = __float_as_uint(o.x); r[3] = __float_as_uint(o.y); r[4] = __float_as_uint(o.z);
                            r[5] = (uint32_t)cr.x; r[6] = (uint32_t)cr.y; r[7] = (uint32_t)cr.z;
                            r[8] = v.launch_id;                         // (the crawl pass takes only its launch's)
                            r[9] = this->iters;
                            r[10] = this->bytes;
                            // (a shadow walk has no normal: its t values are not kept live for this)
                            r[11] = SHADOW ? 0u : __float_as_uint(tX); r[12] = SHADOW ? 0u : __float_as_uint(tY);
                            r[13] = SHADOW ? 0u : __float_as_uint(tZ); r[14] = 0u;   // reserved
                            // (the crawl iteration's voxel q, words 15-17, is recovered from the
                            // stepped position by the crawl pass: see crawl_kernel)
                            r[1] |= v.crawl_rewalk ? 4u : 0u;
                            r[18] = this->lit_saved;
                            // (the flag that the record exists is this sentinel: a bool here would
                            // be carried through every loop as a lane mask -- SGPR spills)
                            this->iters = kDeferredIters;
                            aborted = true;
                            return false;
                        }
                    }
                    if (kx || ky || kz) crawl_off = true;
                } else {
                    // Off the hot loop: fast-forward the identical crawl iterations
                    // exactly, then resume the walk (no region-entry step).
#ifdef VR_CRAWL_PROF
                    const uint32_t n = crawl_run(o, d, qx, qy, qz, px, py, pz, kBudget - this->iters, bits, &this->d_trips);
#else
                    const uint32_t n = crawl_run(o, d, qx, qy, qz, px, py, pz, kBudget - this->iters, bits);
#endif
                    // none (not a real crawl, or its next step leaves the cluster): a few plain
                    // iterations, then re-arm
                    if (n == 0u) {
                        crawl_after = this->iters + 8u;
                    } else {
                        this->iters += n;
                        this->count_ff(n);
                        inside = this->in_region_bits_nz(o);
                        if (!inside || this->iters >= kBudget) break;
                    }
                }
            }
            if (!found) {
                if (inside) aborted = true;     // the next iteration's tick() would have failed
                return false;
            }
            col = s.vcs_vals[vi];
        } else {
            // Cuckoo store (doesVoxelSpaceExist is always true: no cluster skips).
            // Every iteration looks its voxel's key up (CuckooHashTable::lookupVoxel,
            // CuckooHashTable.cuh:59-76).  A key that is not in the tables -- nearly every
            // probe of a walk -- costs the reference key1 and key2 (8 B) and misses: that is
            // answered by the region's key-presence filter (KScene::ht_filter, one bit per
            // voxel, the VCS mask-word order: a wave's neighbouring rays read neighbouring
            // words), so the loop is one coalesced 4-B load, the voxel step and one exit test.
            // The key that IS present ends the walk: after the loop its two slots are probed
            // as the reference does (key1, val1 on a match, else key2, val2), and the bytes
            // of the table it was found in are counted.  (Round 4 probed both slots of every
            // iteration -- random HBM reads, 2.3x the algorithmic bytes at C4, L2 hit 0.55.)
            o = add(o, f3{0.0f, 0.0f, 0.0f});      // -0 -> +0 (in_region_bits_nz below)
            if (!this->in_region_bits_nz(o)) return false;
            if (aborted || this->iters >= kBudget) { aborted = true; return false; }
            const Rcp rx = rcp_setup(EQ ? fabsf(d.x) : d.x), ry = rcp_setup(d.y), rz = rcp_setup(d.z);
            const float gx = px ? 1.0f : -1.0f, gy = py ? 1.0f : -1.0f, gz = pz ? 1.0f : -1.0f;
            const float ex = gx * kEps, ey = gy * kEps, ez = gz * kEps;
            const bool walk_ok = rx.ok && ry.ok && rz.ok && !zx && !zy && !zz;
            const float nlim = walk_ok ? 0x1p-90f : kInf;
            // no cluster skips here: with every lane's direction in div_fast's domain no
            // numerator (a voxel plane's, >= ~EPSILON/2 from o) leaves it -- no check at all
            const bool okw = __builtin_amdgcn_ballot_w64(!walk_ok) == 0;
            // the region's filter words (64-bit: a cuckoo scene has no region bound, vr_internal.h)
            const uint32_t* freg = s.ht_filter + (size_t)reg * kHashFilterWords;
            uint32_t fw = 0, bit = 0;
            uint32_t ic = this->iters + (0x42800000u - kBudget);   // biased count (see the VCS walk)
            // rayMarchVoxelGrid's voxel step (Renderer.cuh:318-331) from o: its t values, min
            auto voxel_step = [&](float& sX, float& sY, float& sZ) -> float {
                const float ax = next_plane_fma(o.x, gx, ex) - o.x, ay = next_plane_fma(o.y, gy, ey) - o.y,
                            az = next_plane_fma(o.z, gz, ez) - o.z;
                if (EQ) {                                 // see grid_original
                    const float am = fminf(fabsf(ax), fminf(fabsf(ay), fabsf(az)));
                    float sMin = div_fast(am, rx);
                    if (!okw) {
                        const bool bad = !(am >= nlim);
                        if (__builtin_expect(__builtin_amdgcn_ballot_w64(bad) != 0, 0)) sMin = bad ? am / fabsf(d.x) : sMin;
                    }
                    return sMin;
                }
                sX = div_fast(ax, rx); sY = div_fast(ay, ry); sZ = div_fast(az, rz);
                if (!okw) {
                    const bool bad = !(fminf(fabsf(ax), fminf(fabsf(ay), fabsf(az))) >= nlim);
                    if (__builtin_expect(__builtin_amdgcn_ballot_w64(bad) != 0, 0)) {
                        sX = bad ? (zx ? kInf : ax / d.x) : sX;
                        sY = bad ? (zy ? kInf : ay / d.y) : sY;
                        sZ = bad ? (zz ? kInf : az / d.z) : sZ;
                    }
                }
                return fminf(sX, fminf(sY, sZ));
            };
            for (;;) {
                const int32_t vx = f2i(o.x), vy = f2i(o.y), vz = f2i(o.z);
                const uint32_t wi = this->word_index((uint32_t)vx, (uint32_t)vy, (uint32_t)vz);
                fw = freg[wi];
                __builtin_amdgcn_sched_barrier(0);   // issue the load before the step
                // the voxel step while the word loads
                float sX = 0.0f, sY = 0.0f, sZ = 0.0f;
                const float sMin = voxel_step(sX, sY, sZ);
                // key1 + key2 of a key the tables do not hold; the hit's own bytes are
                // settled after the loop (8 or 12)
                this->count(8u);
                bit = this->word_bit5((uint32_t)vy, (uint32_t)vz);
                const uint32_t fm = (uint32_t)__builtin_amdgcn_sbfe((int32_t)fw, bit, 1u);   // 0 or ~0: present
                if (!SHADOW && !EQ) {                     // a non-hit step: its t values feed the normal
                    tX = fm ? tX : sX; tY = fm ? tY : sY; tZ = fm ? tZ : sZ;
                }
                // a hit keeps o unstepped: step length (-EPSILON) + EPSILON = +0 (see the VCS walk)
                const float ts = bit_select(fm, -kEps, sMin) + kEps;
                o = EQ ? add(o, f3{ts * d.x, ts * d.x, ts * d.x}) : add(o, scl(ts, d));
                asm("v_add_u32 %0, 1, %0" : "+v"(ic));      // (see the VCS walk)
                const uint32_t ev = max(max(max(max(__float_as_uint(o.x), __float_as_uint(o.y)), __float_as_uint(o.z)), ic), fm);
                if (ev >= 0x42800000u) break;
            }
            this->iters = ic - (0x42800000u - kBudget);
            // why the lane left (see the VCS walk): recomputed from VGPR values
            asm("" : "+v"(fw), "+v"(bit), "+v"(o.x), "+v"(o.y), "+v"(o.z));
            if (!__builtin_amdgcn_ubfe(fw, bit, 1u)) {
                if (this->in_region_bits_nz(o)) aborted = true;    // budget spent inside the region
                return false;
            }
            // A shadow walk's hit needs no value: the reference's lookup returns the voxel's
            // colour, and a shadow walk only asks whether it is EMPTY_VAL -- which no stored colour
            // is (< 2^24) -- so the set filter bit (the tables' exact key set) already answers
            // it.  The two random table reads (HBM for C4's 400-MB store) are skipped; the COUNT
            // build still makes them, for the bytes the reference reads (8 or 12).
            col = 0u;                              // (a shadow walk's hit: any colour but EMPTY_VAL)
            if (!SHADOW || COUNT) {
                // the hit (o unstepped: the probed voxel): CuckooHashTable::lookupVoxel's two probes
                const uint32_t key = lshl_or(lshl_or((uint32_t)f2i(o.x), 10u, (uint32_t)f2i(o.y)), 10u, (uint32_t)f2i(o.z));
                const uint4 m = s.ht_meta[reg];    // {base, M, prime, offset}
                const uint2* t1 = s.ht_slots + m.x;
                const uint2 e1 = t1[hash1(key, m.w) % m.y];
                const uint2 e2 = t1[m.y + hash2(key, m.z) % m.y];
                const bool m1 = e1.x == key;
                this->count(m1 ? 0u : 4u);         // key1 + val1 (8, counted above), or key1 + key2 + val2
                col = m1 ? e1.y : e2.y;
            }
        }
        if (col == kEmpty) return false;
        if (!SHADOW) {
            h.col = col;
            // tMin is always min(tX, tY, tZ) of the same step: recomputed here
            // instead of carried through the loop
            h.nc = normal_from_t(tX, tY, tZ, fminf(tX, fminf(tY, tZ)), d);
            h.so = o;
            h.region = cr;
            h.longest = false;
        }
        return true;
    }

    // rayMarchVoxelGridLongestAxis (Renderer.cuh:760-915) / shadowRayMarchVoxelGridLongestAxis
    // (:495-631) with performVoxelSpaceJump (:696-751) / performShadowVoxelSpaceJump (:441-492),
    // as a convergent state machine: every loop iteration makes exactly ONE probe
    // (existence check, lookup if present) for every lane, whatever it is doing --
    //   main  : the next axis step of the current iteration of the reference loop
    //           (M/S in crossing order, then L; g[axis] += ad[axis] first), or
    //   jump  : performVoxelSpaceJump's `while (!exists(g))` probes (the first one
    //           re-checks the step's own voxel, as the reference does) and cluster skips,
    // then advances that lane's state.  Same probes, ticks and bytes, in the same
    // order, as the nested reference loops; no per-case code copies, no divergent
    // nesting.  The tail falls back to the original DDA (Renderer.cuh:912).
    template <bool SHADOW>
    __device__ __forceinline__ bool grid_longest(f3& oo, f3 od, uint32_t reg, i3 cr, Hit& h) {
        uint32_t L, M, S;
        // Ray::convertRayToLongestAxisDirection (Ray.cuh:19-71)
        float ax = fabsf(od.x), ay = fabsf(od.y), az = fabsf(od.z), k;
        if (ax > ay && ax > az) {
            L = 0; M = ay > az ? 1 : 2; S = ay > az ? 2 : 1; k = 1.0f / ax;
        } else if (ay > az) {
            L = 1; M = ax > az ? 0 : 2; S = ax > az ? 2 : 0; k = 1.0f / ay;
        } else {
            L = 2; M = ax > ay ? 0 : 1; S = ax > ay ? 1 : 0; k = 1.0f / az;
        }
        const f3 ds = scl(k, od);
        f3 old_o = oo;
        i3 g{f2i(oo.x), f2i(oo.y), f2i(oo.z)};
        i3 ad{0, 0, 0};
        const int32_t adL = comp(od, L) < 0.0f ? -1 : 1;
        seti(ad, L, adL);
        f3 ray_o;
        {
            const float gL = (float)geti(g, L), oL = comp(oo, L);
            const float t = adL > 0 ? (gL + kEps + 1.0f - oL) / (float)adL : (gL - kEps - oL) / (float)adL;
            ray_o = add(old_o, scl(t, ds));
        }
        seti(ad, M, f2i(comp(ray_o, M)) - geti(g, M));
        seti(ad, S, f2i(comp(ray_o, S)) - geti(g, S));
        const bool mid_floor = comp(ds, M) < 0.0f;   // decimalToIntFunc (:784)
        float tX = 0.0f, tY = 0.0f, tZ = 0.0f, tMin = 0.0f;   // the jump's last skip (hit normal)
        uint32_t seq = 0, rem = 0;                   // pending axis steps of this iteration (2 bits each)
        bool jumping = false;

        // Top of the reference's `while (isInGrid(grid + diff))` loop: false = loop over
        // (fall back to the original DDA); aborted = budget exhausted.
        auto begin_iter = [&]() -> bool {
            if (!grid_in_region(g.x + ad.x, g.y + ad.y, g.z + ad.z)) return false;
            if (!tick()) return false;
            const int32_t adM = geti(ad, M), adS = geti(ad, S);
            if (adS != 0 && adM != 0) {
                const float om = comp(old_o, M);
                const float t1 = ((mid_floor ? floorf(om) : ceilf(om)) - om) / comp(ds, M);
                const float sp = comp(old_o, S) + comp(ds, S) * t1;
                const int32_t sd = f2i(floorf(sp)) - geti(g, S);
                const uint32_t a0 = sd != 0 ? S : M, a1 = sd != 0 ? M : S;
                seq = a0 | (a1 << 2) | (L << 4);
                rem = 3;
            } else if (adM != 0) {
                seq = M | (L << 2);
                rem = 2;
            } else if (adS != 0) {
                seq = S | (L << 2);
                rem = 2;
            } else {
                seq = L;
                rem = 1;
            }
            return true;
        };

        bool tail = !begin_iter();
        if (aborted) return false;
        while (!tail) {
            const uint32_t axis = seq & 3u;
            i3 pg = g;
            if (!jumping) seti(pg, axis, geti(g, axis) + geti(ad, axis));
            const Blk blk = exists(reg, pg.x, pg.y, pg.z);
            const bool present = !absent(blk);
            const uint32_t col = present ? lookup(reg, blk, pg.x, pg.y, pg.z) : kEmpty;
            g = pg;
            if (col != kEmpty) {
                if (!SHADOW) {
                    h.col = col;
                    h.region = cr;
                    h.longest = true;
                    if (jumping) {                   // performVoxelSpaceJump's hit
                        h.nc = normal_from_t(tX, tY, tZ, tMin, ds);
                        h.so = old_o;
                    } else {                         // an axis step's hit
                        h.nc = this->ncode(axis, copysignf(1.0f, -comp(ds, axis)));
                        if (axis == L) {
                            h.so = ray_o;
                        } else {                     // getLocalHitLocation (Renderer.cuh:753-758)
                            const float o = comp(old_o, axis), dd = comp(ds, axis);
                            const float t = dd > 0.0f ? (ceilf(o) - o) / dd : (floorf(o) - o) / dd;
                            h.so = add(old_o, scl(t, ds));
                        }
                    }
                }
                return true;
            }
            if (!jumping) {
                if (!present) { jumping = true; continue; }   // performVoxelSpaceJump (re-probes g)
                seq >>= 2;
                if (--rem != 0u) continue;
                old_o = ray_o;                       // end of the iteration (:903-906)
                ray_o = add(ray_o, ds);
                seti(ad, M, f2i(comp(ray_o, M)) - geti(g, M));
                seti(ad, S, f2i(comp(ray_o, S)) - geti(g, S));
                tail = !begin_iter();
                if (aborted) return false;
                continue;
            }
            if (!present) {                          // the jump's cluster skip
                if (!tick()) return false;
                const int32_t nx = ds.x > 0.0f ? ((g.x / 8) + 1) * 8 : (g.x / 8) * 8;
                const int32_t ny = ds.y > 0.0f ? ((g.y / 8) + 1) * 8 : (g.y / 8) * 8;
                const int32_t nz = ds.z > 0.0f ? ((g.z / 8) + 1) * 8 : (g.z / 8) * 8;
                tX = ((float)nx - old_o.x) / ds.x;
                tY = ((float)ny - old_o.y) / ds.y;
                tZ = ((float)nz - old_o.z) / ds.z;
                tMin = fminf(tX, fminf(tY, tZ)) + kEps;
                old_o = add(old_o, scl(tMin, ds));
                g = i3{f2i(floorf(old_o.x)), f2i(floorf(old_o.y)), f2i(floorf(old_o.z))};
                if (!grid_in_region(g.x, g.y, g.z)) {
                    oo = old_o;
                    return false;
                }
                continue;
            }
            // the jump landed in an existing cluster without a hit: CONTINUE_VAL
            const float oL = comp(old_o, L), dL = comp(ds, L);
            const float tNext = dL > 0.0f ? (ceilf(oL) - oL) / dL : (floorf(oL) - oL) / dL;
            ray_o = add(old_o, scl(tNext + kEps, ds));
            seti(ad, M, f2i(comp(ray_o, M)) - geti(g, M));
            seti(ad, S, f2i(comp(ray_o, S)) - geti(g, S));
            jumping = false;
            tail = !begin_iter();
            if (aborted) return false;
        }
        oo = old_o;     // Renderer.cuh:912 (direction of originalRay kept)
        return grid_original<SHADOW>(oo, od, reg, cr, h);
    }

    // The VCS longest-axis walk with ONE reference loop iteration per loop
    // iteration (rayMarchVoxelGridLongestAxis, Renderer.cuh:760-915; shadow twin
    // :495-631; performVoxelSpaceJump :696-751 / :441-492), specialised on the
    // ray's axis order: L, M, S (longest, middle, shortest) are compile-time, so
    // the walk state lives in (L, M, S) registers and no axis is selected at run
    // time (a wave runs one pass per order its lanes hold; shadow rays share one).
    // A lane is either
    //   main : one whole iteration of the reference's while loop -- its probes
    //          are known at its top: slot A (the first crossing, M or S), slot B
    //          (both crossings) and slot C (g + ad, the L step); their three mask
    //          words are loaded together and evaluated in order; the first absent
    //          cluster starts a jump, the first stored voxel is the hit, or
    //   jump : one cluster skip of performVoxelSpaceJump and the probe of the
    //          cell it lands in (slot C; the jump's first existence test re-reads
    //          the probe that started it, known absent: counted, not loaded).
    // Probes, ticks and counted bytes are the reference's, in its order; the
    // later probes of an iteration that stops early are loaded but not counted.
    // Returns the hit; `tail` = the loop ended in the region (the caller runs
    // the original DDA from oo, Renderer.cuh:912-914, once for every order).
    template <int A>
    __device__ __forceinline__ static float ax3(f3 v) { return A == 0 ? v.x : (A == 1 ? v.y : v.z); }
    // ds: the longest-axis direction k * d (Ray.cuh:19-71, made by the caller);
    // cls: its sign classes, the same for every lane of the pass (an SGPR): bit 2a
    // = ds_a > 0, bit 2a+1 = ds_a < 0 (a zero or NaN component is neither), so every
    // direction-sign choice of the walk -- axisDiff[L], decimalToIntFunc, the jump's
    // cluster planes, tNext's ceil/floor -- is a scalar select, not a per-lane mask.
    // UNIT (shadow walks of a light whose ds is (+-1, +-1, +-1) exactly, e.g. the
    // reference's normalize(1,1,1), Main.cu:28): every division by ds_a is exact
    // negation or identity, so it is one multiply (x / +-1 == x * +-1 for every x).
    template <bool SHADOW, bool UNIT, int PL, int PM, int PS>
    __device__ __forceinline__ bool walk_longest_vcs(f3& oo, const f3 ds, const uint32_t cls, uint32_t reg,
                                                     bool& tail, uint32_t& hcol, uint32_t& hcode) {
        const float dL = ax3<PL>(ds), dM = ax3<PM>(ds), dS = ax3<PS>(ds);
        auto dv = [](float n, float d) { return UNIT ? n * d : n / d; };
        // (IEEE divisions here: div_fast with reciprocals made at each use, pinned so they
        // are never loop-carried, measured slower -- C3 0.2264 -> 0.2358 ms per frame,
        // profiles/r04/ab_lfd_rolled.txt -- as every hoisted-reciprocal variant before it)
        auto dv3 = [&](float n0, float d0, float n1, float d1, float n2, float d2, float& q0, float& q1, float& q2) {
            q0 = dv(n0, d0); q1 = dv(n1, d1); q2 = dv(n2, d2);
        };
        auto dv1 = [&](float n, float d) { return dv(n, d); };
        const bool posL = (cls >> (2 * PL)) & 1u, posM = (cls >> (2 * PM)) & 1u, posS = (cls >> (2 * PS)) & 1u;
        const bool negL = (cls >> (2 * PL + 1)) & 1u, negM = (cls >> (2 * PM + 1)) & 1u;
        const int32_t offL = posL ? 8 : 0, offM = posM ? 8 : 0, offS = posS ? 8 : 0;
        // walk frame <-> grid axes (x, y, z): constant indices, registers only
        auto xyz = [](auto l, auto m, auto s) {
            struct { decltype(l) c[3]; } r;
            r.c[PL] = l; r.c[PM] = m; r.c[PS] = s;
            return r;
        };
        auto to_f3 = [&](float l, float m, float s) {
            const auto c = xyz(l, m, s);
            return mk(c.c[0], c.c[1], c.c[2]);
        };
        auto to_i3 = [&](int32_t l, int32_t m, int32_t s) {
            const auto c = xyz(l, m, s);
            return i3{c.c[0], c.c[1], c.c[2]};
        };
        auto word = [&](int32_t l, int32_t m, int32_t s) {
            const auto c = xyz((uint32_t)l & 63u, (uint32_t)m & 63u, (uint32_t)s & 63u);
            return this->word_index(c.c[0], c.c[1], c.c[2]);
        };
        auto bit5 = [&](int32_t l, int32_t m, int32_t s) {
            const auto c = xyz((uint32_t)l, (uint32_t)m, (uint32_t)s);
            return this->word_bit5(c.c[1], c.c[2]) & 31u;
        };
        float oL = ax3<PL>(oo), oM = ax3<PM>(oo), oS = ax3<PS>(oo);      // oldRay origin
        int32_t gL = f2i(oL), gM = f2i(oM), gS = f2i(oS);                 // gridValues
        // axisDiff[L] (d_L < 0 <=> ds_L < 0: k > 0, or k = inf with d = 0, or NaN)
        const int32_t aL = negL ? -1 : 1;
        float rL, rM, rS;                                                 // ray origin
        {
            // x / (float)aL with aL = +-1 is exactly x * aL
            const float t = aL > 0 ? ((float)gL + kEps + 1.0f - oL) * (float)aL : ((float)gL - kEps - oL) * (float)aL;
            rL = oL + t * dL; rM = oM + t * dM; rS = oS + t * dS;
        }
        int32_t aM = f2i(rM) - gM, aS = f2i(rS) - gS;
        const bool mid_floor = negM;                                      // decimalToIntFunc (:784)
        // (IEEE divisions: hoisted reciprocals (div_fast) measured slower here, C3
        // 0.385 -> 0.413 ms -- three more VGPRs live through the loop)
        const uint32_t moff = reg << 16;              // SGPR-base loads (see grid_original_rt)
        auto mload = [&](uint32_t w) {
            return *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(s.vcs_mask) + (moff | (w << 3)));
        };
        uint32_t nj = 0;                  // the jump's last skip: getNormalFromTValues' axis (x, y, z)
        bool jumping = false;
        uint32_t stop = 3u, col = 0;
        bool mfirst = false;
        // One exit per iteration (each extra exit of a divergent loop costs lane-mask
        // bookkeeping on every iteration): a lane that must leave computes the rest
        // of the iteration on stale values and leaves at its end, with the reason
        // kOver: past the budget; kCrawl (tile pass): a cluster skip with t = 0 -- a jump
        // crawl, 10^4..10^6 iterations in the reference: the crawl pass walks the pixel
        enum : uint32_t { kGo = 0, kHit = 1, kLeft = 2, kOver = 3, kTail = 4, kCrawl = 5 };
        uint32_t why = kGo, it = this->iters;
        VR_DIAG_COUNT(SHADOW ? 19 : 17);               // longest-axis walks
        for (;;) {
            VR_DIAG_COUNT(SHADOW ? 20 : 18);           // longest-axis loop iterations
            VR_DIAG_COUNT_IF(jumping, 21);             // ... with a jumping lane
            // ---- this iteration's probe slots (A.L = B.L = gL)
            int32_t AM, AS, CL, CM, CS;
            bool vA = false, vB = false;
            mfirst = false;
            uint32_t ex;
            if (!jumping) {
                CL = gL + aL; CM = gM + aM; CS = gS + aS;
                // the loop condition (else the original-DDA tail), then tick()
                const bool out = !grid_in_region(CL, CM, CS);
                it += out ? 0u : 1u;
                ex = out ? kTail : (it > kBudget ? kOver : kGo);
                const bool hasM = aM != 0, hasS = aS != 0;
                bool sfirst = false;
                if (hasM && hasS) {
                    const float t1 = dv1((mid_floor ? floorf(oM) : ceilf(oM)) - oM, dM);
                    const float sp = oS + dS * t1;
                    sfirst = f2i(floorf(sp)) - gS != 0;
                }
                vA = hasM || hasS;
                vB = hasM && hasS;
                mfirst = hasM && !sfirst;
                AM = mfirst ? CM : gM;
                AS = mfirst ? gS : CS;
            } else {
                ++it;                                // tick()
                ex = it > kBudget ? kOver : kGo;
                // performVoxelSpaceJump's cluster skip (:707-725), integer planes from g:
                // d > 0 ? ((g / 8) + 1) * 8 : (g / 8) * 8.  (g / 8) * 8 is g & ~7 for g >= 0
                // (a walk's cells never go below 0; the C division form for any wave
                // holding a negative one)
                int32_t bL = gL & ~7, bM = gM & ~7, bS = gS & ~7;
                if (__builtin_expect(__builtin_amdgcn_ballot_w64((gL | gM | gS) < 0) != 0, 0)) {
                    bL = (gL / 8) * 8; bM = (gM / 8) * 8; bS = (gS / 8) * 8;
                }
                const int32_t nL = bL + offL, nM = bM + offM, nS = bS + offS;
                float jL, jM, jS;
                dv3((float)nL - oL, dL, (float)nM - oM, dM, (float)nS - oS, dS, jL, jM, jS);
                const auto t = xyz(jL, jM, jS);
                const float tm0 = fminf(t.c[0], fminf(t.c[1], t.c[2]));
                const float tMin = tm0 + kEps;
                nj = t.c[0] == tMin ? 0u : (t.c[1] == tMin ? 1u : 2u);
                const float pL = oL, pM = oM, pS = oS;
                const int32_t qL = gL, qM = gM, qS = gS;
                oL = oL + tMin * dL; oM = oM + tMin * dM; oS = oS + tMin * dS;
                gL = f2i(floorf(oL)); gM = f2i(floorf(oM)); gS = f2i(floorf(oS));
                if (ex == kGo && !grid_in_region(gL, gM, gS)) ex = kLeft;   // left the region: no tail
                // t = 0: the ray stood on a cluster plane.  When EPSILON * d cannot move it
                // off (the axis is still on the plane after the step) every further skip in
                // this cluster is the same: a crawl, for the crawl pass.  A one-off walks on.
                // (The t = 0 axis is M or S: |d_L| ~ 1, so EPSILON * d_L always moves L.)
                if (!CRAWL && ex == kGo && tm0 == 0.0f && (oM == pM || oS == pS)) ex = kCrawl;
                if constexpr (CRAWL) {
                    if (ex == kGo) {
                        if (this->same_f(oL, pL) && this->same_f(oM, pM) && this->same_f(oS, pS) && gL == qL &&
                            gM == qM && gS == qS) {
                            // the skip changed nothing (a NaN position): the jump loop never ends
                            ex = kOver;
                        } else if (tm0 == 0.0f) {
                            // A jump crawl: an axis pinned on its cluster plane that EPSILON * d
                            // cannot move, so every skip in this cluster is o += RN(EPSILON * d)
                            // (tMin = 0 + EPSILON) -- the same recurrence as the original walk's
                            // crawl: fast-forward it exactly (ticks and existence reads credited;
                            // the final position stays in the cluster, so the next skip -- whose t
                            // values a hit's normal reads -- is a plain one).
                            f3 on = to_f3(oL, oM, oS);
                            const f3 dd = to_f3(dL, dM, dS);
                            const i3 q = to_i3(qL, qM, qS);
                            const uint32_t n = crawl_run(on, dd, q.x, q.y, q.z, dd.x > 0.0f, dd.y > 0.0f, dd.z > 0.0f,
                                                         kBudget - it, nullptr
#ifdef VR_CRAWL_PROF
                                                         , &this->d_trips
#endif
                                                         );
                            if (n != 0u) {
                                oL = ax3<PL>(on); oM = ax3<PM>(on); oS = ax3<PS>(on);
                                gL = f2i(floorf(oL)); gM = f2i(floorf(oM)); gS = f2i(floorf(oS));
                                it += n;
                                this->count_ff(n);
                            }
                        }
                    }
                }
                CL = gL; CM = gM; CS = gS;
                AM = gM; AS = gS;
            }
            // ---- the mask words of all slots, requested together
            const uint32_t wA = word(gL, AM, AS), wB = word(gL, CM, CS), wC = word(CL, CM, CS);
            const Blk bA = mload(wA), bB = mload(wB), bC = mload(wC);
            // ---- evaluate the slots in the reference's order (A, B, C)
            const uint32_t iA = bit5(gL, AM, AS), iB = bit5(gL, CM, CS), iC = bit5(CL, CM, CS);
            const bool fA = (bA.x >> iA) & 1u, fB = (bB.x >> iB) & 1u, fC = (bC.x >> iC) & 1u;
            const bool eA = vA && (absent(bA) || fA), eB = vB && (absent(bB) || fB);
            stop = eA ? 0u : (eB ? 1u : ((absent(bC) || fC) ? 2u : 3u));
            bool hit = eA ? fA : (eB ? fB : fC);
            // the value index of the stopping slot only
            const uint32_t sx = eA ? bA.x : (eB ? bB.x : bC.x), sy = eA ? bA.y : (eB ? bB.y : bC.y);
            const uint32_t si = eA ? iA : (eB ? iB : iC);
            col = sy + __popc(sx & ((1u << si) - 1u));
            // huge grid coordinates (A or B outside the region; C is inside): the
            // general (aliasing) form, rare
            const bool inr = ex != kGo || !vA || ((((uint32_t)gL | (uint32_t)AM | (uint32_t)AS) < 64u) &&
                                                  (!vB || (((uint32_t)gL | (uint32_t)CM | (uint32_t)CS) < 64u)));
            if (COUNT && inr && ex == kGo) {
                const i3 P[3] = {to_i3(gL, AM, AS), to_i3(gL, CM, CS), to_i3(CL, CM, CS)};
                const Blk B[3] = {bA, bB, bC};
                const uint32_t W[3] = {wA, wB, wC};
                const bool V[3] = {vA, vB, true};
#pragma unroll
                for (uint32_t i = 0; i < 3u; ++i) {
                    if (!V[i] || i > stop) continue;
                    this->count(4);                   // doesVoxelSpaceExist
                    if (absent(B[i])) continue;
                    const uint32_t bit = this->in_cluster(P[i].x, P[i].y, P[i].z) & 31u;
                    this->count_bsearch(s.vcs_mask + (size_t)reg * 8192u + (W[i] & ~15u),
                                        B[i].y + __popc(B[i].x & ((1u << bit) - 1u)), (B[i].x >> bit) & 1u);
                }
            }
            if (__builtin_expect(__builtin_amdgcn_ballot_w64(!inr) != 0, 0)) {
                if (!inr) {
                    stop = 3u; hit = false; col = kEmpty;
                    const i3 P[3] = {to_i3(gL, AM, AS), to_i3(gL, CM, CS), to_i3(CL, CM, CS)};
                    const bool V[3] = {vA, vB, true};
#pragma unroll
                    for (uint32_t i = 0; i < 3u; ++i) {
                        if (!V[i] || stop != 3u) continue;
                        this->count(4);               // doesVoxelSpaceExist
                        const Blk b = i == 2u ? bC : this->mask_word(reg, P[i].x, P[i].y, P[i].z);
                        if (absent(b)) { stop = i; continue; }
                        if (((uint32_t)P[i].x | (uint32_t)P[i].y | (uint32_t)P[i].z) < 64u) {
                            const uint32_t bit = this->in_cluster(P[i].x, P[i].y, P[i].z) & 31u;
                            const bool f = (b.x >> bit) & 1u;
                            const uint32_t vi = b.y + __popc(b.x & ((1u << bit) - 1u));
                            if (COUNT) this->count_bsearch(this->masks(reg, this->cluster_id(P[i].x, P[i].y, P[i].z)), vi, f);
                            if (f) { stop = i; hit = true; col = vi; }
                        } else {
                            const uint32_t c = this->lookup_aliased(reg, P[i].x, P[i].y, P[i].z);
                            if (c != kEmpty) { stop = i; hit = true; col = c | 0x80000000u; }
                        }
                    }
                }
            }
            if (ex != kGo || hit) {
                why = ex != kGo ? ex : kHit;
                break;
            }
            if (jumping && stop == 3u) {
                // landed in an existing cluster without a hit: CONTINUE_VAL (:740-750)
                const float tNext = dv1((posL ? ceilf(oL) : floorf(oL)) - oL, dL);
                rL = oL + (tNext + kEps) * dL; rM = oM + (tNext + kEps) * dM; rS = oS + (tNext + kEps) * dS;
            }
            if (!jumping) {
                if (stop != 3u) {                    // an absent cluster: performVoxelSpaceJump
                    this->count(4);                  // its first existence test (this same cell)
                } else {                             // end of the iteration (:903-906)
                    oL = rL; oM = rM; oS = rS;
                    rL = rL + dL; rM = rM + dM; rS = rS + dS;
                }
                // g = the stopping slot (A, B or C), C at the end of the iteration
                gL = stop == 3u || stop == 2u ? CL : gL;
                gM = stop == 0u ? AM : CM;
                gS = stop == 0u ? AS : CS;
            }
            aM = f2i(rM) - gM;                       // (recomputed from unchanged values: same)
            aS = f2i(rS) - gS;
            jumping = stop != 3u;                    // jump on / start a jump; CONTINUE_VAL ends one
        }
        this->iters = it;
        if (why == kOver || why == kCrawl) {   // (tile pass: shade hands the pixel to the crawl pass)
            aborted = true;
            return false;
        }
        if (why == kHit) {
            // the hit as {colour, normal code, location in oo} from the loop's final
            // state: the caller makes the Hit after the original-DDA tail
            if (!SHADOW) {
                hcol = (col & 0x80000000u) ? (col & 0x7FFFFFFFu) : s.vcs_vals[col];
                // normal: axis a (x, y, z) with copysignf(1, -ds[a]): code = a | sign(ds[a]) << 2
                auto code = [](uint32_t a, float d) { return a | ((__float_as_uint(d) >> 31) << 2); };
                if (jumping) {                       // performVoxelSpaceJump's hit (getNormalFromTValues)
                    const auto d = xyz(dL, dM, dS);
                    hcode = code(nj, nj == 0u ? d.c[0] : (nj == 1u ? d.c[1] : d.c[2]));
                    oo = to_f3(oL, oM, oS);
                } else if (stop == 2u) {             // the L step's hit
                    hcode = code(PL, dL);
                    oo = to_f3(rL, rM, rS);
                } else {                             // a crossing's hit: getLocalHitLocation (:753-758)
                    const bool onM = (stop == 0u) == mfirst;
                    const float o = onM ? oM : oS, dd = onM ? dM : dS;
                    hcode = onM ? code(PM, dM) : code(PS, dS);
                    const float t = dd > 0.0f ? (ceilf(o) - o) / dd : (floorf(o) - o) / dd;
                    oo = to_f3(oL + t * dL, oM + t * dM, oS + t * dS);
                }
            }
            return true;
        }
        oo = to_f3(oL, oM, oS);     // Renderer.cuh:912 (direction of originalRay kept)
        tail = why == kTail;
        return false;
    }
    template <bool SHADOW>
    __device__ __forceinline__ bool grid_longest_vcs(f3& oo, f3 od, uint32_t reg, i3 cr, Hit& h) {
        bool hit = false, tail = false;
        uint32_t hcol = 0, hcode = 0;
        if (SHADOW) {
            // the light: its axis order, longest-axis direction and sign classes are
            // made on the host (kernel arguments: SGPRs), one pass
            f3 ds = ld3(v.Lw);
            // (held in VGPRs, though uniform: as SGPRs the direction and everything made from
            // it -- sign classes, plane offsets, the divisions' operands -- overflowed the
            // SGPR file, and the shadow loops restored spilled SGPRs with 16-22 v_readlane per
            // iteration; as VGPRs, 2-6: C3 per frame in flight 0.1888 -> 0.1863 ms, first
            // render 0.2815 -> 0.2758, profiles/r06/ab/ab_C3_vdir.txt)
            asm volatile("" : "+v"(ds.x), "+v"(ds.y), "+v"(ds.z));
            if (v.L_unit) {
                hit = walk_longest_vcs<SHADOW, true, 2, 1, 0>(oo, ds, v.L_cls, reg, tail, hcol, hcode);
            } else {
                switch (v.L_order) {
                    case 0: hit = walk_longest_vcs<SHADOW, false, 0, 1, 2>(oo, ds, v.L_cls, reg, tail, hcol, hcode); break;
                    case 1: hit = walk_longest_vcs<SHADOW, false, 0, 2, 1>(oo, ds, v.L_cls, reg, tail, hcol, hcode); break;
                    case 2: hit = walk_longest_vcs<SHADOW, false, 1, 0, 2>(oo, ds, v.L_cls, reg, tail, hcol, hcode); break;
                    case 3: hit = walk_longest_vcs<SHADOW, false, 1, 2, 0>(oo, ds, v.L_cls, reg, tail, hcol, hcode); break;
                    case 4: hit = walk_longest_vcs<SHADOW, false, 2, 0, 1>(oo, ds, v.L_cls, reg, tail, hcol, hcode); break;
                    default: hit = walk_longest_vcs<SHADOW, false, 2, 1, 0>(oo, ds, v.L_cls, reg, tail, hcol, hcode); break;
                }
            }
        } else {
            // the axis order of convertRayToLongestAxisDirection (Ray.cuh:19-71) and
            // the longest-axis direction k * d, k = 1 / |d_L|
            const float ax = fabsf(od.x), ay = fabsf(od.y), az = fabsf(od.z);
            const uint32_t order =
                (ax > ay && ax > az) ? (ay > az ? 0u : 1u) : (ay > az ? (ax > az ? 2u : 3u) : (ax > ay ? 4u : 5u));
            const float k = 1.0f / (order < 2u ? ax : (order < 4u ? ay : az));
            const f3 ds = scl(k, od);
            const uint32_t cls = (uint32_t)(ds.x > 0.0f) | (uint32_t)(ds.x < 0.0f) << 1 | (uint32_t)(ds.y > 0.0f) << 2 |
                                 (uint32_t)(ds.y < 0.0f) << 3 | (uint32_t)(ds.z > 0.0f) << 4 | (uint32_t)(ds.z < 0.0f) << 5;
            const uint32_t key = order | cls << 3;
            bool todo = true;
            while (todo) {                            // one pass per (order, signs) present in the wave
                const uint32_t pat = __builtin_amdgcn_readfirstlane(key);
                if (key == pat) {
                    todo = false;
                    const uint32_t pc = pat >> 3;
                    switch (pat & 7u) {
                        case 0: hit = walk_longest_vcs<SHADOW, false, 0, 1, 2>(oo, ds, pc, reg, tail, hcol, hcode); break;
                        case 1: hit = walk_longest_vcs<SHADOW, false, 0, 2, 1>(oo, ds, pc, reg, tail, hcol, hcode); break;
                        case 2: hit = walk_longest_vcs<SHADOW, false, 1, 0, 2>(oo, ds, pc, reg, tail, hcol, hcode); break;
                        case 3: hit = walk_longest_vcs<SHADOW, false, 1, 2, 0>(oo, ds, pc, reg, tail, hcol, hcode); break;
                        case 4: hit = walk_longest_vcs<SHADOW, false, 2, 0, 1>(oo, ds, pc, reg, tail, hcol, hcode); break;
                        default: hit = walk_longest_vcs<SHADOW, false, 2, 1, 0>(oo, ds, pc, reg, tail, hcol, hcode); break;
                    }
                }
            }
        }
        if (aborted) return false;
        // the original-DDA tail; a shadow walk of an equal-component light takes the
        // one-division loop (grid_original's EQ)
        if (tail)
            return grid_original_rt(oo, od, reg, cr, h, SHADOW, SHADOW && VR_LONG_TAIL_EQ && v.L_eq, nullptr, nullptr,
                                    VR_LONG_TAIL_GENERIC);
        if (!SHADOW && hit) {
            const float one = (hcode & 4u) ? 1.0f : -1.0f;
            const uint32_t a = hcode & 3u;
            h.col = hcol;
            h.nc = this->ncode(a, one);
            h.so = oo;
            h.region = cr;
            h.longest = true;
        }
        return hit;
    }

    // rayMarchVoxelScene (Renderer.cuh:338-434) / rayMarchVoxelSceneLongestAxis (:917-1010).
    template <int ALGO>
    __device__ __forceinline__ bool primary(f3 wo, f3 wd, Hit& h) {
        f3 tr = ld3(v.translation);
        f3 so = scl(v.scale_f, sub(wo, tr));      // Ray::convertRayToLocalSpace (Ray.cuh:14-17)
        f3 d = wd;
        // the ray's reciprocals, made once for every division by d in the entry clip
        // (div_fast) and, cuckoo store only (see kFastSetup), in the region walks
        const Rcp rc[3] = {rcp_setup(d.x), rcp_setup(d.y), rcp_setup(d.z)};
        i3 cr{f2i(floorf(so.x / 64.0f)), f2i(floorf(so.y / 64.0f)), f2i(floorf(so.z / 64.0f))};
        VR_DIAG_COUNT(14);                            // primary() calls
        auto cyc = this->cycle_start(cr, so);     // (kExact only: dead code in the tile pass)
        while (!in_scene(cr)) {                   // entry clip (:349-373)
            if (!tick()) return false;
            VR_DIAG_COUNT(15);
            int32_t hi = (int32_t)(s.D + (uint32_t)s.min_coord), lo = s.min_coord;
            int32_t nx = d.x < 0.0f ? hi : lo, ny = d.y < 0.0f ? hi : lo, nz = d.z < 0.0f ? hi : lo;
            const float ax = (float)(nx * kBlock) - so.x, ay = (float)(ny * kBlock) - so.y,
                        az = (float)(nz * kBlock) - so.z;
            float tX = div_fast(ax, rc[0]), tY = div_fast(ay, rc[1]), tZ = div_fast(az, rc[2]);
            // (a numerator is never -0 here; +0 divides exactly)
            const bool fast = (__float_as_uint(ax) == 0u || div_fast_ok(ax, rc[0])) &&
                              (__float_as_uint(ay) == 0u || div_fast_ok(ay, rc[1])) &&
                              (__float_as_uint(az) == 0u || div_fast_ok(az, rc[2]));
            if (__builtin_expect(__builtin_amdgcn_ballot_w64(!fast) != 0, 0)) {
                tX = fast ? tX : ax / d.x;
                tY = fast ? tY : ay / d.y;
                tZ = fast ? tZ : az / d.z;
            }
            if (tX <= 0.0f) tX = kInf;
            if (tY <= 0.0f) tY = kInf;
            if (tZ <= 0.0f) tZ = kInf;
            float tMin = fminf(tX, fminf(tY, tZ));
            if (tMin == kInf) return false;
            so = add(so, scl(tMin + kEps, d));
            cr = i3{f2i(floorf(so.x / 64.0f)), f2i(floorf(so.y / 64.0f)), f2i(floorf(so.z / 64.0f))};
            if (kExact && this->cycle_step(cyc, cr, so)) { aborted = true; return false; }   // never ends
        }
        f3 o = sub(so, mk((float)(cr.x * kBlock), (float)(cr.y * kBlock), (float)(cr.z * kBlock)));
        return primary_regions<ALGO>(o, d, cr, h, nullptr, rc);
    }
    // The region walk of rayMarchVoxelScene(LongestAxis) (:376-433); rs (crawl
    // pass): first finish the region walk a deferral record left at its crawl.
    template <int ALGO>
    __device__ __forceinline__ bool primary_regions(f3 o, f3 d, i3 cr, Hit& h, const uint32_t* rs,
                                                    const Rcp* rc = nullptr) {
        if (CRAWL && rs != nullptr) {
            const bool hit = grid_original_rt(o, d, this->region_at_nocount(cr), cr, h, false, false, rs);
            if (aborted) return false;
            if (hit) return true;
            advance_region(cr, o);
        }
        auto cyc = this->cycle_start(cr, o);
        while (in_scene(cr)) {
            // (VCS longest axis: the direction is made opaque per region round, so the walk's
            // per-direction values -- longest-axis frame, sign classes, the tail's plane signs --
            // are made inside the round instead of hoisted out of it and kept live through every
            // walk, which spilled them: VR_LONG_REMAT)
            if (kRematDir && ALGO == ALGO_LONGEST) asm volatile("" : "+v"(d.x), "+v"(d.y), "+v"(d.z));
            if (!tick()) return false;
            VR_DIAG_COUNT(10);                         // primary region rounds
            uint32_t reg = region_at(cr);
            auto cyc1 = this->cycle_start(cr, o);
            while (reg == kNone) {
                if (!tick()) return false;
                VR_DIAG_COUNT(11);                     // null-region skips
                if (!this->template skip_null<false>(cr, o, d, reg)) return false;
                // kExact: a loop whose state repeats never ends (the reference never
                // returns); the VCS tile pass hands such pixels over through its budget
                if (kExact && this->cycle_step(cyc1, cr, o)) { aborted = true; return false; }
            }
            bool hit = ALGO == ALGO_ORIGINAL ? grid_original<false>(o, d, reg, cr, h, nullptr, rc)
                                             : (STORE == STORE_VCS ? grid_longest_vcs<false>(o, d, reg, cr, h)
                                                                   : grid_longest<false>(o, d, reg, cr, h));
            if (aborted) return false;
            if (hit) return true;
            advance_region(cr, o);
            if (kExact && this->cycle_step(cyc, cr, o)) { aborted = true; return false; }
        }
        return false;
    }

    // isInShadowOriginalRayMarch (Renderer.cuh:174-235) /
    // isInShadowRayMarchVoxelSceneLongestAxis (:633-694).
    template <bool LONGEST, bool EQ = false>
    __device__ __forceinline__ bool shadow(f3 o, i3 cr, const uint32_t* rs = nullptr) {
        f3 d = ld3(v.L);
        // the light's reciprocals, made on the host (uniform: SGPRs, no VGPRs)
        const bool lf = v.L_fast != 0u;
        const Rcp rc[3] = {Rcp{d.x, v.Lr[0], lf}, Rcp{d.y, v.Lr[1], lf}, Rcp{d.z, v.Lr[2], lf}};
        Hit dummy;
        if (CRAWL && rs != nullptr) {            // resume a deferred crawl (as primary_regions)
            const bool hit = grid_original_rt(o, d, this->region_at_nocount(cr), cr, dummy, true, EQ, rs);
            if (aborted) return false;
            if (hit) return true;
            advance_region(cr, o);
        }
        auto cyc = this->cycle_start(cr, o);
        while (in_scene(cr)) {
            if (kRematDir && LONGEST) asm volatile("" : "+s"(d.x), "+s"(d.y), "+s"(d.z));   // (see primary_regions; uniform)
            if (!tick()) return false;
            VR_DIAG_COUNT(12);                         // shadow region rounds
            uint32_t reg = region_at(cr);
            auto cyc1 = this->cycle_start(cr, o);
            while (reg == kNone) {
                if (!tick()) return false;
                VR_DIAG_COUNT(13);
                if (!this->template skip_null<!LONGEST>(cr, o, d, reg)) return false;
                if (kExact && this->cycle_step(cyc1, cr, o)) { aborted = true; return false; }   // (as above)
            }
            bool hit = LONGEST ? (STORE == STORE_VCS ? grid_longest_vcs<true>(o, d, reg, cr, dummy)
                                                     : grid_longest<true>(o, d, reg, cr, dummy))
                               : grid_original<true, EQ>(o, d, reg, cr, dummy, nullptr, rc);
            if (aborted) return false;
            if (hit) return true;
            advance_region(cr, o);
            if (kExact && this->cycle_step(cyc, cr, o)) { aborted = true; return false; }
        }
        return false;
    }
};

// calculateWorldRay (Renderer.cuh:1013-1022) + Camera::generateRay (Camera.cuh:25-29)
// for pixel (x, local row l); false when the row is outside the frame.
// FAST (cuckoo store, see Walker::kFastSetup): divisions with hoisted reciprocals.
template <bool FAST>
__device__ __forceinline__ bool pixel_ray(const KView& v, uint32_t x, uint32_t l, f3& ro, f3& rd) {
    // band = l / band_rows: q0 = mulhi(l, floor(2^32 / band_rows)) is q or q - 1 (see FastMod)
    const uint32_t q0 = __umulhi(l, v.band_minv), r0 = l - q0 * v.band_rows;
    const bool up = r0 >= v.band_rows;
    const uint32_t band = q0 + (up ? 1u : 0u), in_band = up ? r0 - v.band_rows : r0;
    const uint32_t y = v.row0 + (band * v.nranks + v.rank) * v.band_rows + in_band;
    if (y >= v.row_limit) return false;
    if (v.tile_cols) {
        // 2-D tile deal (uniform branch): local column -> frame column (vr_internal.h KView)
        const uint32_t j0 = __umulhi(x, v.tile_minv), r1 = x - j0 * v.tile_cols;
        const bool up1 = r1 >= v.tile_cols;
        const uint32_t j = j0 + (up1 ? 1u : 0u), in_blk = up1 ? r1 - v.tile_cols : r1;
        const uint32_t off = (v.col_rank + v.col_R - (v.col_stride * (band % v.col_R)) % v.col_R) % v.col_R;
        x = (j * v.col_R + off) * v.tile_cols + in_blk;
        if (x >= v.W) return false;
    }
    if (!FAST) {
        float u = ((float)x + 0.5f) / (float)v.W;
        float vv = ((float)(v.H - y) + 0.5f) / (float)v.H;
        ro = add(add(ld3(v.llc), scl(u, ld3(v.hor))), scl(vv, ld3(v.ver)));
        rd = unit(sub(ro, ld3(v.org)));
        return true;
    }
    // correctly rounded divisions by W, H (in [1, 65536]) and |ro - eye| with
    // hoisted reciprocals (div_fast; its domain holds for u and v: numerators
    // in [0.5, 65536])
    const Rcp rW = rcp_setup((float)v.W), rH = rcp_setup((float)v.H);
    float u = div_fast((float)x + 0.5f, rW);
    float vv = div_fast((float)(v.H - y) + 0.5f, rH);
    ro = add(add(ld3(v.llc), scl(u, ld3(v.hor))), scl(vv, ld3(v.ver)));
    const f3 c = sub(ro, ld3(v.org));                  // Vector3::normalize (Vector3.cuh:162, :79)
    const float len = sqrtf(c.x * c.x + c.y * c.y + c.z * c.z);
    const Rcp rl = rcp_setup(len);
    auto okn = [&](float n) { return __float_as_uint(n) == 0u || div_fast_ok(n, rl); };
    rd = f3{div_fast(c.x, rl), div_fast(c.y, rl), div_fast(c.z, rl)};
    if (!(okn(c.x) && okn(c.y) && okn(c.z))) rd = f3{c.x / len, c.y / len, c.z / len};
    return true;
}

// applyLighting at the primary hit (Renderer.cuh:249-258; regionWorldPosition :413)
// times !shadow (:315,737,821): the pixel's colour.
template <int STORE, bool COUNT, bool CRAWL>
__device__ __forceinline__ uint32_t light_and_shadow(Walker<STORE, COUNT, CRAWL>& w, const KView& v, const Hit& h) {
    bool sh = false;
    const f3 rwp = add(ld3(v.translation), mk((float)(h.region.x * kBlock), (float)(h.region.y * kBlock),
                                              (float)(h.region.z * kBlock)));
    const uint32_t lit = w.lighting(h.col, h.nc, rwp, h.so);
    if (v.use_shadows) {
        VR_DIAG_COUNT(16);                             // shadow walks started
        w.lit_saved = lit;
        const bool eq = v.L[0] == v.L[1] && v.L[1] == v.L[2];
        if (h.longest) {
            w.ctx = 2u;
            sh = w.template shadow<true>(h.so, h.region);
        } else {
            sh = eq ? w.template shadow<false, true>(h.so, h.region) : w.template shadow<false>(h.so, h.region);
        }
    }
    return lit * (uint32_t)!sh;
}

// Tile pass: hand this lane's pixel (tile_pixels) to the crawl pass, to be walked there
// from its start (a record with flag 4).  Returns what the tile pass writes for
// it: 0, or kDeferMarker when the list is full (the crawl pass then finds the
// pixel by the marker).
__device__ __forceinline__ uint32_t defer_rewalk(const KView& v) {
    const uint32_t idx = atomicAdd(v.defer, 1u);
    deferral_report(v);
    if (idx < v.defer_cap) {
        uint32_t* r = v.defer + 4 + (size_t)idx * kDeferRecWords;
        r[0] = tile_pixels()[threadIdx.x];
        r[1] = 4u;
        r[8] = v.launch_id;
        return 0u;
    }
    atomicAdd(v.defer + 2, 1u);
    return kDeferMarker;
}

// The crawl pass's LDS for one record lane: its cluster-bit slot.
struct CrawlLds {
    uint32_t* lbm = nullptr;
};
template <class W>
__device__ __forceinline__ void attach(W& w, const CrawlLds* cl) {
    if (!cl) return;
    w.lbm = cl->lbm;
}

// The body of rayMarchSceneOriginal / rayMarchSceneJumpAxis (Renderer.cuh:1033-1063)
// for pixel (x, local row l): colour, algorithmic bytes (+4 for the pixel write).
// Tile pass (!CRAWL): a pixel deferred to the crawl pass -- a crawl record, or a
// walk longer than kTileBudget iterations -- comes back with 0 bytes (the crawl
// pass writes and counts it).  Crawl pass: a walk that never finishes (the
// reference would loop forever) is 0 with only the pixel write counted, as in
// the oracle.
template <int STORE, int ALGO, bool COUNT, bool CRAWL>
__device__ __forceinline__ uint32_t shade(const KScene& s, const KView& v, uint32_t x, uint32_t l,
                                          uint32_t& bytes, uint32_t* iters = nullptr, uint2* ff = nullptr,
                                          uint32_t* dg = nullptr, const CrawlLds* cl = nullptr) {
    uint32_t col = 0;
    bytes = 0;
    if (ff) *ff = uint2{0u, 0u};
    f3 ro, rd;
    if (pixel_ray<true>(v, x, l, ro, rd)) {
        Walker<STORE, COUNT, CRAWL> w(s, v);
        attach(w, cl);
        Hit h;
        const bool hit = w.template primary<ALGO>(ro, rd, h);
        if (!CRAWL && v.pcost) tile_prim()[threadIdx.x] = w.iters;   // (the lane order's primary walk length)
        if (hit) col = light_and_shadow(w, v, h);
        if (iters) *iters = w.iters;              // the walk's length (the work order's cost)
        bytes = w.bytes + 4u;                     // + the pixel write
        if (ff) *ff = uint2{w.ff, w.nl};
#ifdef VR_CRAWL_PROF
        if (dg) { dg[0] = w.iters - w.ff; dg[1] = w.d_runs; dg[2] = w.d_trips; }
#endif
        if (w.aborted) {
            col = 0;
            if (ff) *ff = uint2{0u, 0u};
            if (Walker<STORE, COUNT, CRAWL>::kExact) {
                bytes = 4u;
            } else {
                bytes = 0u;
                if (w.iters != kDeferredIters) col = defer_rewalk(v);
            }
        }
    }
    return col;
}

// The crawl pass's pixel: the walk a deferral record `r` left at its crawl,
// finished from there (its iterations and bytes so far are the record's).
template <int STORE, int ALGO, bool COUNT>
__device__ __forceinline__ uint32_t shade_resume(const KScene& s, const KView& v,
                                                 const uint32_t* r, uint32_t& bytes, uint2& ff,
                                                 uint32_t* dg = nullptr, const CrawlLds* cl = nullptr) {
    const uint32_t x = r[0] & 0xFFFFu, l = r[0] >> 16;
    Walker<STORE, COUNT, true> w(s, v);
    attach(w, cl);
    w.iters = r[9];
    w.bytes = r[10];
    const f3 o{__uint_as_float(r[2]), __uint_as_float(r[3]), __uint_as_float(r[4])};
    const i3 cr{(int32_t)r[5], (int32_t)r[6], (int32_t)r[7]};
    uint32_t col = 0;
    if (!(r[1] & 1u)) {                           // the primary walk crawled
        f3 ro, rd;
        pixel_ray<true>(v, x, l, ro, rd);
        Hit h;
        if (w.template primary_regions<ALGO>(o, rd, cr, h, r)) col = light_and_shadow(w, v, h);
    } else {                                      // the shadow walk crawled
        const bool eq = v.L[0] == v.L[1] && v.L[1] == v.L[2];
        bool sh;
        if (r[1] & 2u) sh = eq ? w.template shadow<true, true>(o, cr, r) : w.template shadow<true>(o, cr, r);
        else sh = eq ? w.template shadow<false, true>(o, cr, r) : w.template shadow<false>(o, cr, r);
        col = r[18] * (uint32_t)!sh;
    }
    bytes = w.bytes + 4u;
    ff = uint2{w.ff, w.nl};
#ifdef VR_CRAWL_PROF
    if (dg) { dg[0] = w.iters - r[9] - w.ff; dg[1] = w.d_runs; dg[2] = w.d_trips; }
#endif
    if (w.aborted) {                              // never finishes (see shade)
        col = 0;
        bytes = 4u;
        ff = uint2{0u, 0u};
    }
    return col;
}

__device__ __forceinline__ void add_bytes(const KView& v, uint32_t lane, unsigned long long b) {
    for (int off = 32; off > 0; off >>= 1) b += __shfl_down(b, off, 64);   // one atomic per wave
    if (lane == 0 && b) atomicAdd(v.bytes, b);
}
// the crawl pass's existence reads credited without a load (KView::stats): n crawl
// iterations fast-forwarded in closed form, m skip steps answered from the LDS cluster bits
__device__ __forceinline__ void add_ff(const KView& v, uint32_t lane, unsigned long long n, unsigned long long m) {
    for (int off = 32; off > 0; off >>= 1) {
        n += __shfl_down(n, off, 64);
        m += __shfl_down(m, off, 64);
    }
    if (lane == 0 && (n | m) && v.stats) {
        atomicAdd(v.stats, n);
        atomicAdd(v.stats + 1, 4ull * (n + m));
    }
}

// Tile pass: one lane per pixel, one wave per 8x8 tile, kTilesX x kTilesY tiles per workgroup.
#ifndef VR_ORIG_WAVES
#define VR_ORIG_WAVES 7
#endif
#ifndef VR_LONG_WAVES
#define VR_LONG_WAVES 6
#endif
// HI: the occupancy for frames in flight, where the other frame's waves fill the tail and
// the pass's throughput counts: one wave per SIMD more for the cuckoo walk (latency-bound
// on its random slot loads: C4 0.0861 -> 0.0855 ms per frame, but 0.1229 -> 0.1246 alone)
// and the longest-axis walk (C3 0.2311 -> 0.2289 per frame, 0.2815 -> 0.2862 alone),
// profiles/r04/ab_orig_waves_C4.txt, ab_long_waves_C3.txt.  The host picks HI for a launch
// whose device is still running another stream's (the AUTO schedule's test).
// (Round 6: 7 for the cuckoo walk too.  Since its shadow walks answer a hit from the filter
// alone -- no table reads -- the 8-wave variant's SGPRs spill into VGPR lanes, 16 v_readlane
// per loop iteration: C4 per frame in flight 0.0500 -> 0.0746 ms at 8 waves, 0.0466 at 7,
// profiles/r06/ab_C4_*.txt.)
#ifndef VR_ORIG_WAVES_HI
#define VR_ORIG_WAVES_HI 7
#endif
// (Round 6: 6 for the VCS longest-axis walk too, the lone kernel's, so frames in flight run
// that kernel.  With its shadow direction in VGPRs and the direction made per region round
// the 7-wave variant spills 30 VGPRs and 212 SGPRs: C3 per frame in flight 0.1851 -> 0.1835 ms
// at 6, profiles/r06/ab/ab_C3_waves_hi.txt.)
#ifndef VR_LONG_WAVES_HI
#define VR_LONG_WAVES_HI 6
#endif
// (a variant equal to the lone one is not built: both launch the lone kernel)
constexpr bool kLongHiVariant = VR_LONG_WAVES_HI != VR_LONG_WAVES;
constexpr bool kOrigHiVariant = VR_ORIG_WAVES_HI != VR_ORIG_WAVES;
template <int ALGO, bool HI> struct TileWaves {
    static constexpr int value = ALGO == ALGO_ORIGINAL ? (HI ? VR_ORIG_WAVES_HI : VR_ORIG_WAVES)
                                                       : (HI ? VR_LONG_WAVES_HI : VR_LONG_WAVES);
};
static_assert(kTilesX * kTilesY == kWavesPerTileGroup, "cost layout (vr_internal.h)");
template <int STORE, int ALGO, bool COUNT, bool HI = false>
__global__ __launch_bounds__(64 * kTilesX * kTilesY, (TileWaves<ALGO, HI>::value)) void march_kernel(KScene s, KView v) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t x, l;
    lane_pixel(v, x, l);
    tile_pixels()[threadIdx.x] = (l << 16) | x;     // (read back only by this lane: no barrier)
    if (v.pcost) tile_prim()[threadIdx.x] = 0u;
    uint32_t bytes = 0, iters = 0;
    if (x < v.LW && l < v.local_rows) {
        // (&iters unconditionally: a pointer chosen by `v.cost ? &iters : nullptr` keeps
        // iters in scratch -- a store and a reload per lane, 8 MB of WRITE_SIZE per C2 launch)
        const uint32_t c = shade<STORE, ALGO, COUNT, false>(s, v, x, l, bytes, &iters);
        // (x and l again from LDS, so they are not live through the walk; the empty asm
        // keeps the compiler from forwarding the stored value instead)
        asm volatile("" ::: "memory");
        const uint32_t p = tile_pixels()[threadIdx.x];
        const size_t at = (size_t)(p >> 16) * v.LW + (p & 0xFFFFu);
        v.out[at] = c;
        if (v.pcost) {                            // the pixel's walk lengths, for the next lane order
            const uint32_t p0 = tile_prim()[threadIdx.x];
            v.pcost[at] = min(p0, 0xFFFFu) << 16 | min(iters - p0, 0xFFFFu);
        }
    }
    if (COUNT) add_bytes(v, lane, bytes);
    if (v.cost) {                                  // the wave's walk length, for the next work order
        for (int off = 32; off > 0; off >>= 1) iters = max(iters, (uint32_t)__shfl_xor((int)iters, off, 64));
        if (lane == 0) {
            uint32_t bx, by;
            tile_group(v, bx, by);
            v.cost[(by * gridDim.x + bx) * kWavesPerTileGroup + wave] = iters;
        }
    }
}

// The lane order of one pixel block (see lane_pixel): its kLanePixels pixels ranked by the
// walk length an earlier launch recorded (KView::pcost), heaviest first, one thread per pixel.
// Keys (length << log2(kLanePixels) | pixel) are all distinct.  Each wave sorts its 64 keys
// with a bitonic network of lane shuffles (no barriers); a key's rank in the block is its
// rank in its wave plus, for each other wave, the number of that wave's sorted keys above it
// (independent binary searches in LDS).  The block's slots are gathered in LDS and stored as
// words.  With cost non-null the kernel also writes each wave's walk length under the new
// lane order -- KView::cost's layout; max(primary) + max(shadow) over the wave's pixels, what
// the wave runs; blocks cut by the grid's edge keep the 8x8 tiles and write each tile's -- so
// the work order made from them next matches the lane order.
constexpr uint32_t kLaneShift = kLaneBlock == 16 ? 8u : 10u;
__global__ __launch_bounds__(kLanePixels) void perm_kernel(const uint32_t* __restrict__ pcost, uint32_t LW,
                                                           uint32_t rows, uint32_t gx, uint32_t gy,
                                                           uint8_t* __restrict__ perm, uint32_t* __restrict__ cost) {
    constexpr uint32_t kWaves = kLanePixels / 64u, kTiles = (kLaneBlock / 8u) * (kLaneBlock / 8u);
    __shared__ uint32_t sorted[kLanePixels];
    __shared__ __attribute__((aligned(16))) PermT slots[kLanePixels];
    __shared__ uint32_t wmax[2u * kWaves];   // per wave slot (or 8x8 tile): max primary, max shadow
    __shared__ uint32_t ps[kLanePixels];     // the pixels' walk lengths (cost writes only)
    static_assert(kTiles == kWaves, "one 8x8 tile per wave slot");
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    const uint32_t nbx = (gx + kLbX - 1u) / kLbX, BX = blockIdx.x % nbx, BY = blockIdx.x / nbx;
    const uint32_t px = t % kLaneBlock, py = t / kLaneBlock;
    const uint32_t x = BX * kLaneBlock + px, l = BY * kLaneBlock + py;
    // a pixel's weight: a wave runs its primary walks until the slowest ends, then its shadow
    // walks, so it costs max(primary) + max(shadow) over its lanes; max(p, s) + (p + s) / 8
    // groups lanes best of the weights tried on the oracle's C2 counts (1.4 % fewer
    // wave-iterations than p + s, profiles/r05/lane_sort_sim.py)
    uint32_t p = 0, s = 0;
    if (x < LW && l < rows) {
        const uint32_t w = pcost[(size_t)l * LW + x];
        p = w >> 16;
        s = w & 0xFFFFu;
    }
    const uint32_t c = min(max(p, s) + ((p + s) >> 3), (1u << (32u - kLaneShift)) - 1u);
    if (cost) {
        if (t < 2u * kWaves) wmax[t] = 0u;
        ps[t] = p << 16 | s;
    }
    if ((BX + 1u) * kLbX > gx || (BY + 1u) * kLbY > gy) {
        if (cost) {                 // the block's 8x8 tiles that exist
            __syncthreads();
            const uint32_t ti = (py >> 3) * (kLaneBlock / 8u) + (px >> 3);
            atomicMax(&wmax[ti], p);
            atomicMax(&wmax[kWaves + ti], s);
            __syncthreads();
            if (t < kTiles) {
                const uint32_t tx = t % (kLaneBlock / 8u), ty = t / (kLaneBlock / 8u);
                const uint32_t col = BX * kLbX + tx / kTilesX, row = BY * kLbY + ty;
                if (col < gx && row < gy)
                    cost[(row * gx + col) * kWavesPerTileGroup + tx % kTilesX] = wmax[t] + wmax[kWaves + t];
            }
        }
        return;
    }
    uint32_t key = (c << kLaneShift) | t;
    for (uint32_t size = 2; size <= 64u; size <<= 1) {
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            const uint32_t other = (uint32_t)__shfl_xor((int)key, (int)stride, 64);
            const bool keep_max = ((lane & stride) == 0u) == ((lane & size) == 0u);
            key = keep_max ? max(key, other) : min(key, other);
        }
    }
    sorted[t] = key;                // lane i of wave w: the wave's i-th largest key
    __syncthreads();
    uint32_t rank = lane;
#pragma unroll
    for (uint32_t o = 1; o < kWaves; ++o) {
        const uint32_t* sw = sorted + (((wave + o) % kWaves) << 6);
        uint32_t lo = 0;            // the number of sw's keys above key (sw descending)
#pragma unroll
        for (uint32_t step = 32; step > 0; step >>= 1)
            if (sw[lo + step - 1u] > key) lo += step;
        rank += lo + (sw[63] > key ? 1u : 0u);    // (all 64 above: lo stops at 63)
    }
    const uint32_t pix = key & (kLanePixels - 1u);
    slots[rank] = (PermT)pix;
    if (cost) {                     // the walk lengths of the pixel this thread's key carries
        const uint32_t w = ps[pix];
        atomicMax(&wmax[rank >> 6], w >> 16);
        atomicMax(&wmax[kWaves + (rank >> 6)], w & 0xFFFFu);
    }
    __syncthreads();
    if (cost && t < kWaves) {
        const uint32_t g = t / kTilesX;
        const uint32_t col = BX * kLbX + g % kLbX, row = BY * kLbY + g / kLbX;
        cost[(row * gx + col) * kWavesPerTileGroup + t % kTilesX] = wmax[t] + wmax[kWaves + t];
    }
    constexpr uint32_t kWords = kLanePixels * sizeof(PermT) / 4u;
    uint32_t* out = reinterpret_cast<uint32_t*>(perm + (size_t)blockIdx.x * kLanePixels * sizeof(PermT));
    if (t < kWords) out[t] = reinterpret_cast<const uint32_t*>(slots)[t];
}

// Heaviest tiles first: a counting sort of the tile groups by the cost an earlier
// launch recorded (the slower of a workgroup's waves; classes of 4 loop iterations,
// class 0 the heaviest, >= 508), in one workgroup with LDS counters.  The order within
// a class is whatever the atomics make it: any permutation renders the same pixels.
// (A stable sort -- grid order within a class, one ballot per class present per 64
// groups -- took ~4x longer and gained nothing, profiles/r03/ab_order_C2_C3.txt.)
constexpr uint32_t kOrderClasses = 128;
__global__ __launch_bounds__(1024) void order_kernel(const uint32_t* __restrict__ cost, uint32_t n, uint32_t columns,
                                                     uint32_t* __restrict__ order) {
    __shared__ uint32_t cnt[kOrderClasses];
    if (threadIdx.x < kOrderClasses) cnt[threadIdx.x] = 0u;
    __syncthreads();
    auto cls = [&](uint32_t i) {
        uint32_t c = 0;
#pragma unroll
        for (uint32_t w = 0; w < kWavesPerTileGroup; ++w) c = max(c, cost[i * kWavesPerTileGroup + w]);
        return kOrderClasses - 1u - min(kOrderClasses - 1u, c >> 2);
    };
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&cnt[cls(i)], 1u);
    __syncthreads();
    if (threadIdx.x == 0) {                        // exclusive prefix sum
        uint32_t run = 0;
        for (uint32_t k = 0; k < kOrderClasses; ++k) {
            const uint32_t c = cnt[k];
            cnt[k] = run;
            run += c;
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) order[atomicAdd(&cnt[cls(i)], 1u)] = (i / columns) << 16 | (i % columns);
}

// Crawl pass: the deferred pixels of this launch, one per lane, with the
// exact crawl fast-forward; the last workgroup resets the slot for reuse.
#ifndef VR_CRAWL_RPW
#define VR_CRAWL_RPW 4
#endif
constexpr uint32_t kCrawlRpw = VR_CRAWL_RPW;
#ifndef VR_CRAWL_MAX_RPW
#define VR_CRAWL_MAX_RPW 32
#endif
constexpr uint32_t kCrawlMaxRpw = VR_CRAWL_MAX_RPW;     // records per wave with an LDS bitmap slot
// Workgroup shape: 2 waves (as the tile pass).  (Round 4 measured an opt-in mode that cached
// the scene's whole region table and cluster bits in each 8-wave workgroup's LDS: no faster
// alone, slower in flight, profiles/r04/crawl/scene_lds_ab.txt -- removed in round 5.)
constexpr uint32_t kCrawlWaves = 2;
// LDS (16-B aligned carve-outs, cdna_hip_programming.md Guideline 17):
//   [0, 16)   record count, overflow count
//   then      16 words (a region's cluster-existence bits) per record lane, kCrawlMaxRpw per wave
constexpr uint32_t kCrawlLdsWords = 4u + kCrawlWaves * kCrawlMaxRpw * 16u;
template <int STORE, int ALGO, bool COUNT>
__global__ __launch_bounds__(64 * kCrawlWaves) void crawl_kernel(KScene s, KView v) {
    __shared__ __attribute__((aligned(16))) uint32_t dyn[kCrawlLdsWords];
    if (threadIdx.x == 0) {
        dyn[0] = v.defer[0];
        dyn[1] = v.defer[2];
    }
    __syncthreads();
    const uint32_t total = dyn[0], overflow = dyn[1];
    // what this launch deferred, for the host's grid size of later launches (a hint only)
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (v.defer_stat) *v.defer_stat = total + overflow;
        if (v.slot_stat) *reinterpret_cast<uint2*>(v.slot_stat) = uint2{v.launch_id, total + overflow};
    }
    if (total == 0u && overflow == 0u) return;   // nothing deferred (the usual case): no reset needed
    const uint32_t n = min(total, v.defer_cap);
    CrawlLds cl;
    unsigned long long bytes = 0, ffs = 0, nls = 0;
    // kCrawlRpw records per wave at a time (lanes 0 .. kCrawlRpw-1): each record is a long
    // chain of dependent iterations, and the lanes of a wave take different paths through
    // the walk, so fewer lanes per wave -- spread over more waves -- finish sooner
    // (v.crawl_rpw: the host's choice per launch -- 4 for a lone frame, whose time is the
    // longest record's chain; 8 with frames in flight, where the pass's issue cycles count:
    // C5 0.6707 -> 0.6514 ms per frame, profiles/r03/rpw_deep/; 32 since round 6, never slower
    // and in some runs 4 % faster, vr_host.cpp crawl_rpw_in_flight)
    const uint32_t rpw = v.crawl_rpw ? v.crawl_rpw : kCrawlRpw;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, wlane = threadIdx.x & 63u;
    const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
    if (STORE == STORE_VCS && s.vcs_cbits && rpw <= kCrawlMaxRpw && wlane < rpw)
        cl.lbm = dyn + 4 + ((threadIdx.x >> 6) * kCrawlMaxRpw + wlane) * 16u;
    for (uint32_t i = wave * rpw + wlane; wlane < rpw && i < n; i += nwaves * rpw) {
        uint32_t* r = v.defer + 4 + (size_t)i * kDeferRecWords;
        // (a record of another launch -- one whose crawl pass the host skipped, believing its
        // view defers nothing -- is not this frame's: never shade it into this frame; its count
        // in this pass's report stops the skipping)
        if (r[8] != v.launch_id) continue;
        uint32_t b;
        const uint32_t x = r[0] & 0xFFFFu, l = r[0] >> 16;
        // The crawl iteration's voxel q (see crawl_voxel), recovered from the stepped
        // position and the walk's direction (the pixel's ray, or the light for a shadow
        // walk) into record words 15-17; if it cannot be, the pixel is walked from its
        // start (as for every record under VR_KERNEL_TILE_REWALK, flag 4).
        bool amb = (r[1] & 4u) != 0u;
        if (!amb) {
            f3 d = ld3(v.L);
            if (!(r[1] & 1u)) {
                f3 ro;
                pixel_ray<true>(v, x, l, ro, d);
            }
            const f3 o{__uint_as_float(r[2]), __uint_as_float(r[3]), __uint_as_float(r[4])};
#pragma unroll 1
            for (uint32_t a = 0; a < 3u; ++a) {
                int32_t qa;
                amb |= !crawl_voxel(comp(o, a), kEps * comp(d, a), qa);
                r[15 + a] = (uint32_t)qa;
            }
        }
        uint2 f{0u, 0u};
#ifdef VR_CRAWL_PROF
        uint32_t dg[3] = {0, 0, 0};
        const long long c0 = clock64(), t0 = wall_clock64();
        v.out[(size_t)l * v.LW + x] = amb ? shade<STORE, ALGO, COUNT, true>(s, v, x, l, b, nullptr, &f, dg, &cl)
                                         : shade_resume<STORE, ALGO, COUNT>(s, v, r, b, f, dg, &cl);
        const long long c1 = clock64(), t1 = wall_clock64();
        if (i < 16384u) {
            g_vr_crawl_prof[8 * i + 0] = (uint32_t)min(c1 - c0, 0xFFFFFFFFll);
            g_vr_crawl_prof[8 * i + 1] = dg[0] | (amb ? 0x80000000u : 0u);
            g_vr_crawl_prof[8 * i + 2] = dg[1];
            g_vr_crawl_prof[8 * i + 3] = dg[2];
            g_vr_crawl_prof[8 * i + 4] = (uint32_t)t0;
            g_vr_crawl_prof[8 * i + 5] = (uint32_t)t1;
        }
#else
        v.out[(size_t)l * v.LW + x] = amb ? shade<STORE, ALGO, COUNT, true>(s, v, x, l, b, nullptr, &f, nullptr, &cl)
                                         : shade_resume<STORE, ALGO, COUNT>(s, v, r, b, f, nullptr, &cl);
#endif
        bytes += b;
        ffs += f.x;
        nls += f.y;
    }
    if (overflow != 0u) {
        // the list overflowed: the pixels the tile pass could not defer carry the marker
        const size_t npx = (size_t)v.local_rows * v.LW;
        for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < npx; i += (size_t)gridDim.x * blockDim.x) {
            if (v.out[i] != kDeferMarker) continue;
            uint32_t b;
            uint2 f{0u, 0u};
            // (a per-record bit slot is not this lane's: none)
            const CrawlLds clo;
            v.out[i] = shade<STORE, ALGO, COUNT, true>(s, v, (uint32_t)(i % v.LW), (uint32_t)(i / v.LW), b, nullptr, &f,
                                                       nullptr, &clo);
            bytes += b;
            ffs += f.x;
            nls += f.y;
        }
    }
    if (COUNT) {
        add_bytes(v, threadIdx.x & 63u, bytes);
        add_ff(v, threadIdx.x & 63u, ffs, nls);
    }
    // Every workgroup has read the count (above) before it adds to `done`; the
    // last one clears the slot for its next launch (ordered by the kernel boundary).
    __syncthreads();
    if (threadIdx.x == 0 && atomicAdd(&v.defer[1], 1u) == gridDim.x - 1u) {
        v.defer[0] = 0;
        v.defer[1] = 0;
        v.defer[2] = 0;
    }
}

// KScene::vcs_cbits: thread (r, w) ORs the existence of cluster slots 32w..32w+31 of
// region r (a present cluster's record has an index in every word, vr_internal.h)
__global__ void cluster_bits_kernel(const uint2* __restrict__ mask, uint32_t n_regions, uint32_t* __restrict__ cbits) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_regions * 16u) return;
    const uint2* m = mask + (size_t)(t >> 4) * 8192u + (size_t)(t & 15u) * 32u * 16u;
    uint32_t b = 0;
    for (uint32_t k = 0; k < 32u; ++k) b |= (m[k * 16u].y != kNone ? 1u : 0u) << k;
    cbits[t] = b;
}

// KScene::ht_filter: workgroup r sets the presence bit of every key in region r's two tables
// (keys are local generate3DPoint keys: x, y, z < 64)
__global__ void hash_filter_kernel(const uint4* __restrict__ meta, const uint2* __restrict__ slots,
                                   uint32_t* __restrict__ filter) {
    using F = Ctx<STORE_VCS, false, kTileBudget>;
    const uint4 m = meta[blockIdx.x];
    uint32_t* f = filter + (size_t)blockIdx.x * kHashFilterWords;
    for (uint32_t i = threadIdx.x; i < 2u * m.y; i += blockDim.x) {
        const uint32_t k = slots[m.x + i].x;
        if (k == kEmpty) continue;
        const uint32_t x = (k >> 20) & 63u, y = (k >> 10) & 63u, z = k & 63u;
        atomicOr(&f[F::word_index(x, y, z)], 1u << (F::word_bit5(y, z) & 31u));
    }
}

__global__ void pack_rgb8_kernel(const uint32_t* __restrict__ w, uint8_t* __restrict__ rgb, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t c = w[i];
    rgb[3 * i + 0] = (uint8_t)(c >> 16);
    rgb[3 * i + 1] = (uint8_t)((c >> 8) & 0xFFu);
    rgb[3 * i + 2] = (uint8_t)(c & 0xFFu);
}

// Rank 0's reassembly of the 2-D tile deal (vr_internal.h TileLayout): one thread per frame
// pixel reads its owner's local pixel -- the inverse of pixel_ray's column map -- and copies
// E bytes.  (The gathered buffers are read once and the frame written once: HBM-bound.)
template <int E>
__global__ void assemble_tiles_kernel(const uint8_t* __restrict__ parts, uint8_t* __restrict__ frame, TileLayout t) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)t.W * t.H) return;
    const uint32_t y = (uint32_t)(i / t.W), x = (uint32_t)(i - (uint64_t)y * t.W);
    const uint32_t b = y / t.band_rows, j = x / t.tile_cols, in_blk = x - j * t.tile_cols;
    const uint32_t rank = (j + t.stride * (b % t.R)) % t.R;
    const uint64_t lx = (uint64_t)(j / t.R) * t.tile_cols + in_blk;
    const uint64_t src = (uint64_t)rank * t.rank_words + (uint64_t)y * t.LW + lx;
#pragma unroll
    for (int k = 0; k < E; ++k) frame[i * E + k] = parts[src * E + k];
}

}  // namespace

// The tile pass, then the crawl pass (a small grid that exits at once when nothing
// was deferred), both on `stream`.  (The crawl pass on a high-priority side stream,
// fenced by events, measured slower on every config: C2 0.1148 -> 0.1224 ms per frame
// with two in flight, 0.154 -> 0.184 alone; profiles/r03/ab_crawl_stream.txt.)
// The crawl pass's grid: kCrawlRpw records per wave, all of them at once (each record is
// a latency-bound chain: C5 rpw 64 / 16 / 8 / 4 -> 0.93 / 0.82 / 0.80 / 0.76 ms per frame in
// flight, profiles/r03/ab_crawl_rpw.txt), at least 64 workgroups.  The host sizes it from
// the count an earlier launch of the device wrote to defer_stat: a launch that defers
// nothing (C2-C4) keeps the small grid (1024 empty workgroups cost C2 0.6 %).
uint32_t crawl_grid(uint32_t records, uint32_t rpw) {
    const uint32_t waves_per_wg = kCrawlWaves;
    rpw = rpw ? rpw : kCrawlRpw;
    const uint64_t waves = ((uint64_t)records * 5u / 4u + rpw - 1u) / rpw;
    const uint64_t wgs = (waves + waves_per_wg - 1u) / waves_per_wg;
    return (uint32_t)std::min<uint64_t>(std::max<uint64_t>(wgs, 64u), 4096u);
}

// VR_NO_CRAWL_PASS: a measurement-only build without the crawl pass (its cost on a
// frame that defers nothing, C2: profiles/r03/ab_no_crawl_pass_C2.txt); wrong for any
// frame that defers a pixel.
#ifdef VR_NO_CRAWL_PASS
constexpr bool kNoCrawlPass = true;
#else
constexpr bool kNoCrawlPass = false;
#endif

void march_grid(const KView& v, uint32_t& columns, uint32_t& rows) {
    columns = (v.LW + 8u * kTilesX - 1u) / (8u * kTilesX);
    rows = (v.local_rows + 8u * kTilesY - 1u) / (8u * kTilesY);
}

size_t perm_bytes(uint32_t gx, uint32_t gy) {
    return (size_t)((gx + kLbX - 1u) / kLbX) * ((gy + kLbY - 1u) / kLbY) * kLanePixels * sizeof(PermT);
}

hipError_t launch_perm(const uint32_t* pcost, uint32_t LW, uint32_t rows, uint32_t gx, uint32_t gy, uint8_t* perm,
                       uint32_t* cost, hipStream_t stream) {
    const uint32_t nb = ((gx + kLbX - 1u) / kLbX) * ((gy + kLbY - 1u) / kLbY);
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(perm_kernel, dim3(nb), dim3(kLanePixels), 0, stream, pcost, LW, rows, gx, gy, perm, cost);
    return hipGetLastError();
}

hipError_t launch_order(const uint32_t* cost, uint32_t n, uint32_t columns, uint32_t* order, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(order_kernel, dim3(1), dim3(1024), 0, stream, cost, n, columns, order);
    return hipGetLastError();
}

hipError_t launch_march(int store, int algo, bool count, const KScene& s, const KView& v, hipStream_t stream,
                        uint32_t crawl_wgs, bool in_flight, bool crawl) {
    uint32_t gx, gy;
    march_grid(v, gx, gy);
    dim3 grid(gx, gy);
    dim3 block(64u * kTilesX * kTilesY);
    if (grid.x == 0 || grid.y == 0) return hipSuccess;
    const dim3 cgrid(crawl_wgs ? crawl_wgs : 64u);
    const dim3 cblock(64u * kCrawlWaves);
#define VR_LAUNCH(ST, AL, CT) VR_LAUNCH_HI(ST, AL, CT, false)
#define VR_LAUNCH_HI(ST, AL, CT, HI)                                                              \
    do {                                                                                           \
        hipLaunchKernelGGL((march_kernel<ST, AL, CT, HI>), grid, block, 0, stream, s, v);          \
        if (v.defer && crawl && !kNoCrawlPass)                                                     \
            hipLaunchKernelGGL((crawl_kernel<ST, AL, CT>), cgrid, cblock, 0, stream, s, v);        \
    } while (0)
#ifdef VR_ISA_ONLY
    // ISA-inspection builds (csrc/Makefile isa1, profiles/loop_isa.py): one kernel pair
    // only, e.g. -DVR_ISA_ONLY=ALGO_LONGEST for the VCS longest-axis tile pass; never a library
    // (-DVR_ISA_STORE=STORE_HASH for a cuckoo pair, with its in-flight variant)
#ifndef VR_ISA_STORE
#define VR_ISA_STORE STORE_VCS
#endif
    (void)algo; (void)count; (void)store;
    if (in_flight) VR_LAUNCH_HI(VR_ISA_STORE, VR_ISA_ONLY, false, true);
    else VR_LAUNCH(VR_ISA_STORE, VR_ISA_ONLY, false);
#else
    // (the in-flight occupancy variants exist for the uninstrumented cuckoo original and
    // VCS longest-axis walks; the VCS original walk is fastest at 7 waves either way)
    const bool hi = in_flight && !count;
    if (store == STORE_VCS) {
        if (algo == ALGO_ORIGINAL) { if (count) VR_LAUNCH(STORE_VCS, ALGO_ORIGINAL, true); else VR_LAUNCH(STORE_VCS, ALGO_ORIGINAL, false); }
        else if (hi && kLongHiVariant) VR_LAUNCH_HI(STORE_VCS, ALGO_LONGEST, false, true);
        else { if (count) VR_LAUNCH(STORE_VCS, ALGO_LONGEST, true); else VR_LAUNCH(STORE_VCS, ALGO_LONGEST, false); }
    } else {
        if (algo == ALGO_ORIGINAL) {
            if (hi && kOrigHiVariant) VR_LAUNCH_HI(STORE_HASH, ALGO_ORIGINAL, false, true);
            else if (count) VR_LAUNCH(STORE_HASH, ALGO_ORIGINAL, true);
            else VR_LAUNCH(STORE_HASH, ALGO_ORIGINAL, false);
        }
        else { if (count) VR_LAUNCH(STORE_HASH, ALGO_LONGEST, true); else VR_LAUNCH(STORE_HASH, ALGO_LONGEST, false); }
    }
#endif
#undef VR_LAUNCH
#undef VR_LAUNCH_HI
    return hipGetLastError();
}

hipError_t launch_cluster_bits(const uint2* vcs_mask, uint32_t n_regions, uint32_t* cbits, hipStream_t stream) {
    if (n_regions == 0) return hipSuccess;
    const uint32_t threads = n_regions * 16u;
    hipLaunchKernelGGL(cluster_bits_kernel, dim3((threads + 255u) / 256u), dim3(256), 0, stream, vcs_mask, n_regions,
                       cbits);
    return hipGetLastError();
}

hipError_t launch_assemble_tiles(const void* parts, void* frame, uint32_t elem_bytes, const TileLayout& t,
                                 hipStream_t stream) {
    const uint64_t n = (uint64_t)t.W * t.H;
    if (n == 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
    const uint8_t* p = static_cast<const uint8_t*>(parts);
    uint8_t* f = static_cast<uint8_t*>(frame);
    switch (elem_bytes) {
    case 1: hipLaunchKernelGGL(assemble_tiles_kernel<1>, grid, block, 0, stream, p, f, t); break;
    case 2: hipLaunchKernelGGL(assemble_tiles_kernel<2>, grid, block, 0, stream, p, f, t); break;
    case 3: hipLaunchKernelGGL(assemble_tiles_kernel<3>, grid, block, 0, stream, p, f, t); break;
    default: hipLaunchKernelGGL(assemble_tiles_kernel<4>, grid, block, 0, stream, p, f, t); break;
    }
    return hipGetLastError();
}

hipError_t launch_hash_filter(const uint4* ht_meta, const uint2* ht_slots, uint32_t n_regions, uint32_t* filter,
                              hipStream_t stream) {
    if (n_regions == 0) return hipSuccess;
    hipLaunchKernelGGL(hash_filter_kernel, dim3(n_regions), dim3(256), 0, stream, ht_meta, ht_slots, filter);
    return hipGetLastError();
}

hipError_t launch_pack_rgb8(const uint32_t* words, uint8_t* rgb, uint64_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(pack_rgb8_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, words, rgb, n);
    return hipGetLastError();
}

}  // namespace vr

#ifdef VR_CRAWL_PROF
extern "C" int vr_crawl_prof_fetch(unsigned int* out, unsigned int n) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vr_crawl_prof), sizeof(unsigned int) * 8 * (n < 16384u ? n : 16384u)) !=
        hipSuccess)
        return -1;
    return 0;
}
#endif
#ifdef VR_DIAG
extern "C" int vr_diag_fetch(unsigned long long* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vr_diag), sizeof(unsigned long long) * 32) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[32] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_vr_diag), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif
