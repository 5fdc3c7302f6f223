/*
 * vr_oracle.c -- CPU restatement of the VoxelRaymarcher hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see vr_oracle.h).  PARITY UNPINNED by the
 * reference: it ships no golden vectors and may not be run here.
 *
 * Every function below restates one reference function; the citation is
 * the reference file:line it follows (paths relative to
 * /root/reference/VoxelRaymarcher/src).  The order of floating-point
 * operations is kept exactly as written in the reference, built with
 * -ffp-contract=off -fno-fast-math -fwrapv (wrapping int arithmetic =
 * what the CUDA device code does), and float->int conversions use the CUDA
 * device semantics (truncate, saturate, NaN -> 0).
 *
 * No iteration budget: every walk runs to the end the reference reaches,
 * however many iterations that takes (C5's cluster-skip crawls run up to
 * ~1.4 million).  The one deliberate, documented deviation is
 * for walks the reference never finishes: a loop iteration that leaves the
 * loop's whole state bit-for-bit unchanged repeats forever (every loop below
 * is a deterministic function of that state), so the pixel is declared
 * non-terminating there -- colour 0 and only the pixel write counted (4 B).
 * Those are the `stationary` checks below; they are exact (a state that does
 * not change cannot reach an exit), they never fire on a walk that ends.
 */
#include "vr_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define EPS 0.0001f                    /* VoxelFunctions.cuh:19 */
#define EMPTY_VAL (1u << 30)           /* VoxelFunctions.cuh:20-21 (EMPTY_KEY == EMPTY_VAL) */
#define CONTINUE_VAL (EMPTY_VAL + 2u)  /* VoxelFunctions.cuh:23 */
#define BLOCK 64                       /* VoxelFunctions.cuh:24 */
#define CLUSTER 8                      /* VoxelFunctions.cuh:25 */

/* Iteration budget per pixel (or_set_iter_budget; UINT64_MAX = none, the
 * default): a diagnostic only -- the restatement runs without one. */
static uint64_t g_budget = UINT64_MAX;

/* ------------------------------------------------------------------ math */

typedef struct { float v[3]; } v3f;
typedef struct { int32_t v[3]; } v3i;
typedef struct { v3f o, d; } ray3;

static inline v3f V3(float a, float b, float c) { v3f r = {{a, b, c}}; return r; }
/* Vector3.cuh:106-109 */
static inline v3f vadd(v3f a, v3f b) { return V3(a.v[0] + b.v[0], a.v[1] + b.v[1], a.v[2] + b.v[2]); }
/* Vector3.cuh:112-115 */
static inline v3f vsub(v3f a, v3f b) { return V3(a.v[0] - b.v[0], a.v[1] - b.v[1], a.v[2] - b.v[2]); }
/* Vector3.cuh:118-121 */
static inline v3f vmul(v3f a, v3f b) { return V3(a.v[0] * b.v[0], a.v[1] * b.v[1], a.v[2] * b.v[2]); }
/* Vector3.cuh:130-133 and 142-145: both orders compute t * v[i] */
static inline v3f vscale(float t, v3f a) { return V3(t * a.v[0], t * a.v[1], t * a.v[2]); }
/* Vector3.cuh:136-139 */
static inline v3f vdivs(v3f a, float t) { return V3(a.v[0] / t, a.v[1] / t, a.v[2] / t); }
/* Vector3.cuh:79 */
static inline float vlength(v3f a) { return sqrtf(a.v[0] * a.v[0] + a.v[1] * a.v[1] + a.v[2] * a.v[2]); }
/* Vector3.cuh:162-165 */
static inline v3f vunit(v3f a) { return vdivs(a, vlength(a)); }
/* Vector3.cuh:148-151 */
static inline float vdot(v3f a, v3f b) { return a.v[0] * b.v[0] + a.v[1] * b.v[1] + a.v[2] * b.v[2]; }
/* Vector3.cuh:154-159 */
static inline v3f vcross(v3f a, v3f b) {
    return V3((a.v[1] * b.v[2] - a.v[2] * b.v[1]),
              (-(a.v[0] * b.v[2] - a.v[2] * b.v[0])),
              (a.v[0] * b.v[1] - a.v[1] * b.v[0]));
}

/* static_cast<int32_t>(float) in CUDA device code: cvt.rzi.s32.f32 --
 * truncate toward zero, saturate, NaN -> 0. */
static inline int32_t f2i(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return INT32_MAX;
    if (f <= -2147483648.0f) return INT32_MIN;
    return (int32_t)f;
}
/* static_cast<uint32_t>(float): cvt.rzi.u32.f32 (saturating, NaN -> 0). */
static inline uint32_t f2u(float f) {
    if (f != f || f <= 0.0f) return 0u;
    if (f >= 4294967296.0f) return UINT32_MAX;
    return (uint32_t)f;
}

void or_set_iter_budget(uint64_t budget) { g_budget = budget; }

/* ------------------------------------------------------------ the scene */

static const uint32_t PRIME_TABLE[14] = {  /* CuckooHashTable.cuh:8-12 */
    668265261u, 12289u, 24593u, 49157u, 98317u, 196613u, 393241u, 786433u,
    1572869u, 3145739u, 6291469u, 12582917u, 25165843u, 50331653u};

typedef struct {
    uint32_t M, offset, prime;
    uint32_t *k1, *v1, *k2, *v2;
} or_cuckoo;

struct or_scene {
    int store;
    uint32_t D;
    int32_t min_coord;
    int32_t* region_slot;   /* D^3, region index or -1 (null StorageStructure*) */
    uint32_t n_regions;
    int64_t* vcs_dir;       /* n_regions*512 offsets into vcs_pool, -1 = no cluster */
    uint32_t* vcs_pool;     /* blocks [n, k0, v0, k1, v1, ...] (VoxelClusterStore.cuh:61-76) */
    or_cuckoo* ht;          /* n_regions tables */
};

/* VoxelFunctions.cuh:41-46 (assert compiled out in release) */
uint32_t or_generate_3d_point(uint32_t x, uint32_t y, uint32_t z) {
    return (x << 20) | (y << 10) | z;
}

/* VoxelClusterStore.cuh:21-24: computed in uint32, returned as `short`. */
uint32_t or_cluster_id(uint32_t x, uint32_t y, uint32_t z) {
    return ((x / 8u) << 6) | ((y / 8u) << 3) | (z / 8u);
}
static inline int32_t cluster_id_short(int32_t x, int32_t y, int32_t z) {
    return (int32_t)(int16_t)(uint16_t)or_cluster_id((uint32_t)x, (uint32_t)y, (uint32_t)z);
}

/* CuckooHashTable.cuh:181-190.  `int` arithmetic: left shifts and adds wrap,
 * right shifts of the int are arithmetic; mixing with the unsigned literals
 * only changes the type, not the bits. */
int32_t or_hash1(int32_t key, uint32_t offset) {
    uint32_t k = (uint32_t)key;
    k = (k + 0x7ed55d16u) + (k << 12);
    k = (k ^ 0xc761c23cu) ^ (uint32_t)((int32_t)k >> 19);
    k = (k + 0x165667b1u) + (k << 5);
    k = (k + 0xd3a2646cu) ^ (k << 9);
    k = (k + 0xfd7046c5u) + (k << 3);
    k = (k ^ 0xb55a4f09u) ^ (uint32_t)((int32_t)k >> 16);
    return (int32_t)(k + offset);
}
/* CuckooHashTable.cuh:193-202 */
int32_t or_hash2(int32_t key, uint32_t prime) {
    uint32_t k = (uint32_t)key;
    k = (k ^ 61u) ^ (uint32_t)((int32_t)k >> 16);
    k = k + (k << 3);
    k = k ^ (uint32_t)((int32_t)k >> 4);
    k = k * prime;
    k = k ^ (uint32_t)((int32_t)k >> 15);
    return (int32_t)k;
}

typedef struct { uint32_t key, val; } kv;

typedef struct { int64_t region; uint32_t key, val; size_t idx; } vrec;
static int vrec_cmp(const void* a, const void* b) {
    const vrec* x = (const vrec*)a; const vrec* y = (const vrec*)b;
    if (x->region != y->region) return x->region < y->region ? -1 : 1;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

/* Deterministic stand-in for Random::getRandomInt (Random.cuh:14-18); any
 * valid cuckoo placement yields identical lookup VALUES, but the
 * bytes a lookup reads depend on the table a key sits in (4 more for table 2),
 * so the stand-in is the product builder's (vr_host.cpp cuckoo_build): the same
 * LCG, seeded from the region's key count and first key. */
static uint32_t lcg_next(uint64_t* s) {
    *s = *s * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(*s >> 33);
}

/* CuckooHashTable.cuh:20-49 + createCuckooHashTable :97-178 */
static int cuckoo_build(or_cuckoo* t, const kv* e, uint32_t n) {
    t->M = (uint32_t)((double)n * 1.25);            /* :23 numElements * 1.25 */
    t->offset = 0; t->prime = PRIME_TABLE[0];
    t->k1 = (uint32_t*)malloc(sizeof(uint32_t) * t->M);
    t->v1 = (uint32_t*)calloc(t->M, sizeof(uint32_t));
    t->k2 = (uint32_t*)malloc(sizeof(uint32_t) * t->M);
    t->v2 = (uint32_t*)calloc(t->M, sizeof(uint32_t));
    if (!t->k1 || !t->v1 || !t->k2 || !t->v2) return -1;
    uint64_t rng = 0x9E3779B97F4A7C15ull ^ (uint64_t)n ^ ((uint64_t)e[0].key << 20);
    for (int attempt = 0; attempt < 4096; ++attempt) {
        for (uint32_t i = 0; i < t->M; ++i) { t->k1[i] = EMPTY_VAL; t->k2[i] = EMPTY_VAL; t->v1[i] = 0; t->v2[i] = 0; }
        int rehash = 0;
        for (uint32_t i = 0; i < n && !rehash; ++i) {
            uint32_t code = e[i].key, value = e[i].val, bucket = 0, it = 0;
            for (;;) {
                if (it >= 300000u) { rehash = 1; break; }  /* :112-123 */
                if (bucket == 0) {
                    uint32_t s = (uint32_t)or_hash1((int32_t)code, t->offset) % t->M;
                    if (t->k1[s] == EMPTY_VAL) { t->k1[s] = code; t->v1[s] = value; break; }
                    uint32_t tc = t->k1[s], tv = t->v1[s];
                    t->k1[s] = code; t->v1[s] = value; code = tc; value = tv; bucket = 1;
                } else {
                    uint32_t s = (uint32_t)or_hash2((int32_t)code, t->prime) % t->M;
                    if (t->k2[s] == EMPTY_VAL) { t->k2[s] = code; t->v2[s] = value; break; }
                    uint32_t tc = t->k2[s], tv = t->v2[s];
                    t->k2[s] = code; t->v2[s] = value; code = tc; value = tv; bucket = 0;
                }
                ++it;
            }
        }
        if (!rehash) return 0;
        t->prime = PRIME_TABLE[lcg_next(&rng) % 14u];
        t->offset = lcg_next(&rng) % 25u;
    }
    return -2;
}

/* VoxelSceneCPU::insertVoxel (VoxelSceneCPU.cuh:16-46) for every voxel,
 * then generateVoxelScene (:49-93) and the per-region storage builders. */
int or_scene_build(int store, const int32_t* xyz, const uint32_t* rgb, size_t n, or_scene** out) {
    *out = NULL;
    or_scene* s = (or_scene*)calloc(1, sizeof(or_scene));
    if (!s) return -1;
    s->store = store;
    vrec* recs = (vrec*)malloc(sizeof(vrec) * (n ? n : 1));
    int32_t minc = 0, maxc = 0;                       /* VoxelSceneCPU.cuh:129-130 */
    int32_t* rc = (int32_t*)malloc(sizeof(int32_t) * 3 * (n ? n : 1));
    for (size_t i = 0; i < n; ++i) {
        int32_t x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
        int32_t rx = f2i(floorf((float)x / 64.0f));   /* :19-21 std::floorf(x / (float)BLOCK_SIZE) */
        int32_t ry = f2i(floorf((float)y / 64.0f));
        int32_t rz = f2i(floorf((float)z / 64.0f));
        uint32_t lx = (uint32_t)(((x % BLOCK) + BLOCK) % BLOCK);   /* :24-26 */
        uint32_t ly = (uint32_t)(((y % BLOCK) + BLOCK) % BLOCK);
        uint32_t lz = (uint32_t)(((z % BLOCK) + BLOCK) % BLOCK);
        int32_t mn = rx < ry ? rx : ry; mn = mn < rz ? mn : rz;   /* :28-35 */
        int32_t mx = rx > ry ? rx : ry; mx = mx > rz ? mx : rz;
        if (mn < minc) minc = mn;
        if (mx > maxc) maxc = mx;
        rc[3 * i] = rx; rc[3 * i + 1] = ry; rc[3 * i + 2] = rz;
        recs[i].key = or_generate_3d_point(lx, ly, lz);
        recs[i].val = rgb[i];
        recs[i].idx = i;
    }
    s->D = (uint32_t)(maxc - minc + 1);
    s->min_coord = minc;
    uint64_t D = s->D;
    for (size_t i = 0; i < n; ++i) {
        uint64_t ax = (uint64_t)(int64_t)(rc[3 * i] - minc), ay = (uint64_t)(int64_t)(rc[3 * i + 1] - minc),
                 az = (uint64_t)(int64_t)(rc[3 * i + 2] - minc);
        recs[i].region = (int64_t)(ax + ay * D + az * D * D);   /* :62 */
    }
    free(rc);
    qsort(recs, n, sizeof(vrec), vrec_cmp);
    /* dedupe: the later insertion wins (map assignment, :46) */
    size_t m = 0;
    for (size_t i = 0; i < n; ++i) {
        if (m > 0 && recs[m - 1].region == recs[i].region && recs[m - 1].key == recs[i].key) recs[m - 1] = recs[i];
        else recs[m++] = recs[i];
    }
    s->region_slot = (int32_t*)malloc(sizeof(int32_t) * D * D * D);
    for (uint64_t i = 0; i < D * D * D; ++i) s->region_slot[i] = -1;
    uint32_t nr = 0;
    for (size_t i = 0; i < m; ++i)
        if (i == 0 || recs[i].region != recs[i - 1].region) s->region_slot[recs[i].region] = (int32_t)nr++;
    s->n_regions = nr;
    int rc_ok = 0;
    if (store == OR_STORE_VCS) {
        s->vcs_dir = (int64_t*)malloc(sizeof(int64_t) * 512 * (nr ? nr : 1));
        s->vcs_pool = (uint32_t*)malloc(sizeof(uint32_t) * (m * 2 + 512 * (size_t)nr + 1));
        size_t pool = 0, i = 0;
        uint32_t r = 0;
        while (i < m) {
            size_t j = i;
            while (j < m && recs[j].region == recs[i].region) ++j;
            /* VoxelClusterStore.cuh:37-85: bucket by cluster, keys ascending,
             * block = [n, (k,v) x n].  recs[i..j) is already sorted by key, so a
             * stable counting scatter by cluster id keeps each block sorted. */
            int64_t* dir = s->vcs_dir + (size_t)r * 512;
            uint32_t counts[512] = {0}, start[512];
            for (size_t k = i; k < j; ++k) {
                uint32_t key = recs[k].key;
                counts[or_cluster_id(key >> 20, (key >> 10) & 0x3FFu, key & 0x3FFu)]++;
            }
            size_t p = pool;
            for (int c = 0; c < 512; ++c) {
                if (!counts[c]) { dir[c] = -1; continue; }
                dir[c] = (int64_t)p;
                s->vcs_pool[p] = counts[c];
                start[c] = (uint32_t)(p + 1 - pool);
                p += 1 + 2 * (size_t)counts[c];
            }
            for (size_t k = i; k < j; ++k) {
                uint32_t key = recs[k].key;
                uint32_t c = or_cluster_id(key >> 20, (key >> 10) & 0x3FFu, key & 0x3FFu);
                s->vcs_pool[pool + start[c]] = key;
                s->vcs_pool[pool + start[c] + 1] = recs[k].val;
                start[c] += 2;
            }
            pool = p;
            ++r; i = j;
        }
    } else {
        s->ht = (or_cuckoo*)calloc(nr ? nr : 1, sizeof(or_cuckoo));
        size_t i = 0; uint32_t r = 0;
        kv* tmp = (kv*)malloc(sizeof(kv) * (m ? m : 1));
        while (i < m) {
            size_t j = i;
            while (j < m && recs[j].region == recs[i].region) ++j;
            for (size_t k = i; k < j; ++k) { tmp[k - i].key = recs[k].key; tmp[k - i].val = recs[k].val; }
            if (cuckoo_build(&s->ht[r], tmp, (uint32_t)(j - i)) != 0) rc_ok = -3;
            ++r; i = j;
        }
        free(tmp);
    }
    free(recs);
    if (rc_ok) { or_scene_free(s); return rc_ok; }
    *out = s;
    return 0;
}

void or_scene_free(or_scene* s) {
    if (!s) return;
    free(s->region_slot);
    free(s->vcs_dir);
    free(s->vcs_pool);
    if (s->ht) {
        for (uint32_t r = 0; r < s->n_regions; ++r) {
            free(s->ht[r].k1); free(s->ht[r].v1); free(s->ht[r].k2); free(s->ht[r].v2);
        }
        free(s->ht);
    }
    free(s);
}
/* Test helper: the table (1 or 2) a key of region index r sits in, 0 if absent, -1 if
 * r or the store is wrong; *rehashed = the region's table needed a rehash (prime or
 * offset differ from the first attempt's). */
int or_scene_cuckoo_table(const or_scene* s, uint32_t r, uint32_t key, int* rehashed) {
    if (s->store != OR_STORE_HASHTABLE || r >= s->n_regions) return -1;
    const or_cuckoo* t = &s->ht[r];
    if (rehashed) *rehashed = t->prime != PRIME_TABLE[0] || t->offset != 0;
    uint32_t M = t->M;
    if (M == 0) return 0;
    uint32_t k1 = ((uint32_t)or_hash1((int32_t)key, t->offset) % M + M) % M;
    if (t->k1[k1] == key) return 1;
    uint32_t k2 = ((uint32_t)or_hash2((int32_t)key, t->prime) % M + M) % M;
    if (t->k2[k2] == key) return 2;
    return 0;
}
uint32_t or_scene_diameter(const or_scene* s) { return s->D; }
int32_t or_scene_min_coord(const or_scene* s) { return s->min_coord; }
uint32_t or_scene_region_count(const or_scene* s) { return s->n_regions; }

/* ---------------------------------------------------- per-ray context */

typedef struct {
    const or_scene* s;
    const or_lighting* lit;
    v3f translation;
    uint64_t bytes;
    uint64_t iters;
    int aborted;
    int in_shadow;          /* statistics only: counting into st[1] while walking a shadow ray */
    uint64_t* st;           /* optional work statistics, OR_STAT_* x 2 (primary, shadow) */
} ctx;

/* work statistics (or_render_stats) */
enum { OR_STAT_REGION = 0, OR_STAT_EXISTS, OR_STAT_SKIP, OR_STAT_LOOKUP, OR_STAT_PROBE, OR_STAT_HIT,
       OR_STAT_ITERS, OR_STAT_OUTSIDE, OR_STAT_ALIAS, OR_STAT_N };
#define STAT(c, k) do { if ((c)->st) (c)->st[(c)->in_shadow * OR_STAT_N + (k)]++; } while (0)

static inline int tick(ctx* c) {
    if (c->aborted) return 0;
    STAT(c, OR_STAT_ITERS);
    if (++c->iters > g_budget) { c->aborted = 1; return 0; }
    return 1;
}

/* Loop state comparison for the non-termination checks: the same bits, or both
 * NaN (NaN payloads may change once; every later use treats them alike). */
static inline int same_f(float a, float b) {
    uint32_t x, y;
    memcpy(&x, &a, 4); memcpy(&y, &b, 4);
    return x == y || (a != a && b != b);
}
static inline int same_v(v3f a, v3f b) { return same_f(a.v[0], b.v[0]) && same_f(a.v[1], b.v[1]) && same_f(a.v[2], b.v[2]); }
static inline int same_i(v3i a, v3i b) { return a.v[0] == b.v[0] && a.v[1] == b.v[1] && a.v[2] == b.v[2]; }
/* The loop would repeat this iteration forever: give up on the pixel. */
static inline int stationary(ctx* c) { c->aborted = 1; return 0; }
/* Brent's cycle detection for the region-level loops (entry clip, region rounds,
 * null-region skips), whose rounds are functions of (region, position) alone: a snapshot
 * at rounds 1, 2, 4, ...; a later state equal to it repeats forever.  Finds a repeat of
 * any period (a fixed point at the first repeat).  The kernels use the same test
 * (vr_device.h Ctx::cycle_step); the pixel's result does not depend on when a repeat is
 * found (colour 0, only the pixel write counted). */
typedef struct { v3i c; v3f o; uint32_t lam, pow; } cycle;
static inline cycle cycle_start(v3i c, v3f o) { cycle y = {c, o, 0u, 1u}; return y; }
static inline int cycle_step(cycle* y, v3i c, v3f o) {
    if (same_i(c, y->c) && same_v(o, y->o)) return 1;
    if (++y->lam == y->pow) { y->c = c; y->o = o; y->pow <<= 1; y->lam = 0u; }
    return 0;
}

/* Test hook for the cycle test alone: a loop whose state sequence is `prefix` distinct
 * states, then `period` distinct states repeating (period 0: never repeats).  Returns the
 * round at which cycle_step reports the repeat, or -1 if none within max_rounds. */
int64_t or_cycle_selftest(uint32_t prefix, uint32_t period, uint32_t max_rounds) {
    #define OR_STATE(k) ((v3i){{(int32_t)(k), -(int32_t)(k), 7}}), V3((float)(k) * 0.5f, 1.0f, (float)(k))
    cycle y = cycle_start(OR_STATE(0u));
    for (uint32_t r = 1; r <= max_rounds; ++r) {
        const uint32_t k = (period == 0u || r < prefix) ? r : prefix + (r - prefix) % period;
        if (cycle_step(&y, OR_STATE(k))) return (int64_t)r;
    }
    #undef OR_STATE
    return -1;
}

/* VoxelScene::isRayInScene (Renderer.cuh:38-44) */
static inline int in_scene(const ctx* c, v3i r) {
    uint32_t D = c->s->D, mc = (uint32_t)c->s->min_coord;
    return ((uint32_t)r.v[0] - mc) < D && ((uint32_t)r.v[1] - mc) < D && ((uint32_t)r.v[2] - mc) < D;
}
/* VoxelScene::getRegionStorageStructure (Renderer.cuh:29-36); +4 B per read */
static inline int32_t region_at(ctx* c, v3i r) {
    uint32_t D = c->s->D, mc = (uint32_t)c->s->min_coord;
    uint32_t ux = (uint32_t)r.v[0] - mc, uy = (uint32_t)r.v[1] - mc, uz = (uint32_t)r.v[2] - mc;
    c->bytes += 4;
    STAT(c, OR_STAT_REGION);
    return c->s->region_slot[ux + uy * D + uz * D * D];
}

/* StorageStructure::doesVoxelSpaceExist (StorageStructure.cuh:29-32,49-52)
 * -> VoxelClusterStore::doesClusterExist (VoxelClusterStore.cuh:93-99).
 * A cluster id outside [0,512) (coords outside the region) would read past
 * the reference's directory; it is defined here as "no cluster". */
static inline int space_exists(ctx* c, int32_t reg, int32_t x, int32_t y, int32_t z) {
    if (c->s->store != OR_STORE_VCS) return 1;
    c->bytes += 4;
    STAT(c, OR_STAT_EXISTS);
    int32_t cid = cluster_id_short(x, y, z);
    if (((uint32_t)x | (uint32_t)y | (uint32_t)z) >= (uint32_t)BLOCK) {
        STAT(c, OR_STAT_OUTSIDE);                         /* a probe outside the region */
        if (cid >= 0 && cid < 512) STAT(c, OR_STAT_ALIAS); /* ... whose short id aliases a cluster */
    }
    if (cid < 0 || cid >= 512) { STAT(c, OR_STAT_SKIP); return 0; }
    if (c->s->vcs_dir[(size_t)reg * 512 + (size_t)cid] >= 0) return 1;
    STAT(c, OR_STAT_SKIP);
    return 0;
}

/* VoxelClusterStore::lookupVoxel + performBinarySearch (VoxelClusterStore.cuh:101-135)
 * CuckooHashTable::lookupVoxel (CuckooHashTable.cuh:59-76) */
static uint32_t lookup_voxel(ctx* c, int32_t reg, int32_t x, int32_t y, int32_t z) {
    const or_scene* s = c->s;
    uint32_t key = or_generate_3d_point((uint32_t)x, (uint32_t)y, (uint32_t)z);
    STAT(c, OR_STAT_LOOKUP);
    if (s->store == OR_STORE_VCS) {
        int32_t cid = cluster_id_short(x, y, z);
        if (cid < 0 || cid >= 512) return EMPTY_VAL;
        int64_t off = s->vcs_dir[(size_t)reg * 512 + (size_t)cid];
        if (off < 0) return EMPTY_VAL;
        const uint32_t* blk = s->vcs_pool + off;
        uint32_t bs = blk[0];
        c->bytes += 4;
        int32_t low = 0, high = (int32_t)bs - 1;
        while (low <= high) {
            int32_t mid = low + (high - low) / 2;
            uint32_t k = blk[mid * 2 + 1];
            c->bytes += 4;
            STAT(c, OR_STAT_PROBE);
            if (k == key) { c->bytes += 4; STAT(c, OR_STAT_HIT); return blk[mid * 2 + 2]; }
            if (k < key) low = mid + 1; else high = mid - 1;
        }
        return EMPTY_VAL;
    } else {
        const or_cuckoo* t = &s->ht[reg];
        uint32_t M = t->M;
        uint32_t k1 = ((uint32_t)or_hash1((int32_t)key, t->offset) % M + M) % M;
        c->bytes += 4;
        STAT(c, OR_STAT_PROBE);
        if (t->k1[k1] == key) { c->bytes += 4; STAT(c, OR_STAT_HIT); return t->v1[k1]; }
        uint32_t k2 = ((uint32_t)or_hash2((int32_t)key, t->prime) % M + M) % M;
        c->bytes += 4;
        STAT(c, OR_STAT_PROBE);
        if (t->k2[k2] == key) { c->bytes += 4; STAT(c, OR_STAT_HIT); return t->v2[k2]; }
        return EMPTY_VAL;
    }
}

uint32_t or_scene_lookup(const or_scene* s, int32_t rx, int32_t ry, int32_t rz, int32_t x, int32_t y, int32_t z) {
    ctx c; memset(&c, 0, sizeof c); c.s = s;
    v3i r = {{rx, ry, rz}};
    if (!in_scene(&c, r)) return EMPTY_VAL;
    int32_t reg = region_at(&c, r);
    if (reg < 0) return EMPTY_VAL;
    if (!space_exists(&c, reg, x, y, z)) return EMPTY_VAL;
    return lookup_voxel(&c, reg, x, y, z);
}

/* --------------------------------------------------------- lighting */

/* voxelfunc::convertRGBIntegerColorToVector (VoxelFunctions.cuh:69-75) */
static inline v3f rgb_to_vec(uint32_t c) {
    return V3((float)(c >> 16) / 255.0f, (float)((c >> 8) & 0xFFu) / 255.0f, (float)(c & 0xFFu) / 255.0f);
}
/* voxelfunc::convertRGBVectorToInteger (VoxelFunctions.cuh:77-83) */
static inline uint32_t vec_to_rgb(v3f v) {
    uint32_t r = f2u(v.v[0] * 255.0f), g = f2u(v.v[1] * 255.0f), b = f2u(v.v[2] * 255.0f);
    return (r << 16) | (g << 8) | b;
}
/* applyDirectionalLightingToColor (Renderer.cuh:57-66) */
static uint32_t light_directional(const ctx* c, uint32_t color, v3f n) {
    v3f L = V3(c->lit->light_dir[0], c->lit->light_dir[1], c->lit->light_dir[2]);
    v3f LC = V3(c->lit->light_color[0], c->lit->light_color[1], c->lit->light_color[2]);
    float diff = fmaxf(vdot(n, L), 0.0f);
    v3f diffuse = vscale(diff, LC);
    v3f col = rgb_to_vec(color);
    return vec_to_rgb(vmul(col, diffuse));
}
/* applyPointLightingToColor (Renderer.cuh:68-86) */
static uint32_t light_point(const ctx* c, uint32_t color, v3f pos, v3f n) {
    v3f LP = V3(c->lit->light_pos[0], c->lit->light_pos[1], c->lit->light_pos[2]);
    v3f LC = V3(c->lit->light_color[0], c->lit->light_color[1], c->lit->light_color[2]);
    v3f p2l = vsub(LP, pos);
    float dist = vlength(p2l);
    v3f ldir = vunit(p2l);
    float att = 1.0f / (1.0f + 0.045f * dist + 0.0075f * (dist * dist));
    float diff = fmaxf(vdot(n, ldir), 0.0f);
    v3f diffuse = vscale(diff, LC);
    v3f col = rgb_to_vec(color);
    return vec_to_rgb(vmul(vscale(att, diffuse), col));
}
/* applyLighting (Renderer.cuh:249-258); getHitLocation (:88-91) */
static uint32_t apply_lighting(const ctx* c, uint32_t color, v3f n, v3f region_world, v3f ray_origin) {
    if (c->lit->use_point_light) return light_point(c, color, vadd(region_world, ray_origin), n);
    return light_directional(c, color, n);
}
/* getNormalFromTValues (Renderer.cuh:237-247) */
static inline v3f normal_from_t(float tX, float tY, float tZ, float tMin, v3f d) {
    if (tX == tMin) return V3(copysignf(1.0f, -d.v[0]), 0.0f, 0.0f);
    if (tY == tMin) return V3(0.0f, copysignf(1.0f, -d.v[1]), 0.0f);
    return V3(0.0f, 0.0f, copysignf(1.0f, -d.v[2]));
}

/* ------------------------------------------------------- traversal */

/* applyCeilAndPosEpsilon1 / applyFloorAndNegEpsilon1 (Renderer.cuh:47-55) */
static inline float next_plane(int positive, float x) { return positive ? ceilf(x) + EPS : floorf(x) - EPS; }

/* isRayInRegion (Renderer.cuh:93-98) */
static inline int in_region(v3f o) {
    return o.v[0] >= 0.0f && o.v[0] < (float)BLOCK && o.v[1] >= 0.0f && o.v[1] < (float)BLOCK &&
           o.v[2] >= 0.0f && o.v[2] < (float)BLOCK;
}
/* areGridValuesInRegion (Renderer.cuh:436-439) */
static inline int grid_in_region(int32_t a, int32_t b, int32_t d) {
    return (uint32_t)a < (uint32_t)BLOCK && (uint32_t)b < (uint32_t)BLOCK && (uint32_t)d < (uint32_t)BLOCK;
}

/* Region advance shared by every region loop (e.g. Renderer.cuh:421-429):
 * diff = floorf(o/64), region += diff, origin -= diff*64 (scale 1). */
static inline void advance_region(v3i* cr, ray3* lr) {
    int32_t dx = f2i(floorf(lr->o.v[0] / (float)BLOCK));
    int32_t dy = f2i(floorf(lr->o.v[1] / (float)BLOCK));
    int32_t dz = f2i(floorf(lr->o.v[2] / (float)BLOCK));
    cr->v[0] += dx; cr->v[1] += dy; cr->v[2] += dz;
    v3f t = V3((float)(dx * BLOCK), (float)(dy * BLOCK), (float)(dz * BLOCK));
    lr->o = vscale(1.0f, vsub(lr->o, t));   /* Ray::convertRayToLocalSpace (Ray.cuh:14-17), scale 1 */
}

/* Null-region skip loop body (Renderer.cuh:386-406; guarded form :187-207).
 * Returns 0 when the ray leaves the scene. */
static inline int skip_null_region(ctx* c, v3i* cr, ray3* lr, int guarded, int32_t* reg) {
    v3f o = lr->o, d = lr->d;
    float nx = d.v[0] > 0.0f ? (float)BLOCK + EPS : 0.0f - EPS;
    float ny = d.v[1] > 0.0f ? (float)BLOCK + EPS : 0.0f - EPS;
    float nz = d.v[2] > 0.0f ? (float)BLOCK + EPS : 0.0f - EPS;
    float tX, tY, tZ;
    if (guarded) {
        tX = d.v[0] != 0.0f ? (nx - o.v[0]) / d.v[0] : INFINITY;
        tY = d.v[1] != 0.0f ? (ny - o.v[1]) / d.v[1] : INFINITY;
        tZ = d.v[2] != 0.0f ? (nz - o.v[2]) / d.v[2] : INFINITY;
    } else {
        tX = (nx - o.v[0]) / d.v[0];
        tY = (ny - o.v[1]) / d.v[1];
        tZ = (nz - o.v[2]) / d.v[2];
    }
    float tMin = fminf(tX, fminf(tY, tZ));
    lr->o = vadd(o, vscale(tMin, d));       /* no EPSILON here (:396) */
    advance_region(cr, lr);
    if (!in_scene(c, *cr)) return 0;
    *reg = region_at(c, *cr);
    return 1;
}

/* shadowRayMarchVoxelGrid (Renderer.cuh:100-172) */
static uint32_t shadow_grid_original(ctx* c, ray3* ray, int32_t reg) {
    v3f d = ray->d;
    int px = d.v[0] > 0.0f, py = d.v[1] > 0.0f, pz = d.v[2] > 0.0f;
    v3f o = ray->o;
    float nX = next_plane(px, o.v[0]), nY = next_plane(py, o.v[1]), nZ = next_plane(pz, o.v[2]);
    float tX = d.v[0] != 0.0f ? (nX - o.v[0]) / d.v[0] : INFINITY;
    float tY = d.v[1] != 0.0f ? (nY - o.v[1]) / d.v[1] : INFINITY;
    float tZ = d.v[2] != 0.0f ? (nZ - o.v[2]) / d.v[2] : INFINITY;
    float tMin = fminf(tX, fminf(tY, tZ));
    ray->o = vadd(o, vscale(tMin + EPS, d));
    while (in_region(ray->o)) {
        if (!tick(c)) return EMPTY_VAL;
        o = ray->o;
        int32_t vx = f2i(o.v[0]), vy = f2i(o.v[1]), vz = f2i(o.v[2]);
        if (!space_exists(c, reg, vx, vy, vz)) {
            int32_t cx = px ? ((vx / CLUSTER) + 1) * CLUSTER : (vx / CLUSTER) * CLUSTER;
            int32_t cy = py ? ((vy / CLUSTER) + 1) * CLUSTER : (vy / CLUSTER) * CLUSTER;
            int32_t cz = pz ? ((vz / CLUSTER) + 1) * CLUSTER : (vz / CLUSTER) * CLUSTER;
            float sX = d.v[0] != 0.0f ? ((float)cx - o.v[0]) / d.v[0] : INFINITY;
            float sY = d.v[1] != 0.0f ? ((float)cy - o.v[1]) / d.v[1] : INFINITY;
            float sZ = d.v[2] != 0.0f ? ((float)cz - o.v[2]) / d.v[2] : INFINITY;
            float sMin = fminf(sX, fminf(sY, sZ));
            ray->o = vadd(o, vscale(sMin + EPS, d));
            if (same_v(ray->o, o)) return stationary(c), EMPTY_VAL;
            continue;
        }
        uint32_t col = lookup_voxel(c, reg, vx, vy, vz);
        if (col != EMPTY_VAL) return col;
        nX = next_plane(px, o.v[0]); nY = next_plane(py, o.v[1]); nZ = next_plane(pz, o.v[2]);
        tX = d.v[0] != 0.0f ? (nX - o.v[0]) / d.v[0] : INFINITY;
        tY = d.v[1] != 0.0f ? (nY - o.v[1]) / d.v[1] : INFINITY;
        tZ = d.v[2] != 0.0f ? (nZ - o.v[2]) / d.v[2] : INFINITY;
        tMin = fminf(tX, fminf(tY, tZ));
        ray->o = vadd(o, vscale(tMin + EPS, d));
        if (same_v(ray->o, o)) return stationary(c), EMPTY_VAL;
    }
    return EMPTY_VAL;
}

/* isInShadowOriginalRayMarch (Renderer.cuh:174-235) */
static int shadow_scene_original(ctx* c, ray3 lr, v3i cr) {
    if (!c->lit->use_shadows) return 0;
    c->in_shadow = 1;
    cycle cyc = cycle_start(cr, lr.o);
    while (in_scene(c, cr)) {
        if (!tick(c)) return 0;
        int32_t reg = region_at(c, cr);
        cycle cyc1 = cycle_start(cr, lr.o);
        while (reg < 0) {
            if (!tick(c)) return 0;
            if (!skip_null_region(c, &cr, &lr, 1, &reg)) return 0;
            if (cycle_step(&cyc1, cr, lr.o)) return stationary(c);
        }
        uint32_t col = shadow_grid_original(c, &lr, reg);
        if (c->aborted) return 0;
        if (col != EMPTY_VAL) return 1;
        advance_region(&cr, &lr);
        if (cycle_step(&cyc, cr, lr.o)) return stationary(c);
    }
    return 0;
}

/* rayMarchVoxelGrid (Renderer.cuh:260-336) */
static uint32_t grid_original(ctx* c, ray3* ray, v3f rwp, int32_t reg, v3i cr) {
    v3f d = ray->d;
    int px = d.v[0] > 0.0f, py = d.v[1] > 0.0f, pz = d.v[2] > 0.0f;
    v3f o = ray->o;
    float nX = next_plane(px, o.v[0]), nY = next_plane(py, o.v[1]), nZ = next_plane(pz, o.v[2]);
    float tX = (nX - o.v[0]) / d.v[0];
    float tY = (nY - o.v[1]) / d.v[1];
    float tZ = (nZ - o.v[2]) / d.v[2];
    float tMin = fminf(tX, fminf(tY, tZ));
    ray->o = vadd(o, vscale(tMin + EPS, d));
    while (in_region(ray->o)) {
        if (!tick(c)) return EMPTY_VAL;
        o = ray->o;
        int32_t vx = f2i(o.v[0]), vy = f2i(o.v[1]), vz = f2i(o.v[2]);
        if (!space_exists(c, reg, vx, vy, vz)) {
            /* block-scoped tX..tMin shadow the outer ones (:297-301): the
             * outer values stay stale for the next hit's normal */
            int32_t cx = px ? ((vx / 8) + 1) * 8 : (vx / 8) * 8;
            int32_t cy = py ? ((vy / 8) + 1) * 8 : (vy / 8) * 8;
            int32_t cz = pz ? ((vz / 8) + 1) * 8 : (vz / 8) * 8;
            float sX = ((float)cx - o.v[0]) / d.v[0];
            float sY = ((float)cy - o.v[1]) / d.v[1];
            float sZ = ((float)cz - o.v[2]) / d.v[2];
            float sMin = fminf(sX, fminf(sY, sZ));
            ray->o = vadd(o, vscale(sMin + EPS, d));
            if (same_v(ray->o, o)) return stationary(c), EMPTY_VAL;
            continue;
        }
        uint32_t col = lookup_voxel(c, reg, vx, vy, vz);
        if (col != EMPTY_VAL) {
            v3f n = normal_from_t(tX, tY, tZ, tMin, d);
            uint32_t lit = apply_lighting(c, col, n, rwp, o);
            ray3 sr = {o, V3(c->lit->light_dir[0], c->lit->light_dir[1], c->lit->light_dir[2])};
            return lit * (uint32_t)!shadow_scene_original(c, sr, cr);
        }
        nX = next_plane(px, o.v[0]); nY = next_plane(py, o.v[1]); nZ = next_plane(pz, o.v[2]);
        tX = (nX - o.v[0]) / d.v[0];
        tY = (nY - o.v[1]) / d.v[1];
        tZ = (nZ - o.v[2]) / d.v[2];
        tMin = fminf(tX, fminf(tY, tZ));
        ray->o = vadd(o, vscale(tMin + EPS, d));
        if (same_v(ray->o, o)) return stationary(c), EMPTY_VAL;
    }
    return EMPTY_VAL;
}

/* Ray::convertRayToLongestAxisDirection (Ray.cuh:19-71) */
static ray3 to_longest_axis(ray3 r, uint32_t* L, uint32_t* M, uint32_t* S) {
    float ax = fabsf(r.d.v[0]), ay = fabsf(r.d.v[1]), az = fabsf(r.d.v[2]);
    float k;
    if (ax > ay && ax > az) {
        *L = 0; if (ay > az) { *M = 1; *S = 2; } else { *M = 2; *S = 1; }
        k = 1.0f / ax;
    } else if (ay > az) {
        *L = 1; if (ax > az) { *M = 0; *S = 2; } else { *M = 2; *S = 0; }
        k = 1.0f / ay;
    } else {
        *L = 2; if (ax > ay) { *M = 0; *S = 1; } else { *M = 1; *S = 0; }
        k = 1.0f / az;
    }
    ray3 out = {r.o, vscale(k, r.d)};
    return out;
}

/* getLocalHitLocation (Renderer.cuh:753-758) */
static inline v3f local_hit(ray3 old, uint32_t a) {
    float t = old.d.v[a] > 0.0f ? (ceilf(old.o.v[a]) - old.o.v[a]) / old.d.v[a]
                                : (floorf(old.o.v[a]) - old.o.v[a]) / old.d.v[a];
    return vadd(old.o, vscale(t, old.d));
}

static int shadow_scene_longest(ctx* c, ray3 lr, v3i cr);

/* performVoxelSpaceJump (Renderer.cuh:696-751) and its shadow twin
 * performShadowVoxelSpaceJump (:441-492; shadow != 0: no lighting). */
static uint32_t voxel_space_jump(ctx* c, ray3* orig, v3f rwp, int32_t reg, ray3* old, ray3* ray,
                                 int32_t* g, int32_t* ad, uint32_t L, uint32_t M, uint32_t S,
                                 v3i cr, int shadow) {
    float tX = 0.0f, tY = 0.0f, tZ = 0.0f, tMin = 0.0f;
    while (!space_exists(c, reg, g[0], g[1], g[2])) {
        if (!tick(c)) return EMPTY_VAL;
        v3f o = old->o, d = old->d;
        v3i g0 = {{g[0], g[1], g[2]}};
        int32_t nx = d.v[0] > 0.0f ? ((g[0] / 8) + 1) * 8 : (g[0] / 8) * 8;
        int32_t ny = d.v[1] > 0.0f ? ((g[1] / 8) + 1) * 8 : (g[1] / 8) * 8;
        int32_t nz = d.v[2] > 0.0f ? ((g[2] / 8) + 1) * 8 : (g[2] / 8) * 8;
        tX = ((float)nx - o.v[0]) / d.v[0];
        tY = ((float)ny - o.v[1]) / d.v[1];
        tZ = ((float)nz - o.v[2]) / d.v[2];
        tMin = fminf(tX, fminf(tY, tZ)) + EPS;
        old->o = vadd(o, vscale(tMin, d));
        g[0] = f2i(floorf(old->o.v[0]));
        g[1] = f2i(floorf(old->o.v[1]));
        g[2] = f2i(floorf(old->o.v[2]));
        if (!grid_in_region(g[0], g[1], g[2])) {
            orig->o = old->o;                 /* direction of originalRay kept */
            return EMPTY_VAL;
        }
        v3i g1 = {{g[0], g[1], g[2]}};
        if (same_v(old->o, o) && same_i(g1, g0)) return stationary(c), EMPTY_VAL;
    }
    uint32_t col = lookup_voxel(c, reg, g[0], g[1], g[2]);
    if (col != EMPTY_VAL) {
        if (shadow) return col;
        v3f n = normal_from_t(tX, tY, tZ, tMin, old->d);
        uint32_t lit = apply_lighting(c, col, n, rwp, old->o);
        ray3 sr = {old->o, V3(c->lit->light_dir[0], c->lit->light_dir[1], c->lit->light_dir[2])};
        return lit * (uint32_t)!shadow_scene_longest(c, sr, cr);
    }
    float oL = old->o.v[L], dL = old->d.v[L];
    float tNext = dL > 0.0f ? (ceilf(oL) - oL) / dL : (floorf(oL) - oL) / dL;
    ray->o = vadd(old->o, vscale(tNext + EPS, old->d));
    ray->d = old->d;
    ad[M] = f2i(ray->o.v[M]) - g[M];
    ad[S] = f2i(ray->o.v[S]) - g[S];
    return CONTINUE_VAL;
}

/* One axis step of the longest-axis walk: the repeated block
 * "grid += diff; exists? else jump; lookup; hit -> lighting + shadow"
 * (Renderer.cuh:807-823, 825-841, 846-862, 867-883, 886-901 and the shadow
 * twins :542-617).  Returns 0 to continue the step sequence, 1 when `*res`
 * must be returned from the grid walk, 2 for the loop's `continue`. */
static int axis_step(ctx* c, ray3* orig, v3f rwp, int32_t reg, ray3* old, ray3* ray, int32_t* g,
                     int32_t* ad, uint32_t L, uint32_t M, uint32_t S, v3i cr, int shadow,
                     uint32_t axis, int long_axis_hit, uint32_t* res) {
    g[axis] += ad[axis];
    if (!space_exists(c, reg, g[0], g[1], g[2])) {
        uint32_t jr = voxel_space_jump(c, orig, rwp, reg, old, ray, g, ad, L, M, S, cr, shadow);
        if (c->aborted) { *res = EMPTY_VAL; return 1; }
        if (jr != CONTINUE_VAL) { *res = jr; return 1; }
        return 2;
    }
    uint32_t col = lookup_voxel(c, reg, g[0], g[1], g[2]);
    if (col != EMPTY_VAL) {
        if (shadow) { *res = col; return 1; }
        v3f n = V3(0.0f, 0.0f, 0.0f);
        n.v[axis] = copysignf(1.0f, -ray->d.v[axis]);
        v3f hit = long_axis_hit ? ray->o : local_hit(*old, axis);
        uint32_t lit = apply_lighting(c, col, n, rwp, hit);
        ray3 sr = {hit, V3(c->lit->light_dir[0], c->lit->light_dir[1], c->lit->light_dir[2])};
        *res = lit * (uint32_t)!shadow_scene_longest(c, sr, cr);
        return 1;
    }
    return 0;
}

/* rayMarchVoxelGridLongestAxis (Renderer.cuh:760-915) and its shadow twin
 * shadowRayMarchVoxelGridLongestAxis (:495-631). */
static uint32_t grid_longest(ctx* c, ray3* orig, v3f rwp, int32_t reg, v3i cr, int shadow) {
    uint32_t L, M, S;
    ray3 old = to_longest_axis(*orig, &L, &M, &S);
    int32_t g[3] = {f2i(orig->o.v[0]), f2i(orig->o.v[1]), f2i(orig->o.v[2])};
    int32_t ad[3] = {0, 0, 0};
    ad[L] = orig->d.v[L] < 0.0f ? -1 : 1;
    float t = ad[L] > 0 ? ((float)g[L] + EPS + 1.0f - orig->o.v[L]) / (float)ad[L]
                        : ((float)g[L] - EPS - orig->o.v[L]) / (float)ad[L];
    ray3 ray = {vadd(old.o, vscale(t, old.d)), old.d};
    ad[M] = f2i(ray.o.v[M]) - g[M];
    ad[S] = f2i(ray.o.v[S]) - g[S];
    int mid_floor = ray.d.v[M] < 0.0f;     /* decimalToIntFunc (:784) */
    uint32_t res;
    while (grid_in_region(g[L] + ad[L], g[M] + ad[M], g[S] + ad[S])) {
        if (!tick(c)) return EMPTY_VAL;
        int r;
        if (ad[S] != 0 && ad[M] != 0) {
            float om = old.o.v[M];
            float t1 = ((mid_floor ? floorf(om) : ceilf(om)) - om) / old.d.v[M];
            float sp = old.o.v[S] + old.d.v[S] * t1;
            int32_t sd = f2i(floorf(sp)) - g[S];
            uint32_t a0 = M, a1 = S;
            if (sd != 0) { a0 = S; a1 = M; }
            r = axis_step(c, orig, rwp, reg, &old, &ray, g, ad, L, M, S, cr, shadow, a0, 0, &res);
            if (r == 1) return res;
            if (r == 2) continue;
            r = axis_step(c, orig, rwp, reg, &old, &ray, g, ad, L, M, S, cr, shadow, a1, 0, &res);
            if (r == 1) return res;
            if (r == 2) continue;
        } else if (ad[M] != 0) {
            r = axis_step(c, orig, rwp, reg, &old, &ray, g, ad, L, M, S, cr, shadow, M, 0, &res);
            if (r == 1) return res;
            if (r == 2) continue;
        } else if (ad[S] != 0) {
            r = axis_step(c, orig, rwp, reg, &old, &ray, g, ad, L, M, S, cr, shadow, S, 0, &res);
            if (r == 1) return res;
            if (r == 2) continue;
        }
        r = axis_step(c, orig, rwp, reg, &old, &ray, g, ad, L, M, S, cr, shadow, L, 1, &res);
        if (r == 1) return res;
        if (r == 2) continue;
        old = ray;
        ray.o = vadd(ray.o, ray.d);
        ad[M] = f2i(ray.o.v[M]) - g[M];
        ad[S] = f2i(ray.o.v[S]) - g[S];
    }
    if (c->aborted) return EMPTY_VAL;
    orig->o = old.o;                        /* :912 */
    return shadow ? shadow_grid_original(c, orig, reg) : grid_original(c, orig, rwp, reg, cr);
}

/* isInShadowRayMarchVoxelSceneLongestAxis (Renderer.cuh:633-694) */
static int shadow_scene_longest(ctx* c, ray3 lr, v3i cr) {
    if (!c->lit->use_shadows) return 0;
    c->in_shadow = 1;
    cycle cyc = cycle_start(cr, lr.o);
    while (in_scene(c, cr)) {
        if (!tick(c)) return 0;
        int32_t reg = region_at(c, cr);
        cycle cyc1 = cycle_start(cr, lr.o);
        while (reg < 0) {
            if (!tick(c)) return 0;
            if (!skip_null_region(c, &cr, &lr, 0, &reg)) return 0;
            if (cycle_step(&cyc1, cr, lr.o)) return stationary(c);
        }
        uint32_t col = grid_longest(c, &lr, V3(0, 0, 0), reg, cr, 1);
        if (c->aborted) return 0;
        if (col != EMPTY_VAL) return 1;
        advance_region(&cr, &lr);
        if (cycle_step(&cyc, cr, lr.o)) return stationary(c);
    }
    return 0;
}

/* rayMarchVoxelScene (Renderer.cuh:338-434) / rayMarchVoxelSceneLongestAxis (:917-1010) */
static uint32_t scene_march(ctx* c, ray3 world, uint32_t scale, int algo) {
    const or_scene* s = c->s;
    ray3 sr = {vscale((float)scale, vsub(world.o, c->translation)), world.d};   /* Ray.cuh:14-17 */
    v3f d = sr.d;
    v3i cr = {{f2i(floorf(sr.o.v[0] / (float)BLOCK)), f2i(floorf(sr.o.v[1] / (float)BLOCK)),
               f2i(floorf(sr.o.v[2] / (float)BLOCK))}};
    /* entry clip (:349-373) */
    cycle cyc0 = cycle_start(cr, sr.o);
    while (!in_scene(c, cr)) {
        if (!tick(c)) return 0;
        int32_t hi = (int32_t)(s->D + (uint32_t)s->min_coord), lo = 0 + s->min_coord;
        int32_t nx = d.v[0] < 0.0f ? hi : lo, ny = d.v[1] < 0.0f ? hi : lo, nz = d.v[2] < 0.0f ? hi : lo;
        float tX = ((float)(nx * BLOCK) - sr.o.v[0]) / d.v[0];
        float tY = ((float)(ny * BLOCK) - sr.o.v[1]) / d.v[1];
        float tZ = ((float)(nz * BLOCK) - sr.o.v[2]) / d.v[2];
        if (tX <= 0.0f) tX = INFINITY;
        if (tY <= 0.0f) tY = INFINITY;
        if (tZ <= 0.0f) tZ = INFINITY;
        float tMin = fminf(tX, fminf(tY, tZ));
        if (tMin == INFINITY) return 0;
        sr.o = vadd(sr.o, vscale(tMin + EPS, d));
        cr.v[0] = f2i(floorf(sr.o.v[0] / (float)BLOCK));
        cr.v[1] = f2i(floorf(sr.o.v[1] / (float)BLOCK));
        cr.v[2] = f2i(floorf(sr.o.v[2] / (float)BLOCK));
        if (cycle_step(&cyc0, cr, sr.o)) return stationary(c);
    }
    ray3 lr = {vscale(1.0f, vsub(sr.o, V3((float)(cr.v[0] * BLOCK), (float)(cr.v[1] * BLOCK),
                                          (float)(cr.v[2] * BLOCK)))), d};
    cycle cyc = cycle_start(cr, lr.o);
    while (in_scene(c, cr)) {
        if (!tick(c)) return 0;
        int32_t reg = region_at(c, cr);
        cycle cyc1 = cycle_start(cr, lr.o);
        while (reg < 0) {
            if (!tick(c)) return 0;
            if (!skip_null_region(c, &cr, &lr, 0, &reg)) return 0;
            if (cycle_step(&cyc1, cr, lr.o)) return stationary(c);
        }
        v3f rwp = vadd(c->translation, V3((float)(cr.v[0] * BLOCK), (float)(cr.v[1] * BLOCK),
                                          (float)(cr.v[2] * BLOCK)));
        uint32_t col = algo == OR_ALGO_ORIGINAL ? grid_original(c, &lr, rwp, reg, cr)
                                                : grid_longest(c, &lr, rwp, reg, cr, 0);
        if (c->aborted) return 0;
        if (col != EMPTY_VAL) return col;
        advance_region(&cr, &lr);
        if (cycle_step(&cyc, cr, lr.o)) return stationary(c);
    }
    return 0;
}

/* ------------------------------------------------------------ camera */

#define OR_PI 3.141592f   /* MathConstants.cuh:3 */

/* Camera::Camera (Camera.cuh:11-23) */
void or_camera_make(const float eye[3], const float look_at[3], const float up[3], float fov_deg,
                    float aspect, or_camera* out) {
    float half_h = tanf((fov_deg * OR_PI / 180.f) / 2.0f);
    float half_w = half_h * aspect;
    v3f o = V3(eye[0], eye[1], eye[2]);
    v3f w = vunit(vsub(V3(look_at[0], look_at[1], look_at[2]), o));
    v3f u = vunit(vcross(w, V3(up[0], up[1], up[2])));
    v3f v = vcross(u, w);
    v3f llc = vadd(vsub(vsub(o, vscale(half_w, u)), vscale(half_h, v)), w);
    v3f hor = vscale(2 * half_w, u);
    v3f ver = vscale(2 * half_h, v);
    for (int i = 0; i < 3; ++i) {
        out->origin[i] = o.v[i]; out->lower_left[i] = llc.v[i]; out->horizontal[i] = hor.v[i];
        out->vertical[i] = ver.v[i]; out->forward[i] = w.v[i];
    }
}

/* setupConstantValues (Main.cu:26-42) */
void or_lighting_default(or_lighting* out) {
    v3f L = vunit(V3(1.0f, 1.0f, 1.0f));
    for (int i = 0; i < 3; ++i) { out->light_dir[i] = L.v[i]; out->light_color[i] = 1.0f; }
    out->light_pos[0] = 10.0f; out->light_pos[1] = 10.0f; out->light_pos[2] = -10.0f;
    out->use_point_light = 0;
    out->use_shadows = 1;
}

/* calculateWorldRay (Renderer.cuh:1013-1022) + Camera::generateRay (Camera.cuh:25-29),
 * then the kernel body (Renderer.cuh:1033-1063). */
static uint32_t render_pixel(const or_scene* s, int algo, const or_camera* cam, const or_lighting* lit,
                             v3f tr, uint32_t scale, uint32_t W, uint32_t H, uint32_t x, uint32_t y,
                             uint64_t* bytes, uint64_t* st) {
    float u = ((float)x + 0.5f) / (float)W;
    float v = ((float)(H - y) + 0.5f) / (float)H;
    v3f llc = V3(cam->lower_left[0], cam->lower_left[1], cam->lower_left[2]);
    v3f hor = V3(cam->horizontal[0], cam->horizontal[1], cam->horizontal[2]);
    v3f ver = V3(cam->vertical[0], cam->vertical[1], cam->vertical[2]);
    v3f org = V3(cam->origin[0], cam->origin[1], cam->origin[2]);
    v3f ro = vadd(vadd(llc, vscale(u, hor)), vscale(v, ver));
    ray3 world = {ro, vunit(vsub(ro, org))};
    ctx c; memset(&c, 0, sizeof c);
    c.s = s; c.lit = lit; c.translation = tr; c.st = st;
    uint32_t col = scene_march(&c, world, scale, algo);
    if (c.aborted) { col = 0; c.bytes = 0; }   /* never finishes: only the write counts */
    c.bytes += 4;                /* the pixel write */
    if (bytes) *bytes = c.bytes;
    return col;
}

int or_render(const or_scene* s, int algo, const or_camera* cam, const or_lighting* lit,
              const float translation[3], uint32_t scale, uint32_t width, uint32_t height,
              uint32_t row_begin, uint32_t row_end, uint32_t* out, uint64_t* bytes_out, int nthreads) {
    if (!s || !cam || !lit || !out || row_end > height || row_begin > row_end) return -1;
    v3f tr = V3(translation ? translation[0] : 0.0f, translation ? translation[1] : 0.0f,
                translation ? translation[2] : 0.0f);
    uint64_t total = 0;
    long rows = (long)(row_end - row_begin);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total)
#endif
    for (long r = 0; r < rows; ++r) {
        uint32_t y = row_begin + (uint32_t)r;
        for (uint32_t x = 0; x < width; ++x) {
            uint64_t b = 0;
            out[(size_t)r * width + x] = render_pixel(s, algo, cam, lit, tr, scale, width, height, x, y, &b, NULL);
            total += b;
        }
    }
    (void)nthreads;
    if (bytes_out) *bytes_out = total;
    return 0;
}

int or_render_pixels(const or_scene* s, int algo, const or_camera* cam, const or_lighting* lit,
                     const float translation[3], uint32_t scale, uint32_t width, uint32_t height,
                     const uint32_t* px, const uint32_t* py, size_t n, uint32_t* out,
                     uint64_t* bytes_per_pixel) {
    if (!s || !cam || !lit || !out) return -1;
    v3f tr = V3(translation ? translation[0] : 0.0f, translation ? translation[1] : 0.0f,
                translation ? translation[2] : 0.0f);
    for (size_t i = 0; i < n; ++i) {
        uint64_t b = 0;
        out[i] = render_pixel(s, algo, cam, lit, tr, scale, width, height, px[i], py[i], &b, NULL);
        if (bytes_per_pixel) bytes_per_pixel[i] = b;
    }
    return 0;
}

/* Work statistics of rows [row_begin,row_end): st[2*OR_STAT_N] = counts of
 * region reads, existence checks, cluster skips, lookups, probes, hits, loop
 * iterations, existence checks outside the region and those of them whose
 * `short` cluster id aliases into the directory, for primary (st[0..8]) and
 * shadow (st[9..17]) walks. */
int or_render_stats(const or_scene* s, int algo, const or_camera* cam, const or_lighting* lit,
                    const float translation[3], uint32_t scale, uint32_t width, uint32_t height,
                    uint32_t row_begin, uint32_t row_end, uint64_t* st) {
    if (!s || !cam || !lit || !st) return -1;
    v3f tr = V3(translation ? translation[0] : 0.0f, translation ? translation[1] : 0.0f,
                translation ? translation[2] : 0.0f);
    memset(st, 0, sizeof(uint64_t) * 2 * OR_STAT_N);
    for (uint32_t y = row_begin; y < row_end; ++y)
        for (uint32_t x = 0; x < width; ++x) {
            uint64_t b = 0;
            (void)render_pixel(s, algo, cam, lit, tr, scale, width, height, x, y, &b, st);
        }
    return 0;
}

/* Per-pixel work statistics of rows [row_begin,row_end): st[(r*width+x)*2*OR_STAT_N + k]
 * (same counters as or_render_stats), for wave-divergence studies. */
int or_pixel_stats(const or_scene* s, int algo, const or_camera* cam, const or_lighting* lit,
                   const float translation[3], uint32_t scale, uint32_t width, uint32_t height,
                   uint32_t row_begin, uint32_t row_end, uint64_t* st, int nthreads) {
    if (!s || !cam || !lit || !st || row_end > height || row_begin > row_end) return -1;
    v3f tr = V3(translation ? translation[0] : 0.0f, translation ? translation[1] : 0.0f,
                translation ? translation[2] : 0.0f);
    long rows = (long)(row_end - row_begin);
    memset(st, 0, sizeof(uint64_t) * 2 * OR_STAT_N * (size_t)rows * width);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (long r = 0; r < rows; ++r)
        for (uint32_t x = 0; x < width; ++x) {
            uint64_t b = 0;
            (void)render_pixel(s, algo, cam, lit, tr, scale, width, height, x, row_begin + (uint32_t)r, &b,
                               st + ((size_t)r * width + x) * 2 * OR_STAT_N);
        }
    (void)nthreads;
    return 0;
}
