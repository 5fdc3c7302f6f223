/*
 * vr_oracle.h -- CPU restatement of the VoxelRaymarcher hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the shipped product (libvr.so, the
 * CLI, the Python host package) links, loads or calls this code.  It is used
 * by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
 * checker -- never as the thing measured on the GPU.
 *
 * PARITY UNPINNED: the reference (lukeduball/VoxelRaymarcher, CUDA 11.2)
 * ships no tests, golden vectors or fixtures, its only scene file is a
 * stripped large blob, and running any build of its sources was refused by
 * the environment.  This restatement follows the
 * reference source text line by line (citations in vr_oracle.c) under the
 * floating-point policy of SURVEY.md section 8c / 9:
 *   no contraction, correctly rounded / and sqrtf, fminf/fmaxf, truncating
 *   saturating float->int (NaN -> 0, CUDA __float2int_rz semantics).
 */
#ifndef VR_ORACLE_H
#define VR_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* = StorageType {VOXEL_CLUSTER_STORE, HASH_TABLE} (VoxelFunctions.cuh:37) */
enum { OR_STORE_VCS = 0, OR_STORE_HASHTABLE = 1 };
/* = rayMarchFunctionID (Main.cu:58-68,119-128): 0 longest axis, 1 original */
enum { OR_ALGO_LONGESTAXIS = 0, OR_ALGO_ORIGINAL = 1 };

/* Camera fields in Camera.cuh:34-39 order. */
typedef struct {
    float origin[3];
    float lower_left[3];
    float horizontal[3];
    float vertical[3];
    float forward[3];
} or_camera;

/* The __constant__ lighting block of VoxelFunctions.cuh:27-35 as set by
 * setupConstantValues (Main.cu:26-42). */
typedef struct {
    float light_dir[3];
    float light_color[3];
    float light_pos[3];
    int32_t use_point_light;
    int32_t use_shadows;
} or_lighting;

typedef struct or_scene or_scene;

/* Camera::Camera (Camera.cuh:11-23), host side. */
void or_camera_make(const float eye[3], const float look_at[3], const float up[3],
                    float fov_deg, float aspect, or_camera* out);

/* Main.cu:26-42 defaults (LIGHT_DIRECTION = normalize(1,1,1), white, shadows on). */
void or_lighting_default(or_lighting* out);

/* VoxelSceneCPU::insertVoxel + generateVoxelScene (VoxelSceneCPU.cuh:16-93)
 * over n voxels (xyz interleaved, 3n int32) with packed 0x00RRGGBB colours.
 * Later duplicates overwrite earlier ones (unordered_map assignment, :46). */
int or_scene_build(int store, const int32_t* xyz, const uint32_t* rgb, size_t n,
                   or_scene** out);
void or_scene_free(or_scene* s);
uint32_t or_scene_diameter(const or_scene* s);
int32_t or_scene_min_coord(const or_scene* s);
uint32_t or_scene_region_count(const or_scene* s);

/* Lookup restated from the storage structures (for known-answer tests):
 * local coords inside region (rx,ry,rz); returns colour or 1<<30. */
uint32_t or_scene_lookup(const or_scene* s, int32_t rx, int32_t ry, int32_t rz,
                         int32_t x, int32_t y, int32_t z);

/* Test helper: the cuckoo table (1, 2) key sits in within region index r (0 absent,
 * -1 not a hashtable region); *rehashed = that region's table was rehashed. */
int or_scene_cuckoo_table(const or_scene* s, uint32_t r, uint32_t key, int* rehashed);

/* Diagnostic: an iteration budget per pixel for every later render
 * (process-global; UINT64_MAX = none, the default).  A pixel that exceeds it
 * renders as 0 with 4 bytes, like a walk that never finishes. */
void or_set_iter_budget(uint64_t budget);
/* Test hook: the region-level loops' cycle test (Brent) on a synthetic state sequence --
 * `prefix` distinct states, then `period` distinct states repeating (0: none); the round
 * the repeat is found at, or -1. */
int64_t or_cycle_selftest(uint32_t prefix, uint32_t period, uint32_t max_rounds);

/* Known-answer helpers. */
int32_t or_hash1(int32_t key, uint32_t offset);                 /* CuckooHashTable.cuh:181-190 */
int32_t or_hash2(int32_t key, uint32_t prime);                  /* CuckooHashTable.cuh:193-202 */
uint32_t or_cluster_id(uint32_t x, uint32_t y, uint32_t z);     /* VoxelClusterStore.cuh:21-24 */
uint32_t or_generate_3d_point(uint32_t x, uint32_t y, uint32_t z); /* VoxelFunctions.cuh:41-46 */

/* Render rows [row_begin,row_end) of a W x H image into out
 * ((row_end-row_begin)*W packed 0x00RRGGBB words).  Mirrors the kernels
 * rayMarchSceneOriginal / rayMarchSceneJumpAxis (Renderer.cuh:1033-1063).
 * bytes_out (optional) receives the SURVEY 8(d) algorithmic byte count.
 * nthreads <= 0 -> OpenMP default. */
int or_render(const or_scene* s, int algo, const or_camera* cam, const or_lighting* lit,
              const float translation[3], uint32_t scale, uint32_t width, uint32_t height,
              uint32_t row_begin, uint32_t row_end, uint32_t* out, uint64_t* bytes_out,
              int nthreads);

/* Render a list of pixels (px[i], py[i]); per-pixel bytes optional. */
int or_render_pixels(const or_scene* s, int algo, const or_camera* cam, const or_lighting* lit,
                     const float translation[3], uint32_t scale, uint32_t width, uint32_t height,
                     const uint32_t* px, const uint32_t* py, size_t n, uint32_t* out,
                     uint64_t* bytes_per_pixel);

/* Work statistics (single-threaded): 2 x 9 counters, primary then shadow:
 * region reads, existence checks, cluster skips, lookups, key probes, hits, loop iterations,
 * existence checks at coordinates outside [0,64), and those whose `short` cluster id still
 * lands in the directory (VoxelClusterStore.cuh:21-24 aliasing). */
int or_render_stats(const or_scene* s, int algo, const or_camera* cam, const or_lighting* lit,
                    const float translation[3], uint32_t scale, uint32_t width, uint32_t height,
                    uint32_t row_begin, uint32_t row_end, uint64_t* st);

/* Per-pixel version: st[(r * width + x) * 18 + k] for row r - row_begin. OpenMP. */
int or_pixel_stats(const or_scene* s, int algo, const or_camera* cam, const or_lighting* lit,
                   const float translation[3], uint32_t scale, uint32_t width, uint32_t height,
                   uint32_t row_begin, uint32_t row_end, uint64_t* st, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
