/*
 * vr.h -- C ABI of the MI355X-native voxel ray-march renderer (libvr.so).
 *
 * Drop-in boundary for the hot path of lukeduball/VoxelRaymarcher.  Every
 * entry point names the reference interface it replaces (paths relative to
 * /root/reference/VoxelRaymarcher/src).  No HIP or torch types appear in the
 * signatures: device buffers are plain pointers, streams are `void*`
 * (a hipStream_t, NULL = the null stream).
 *
 * Return codes: VR_OK (0) or a negative VR_E_*; vr_last_error() gives a
 * thread-local message for the last failure on the calling thread.
 */
#ifndef VR_H
#define VR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VR_OK 0
#define VR_E_INVALID (-1)   /* bad argument */
#define VR_E_HIP (-2)       /* HIP runtime error / no device */
#define VR_E_NOMEM (-3)     /* host or device allocation failed */
#define VR_E_IO (-4)        /* file could not be read or written */
#define VR_E_BUILD (-5)     /* storage structure could not be built */
#define VR_E_PARSE (-6)     /* malformed .vox line (std::stoi would throw) */

/* = enum class StorageType {VOXEL_CLUSTER_STORE, HASH_TABLE}
 *   (geometry/VoxelFunctions.cuh:37; selected in main/Main.cu:45-55) */
typedef enum { VR_STORE_VCS = 0, VR_STORE_HASHTABLE = 1 } vr_store;

/* = rayMarchFunctionID (main/Main.cu:58-68,119-128):
 *   0 -> rayMarchSceneJumpAxis, 1 -> rayMarchSceneOriginal */
typedef enum { VR_ALGO_LONGESTAXIS = 0, VR_ALGO_ORIGINAL = 1 } vr_algo;

/* = class Camera field order (renderer/camera/Camera.cuh:34-39) */
typedef struct {
    float origin[3];
    float lower_left[3];
    float horizontal[3];
    float vertical[3];
    float forward[3];
} vr_camera;

/* = the __constant__ block LIGHT_DIRECTION / LIGHT_COLOR / LIGHT_POSITION /
 *   USE_POINT_LIGHT / USE_SHADOWS (geometry/VoxelFunctions.cuh:27-35) as
 *   uploaded by setupConstantValues (main/Main.cu:26-42). */
typedef struct {
    float light_dir[3];
    float light_color[3];
    float light_pos[3];
    int32_t use_point_light;
    int32_t use_shadows;
} vr_lighting;

/* Immutable per-device scene: region table + VCS or cuckoo storage images.
 * Replaces VoxelSceneCPU::generateVoxelScene's device pointer table
 * (geometry/VoxelSceneCPU.cuh:49-93) plus the device-side virtual adapters
 * built by the generateVoxelScene kernel (renderer/Renderer.cuh:1066-1086). */
typedef struct vr_scene vr_scene;

typedef struct {
    uint32_t diameter;       /* = VoxelSceneCPU::getArrayDiameter (VoxelSceneCPU.cuh:107-110) */
    int32_t min_coord;       /* = VoxelSceneCPU::getMinCoord (:118-121) */
    uint32_t region_count;   /* non-empty 64^3 regions */
    uint32_t store;          /* vr_store */
    uint64_t voxel_count;    /* distinct voxels after duplicate resolution */
    uint64_t device_bytes;   /* HBM footprint of the scene */
    int32_t device;
} vr_scene_info;

/* Synthetic grid generator; counter-hash occupancy. */
typedef struct {
    uint32_t n;              /* grid side, multiple of 64, <= 1024 */
    double p_region, p_cluster, p_voxel;
    uint64_t seed;
} vr_synth_params;

/* Camera::Camera(o, lookAt, globalUp, fov, aspect) (Camera.cuh:11-23), host. */
int vr_camera_make(const float eye[3], const float look_at[3], const float up[3],
                   float fov_deg, float aspect, vr_camera* out);

/* setupConstantValues defaults (Main.cu:26-42): directional light
 * normalize(1,1,1), white, point light at (10,10,-10) disabled, shadows on. */
int vr_lighting_default(vr_lighting* out);

/* Light direction as the reference uploads it: makeUnitVector(dir)
 * (Main.cu:28, Vector3.cuh:162-165: v / sqrtf(x*x+y*y+z*z), three divides).
 * VR_E_INVALID for a zero, NaN or infinite vector. Other lighting fields are
 * plain data (light_color, light_pos, use_point_light, use_shadows). */
int vr_lighting_set_direction(vr_lighting* lit, const float dir[3]);

/* VoxelSceneCPU::insertVoxel for every voxel (VoxelSceneCPU.cuh:16-46), then
 * generateVoxelScene(storageType) (:49-93) -- VoxelClusterStore ctor
 * (storage/VoxelClusterStore.cuh:37-85) or CuckooHashTable ctor
 * (storage/CuckooHashTable.cuh:20-49,97-178) per region -- and the upload to
 * `device`.  xyz: 3n int32 world voxel coordinates; rgb: n colours
 * 0x00RRGGBB (must be < 2^24).  Later duplicates overwrite earlier ones. */
int vr_scene_create(int device, vr_store store, const int32_t* xyz, const uint32_t* rgb,
                    size_t n, vr_scene** out);

/* Where the scene image is built.  DEVICE: region
 * bucketing, a stable radix sort by (region, cluster, key), last-insertion
 * dedupe, mask records and cuckoo tables on the GPU; HOST: the same on the
 * CPU.  Both produce byte-identical device images (vr_scene_digest).  AUTO =
 * DEVICE (what vr_scene_create uses). */
typedef enum { VR_BUILD_AUTO = 0, VR_BUILD_DEVICE = 1, VR_BUILD_HOST = 2 } vr_build;

/* vr_scene_create with the voxel arrays optionally already on `device`
 * (inputs_on_device != 0) and an explicit builder; `stream` orders the device
 * build (NULL = default stream).  Returns when the scene is ready. */
int vr_scene_create_ex(int device, vr_store store, const int32_t* xyz, const uint32_t* rgb, size_t n,
                       int inputs_on_device, vr_build build, void* stream, vr_scene** out);

/* FNV-1a digest of each device buffer (region table, VCS masks, VCS colours,
 * cuckoo meta, cuckoo slots) -- to compare builds. */
int vr_scene_digest(const vr_scene* s, uint64_t out[5]);

/* VoxelFile::readVoxelFile (geometry/VoxelFile.cuh:9-35) + vr_scene_create.
 * Unlike the reference the path is used as given (no "resources/" prefix).
 * Accepts the .vox CSV (parsed in parallel, same rules and first-error line)
 * or the .vxb binary sidecar (detected by its magic). */
int vr_scene_load_vox(int device, vr_store store, const char* path, vr_scene** out);

int vr_scene_get_info(const vr_scene* s, vr_scene_info* out);
void vr_scene_destroy(vr_scene* s);

/* rayMarchSceneOriginal / rayMarchSceneJumpAxis (Renderer.cuh:1033-1063) as
 * launched by runRaymarchingKernel (Main.cu:105-163), for image rows
 * [row_begin, row_end) of a width x height frame.  out_dev: device buffer of
 * (row_end-row_begin)*width uint32, row-major, y = 0 the top row, each the
 * packed 0x00RRGGBB word the reference hands to writeColorToFramebuffer
 * (Renderer.cuh:1024-1031).  translation/scale = VoxelSceneInfo
 * (renderer/VoxelSceneInfo.cuh:5-15).  Asynchronous on `stream`. */
int vr_render(const vr_scene* s, vr_algo algo, const vr_camera* cam, const vr_lighting* lit,
              const float translation[3], uint32_t scale, uint32_t width, uint32_t height,
              uint32_t row_begin, uint32_t row_end, uint32_t* out_dev, void* stream);

/* Multi-GPU tile partition: the frame is cut into bands of band_rows rows;
 * band b belongs to rank b % nranks.  out_dev holds this rank's bands packed
 * in order: ceil(ceil(height/band_rows)/nranks)*band_rows*width uint32
 * (rows past the frame or past this rank's last band are written as 0), so
 * every rank's buffer has the same size for an RCCL gather. */
int vr_render_bands(const vr_scene* s, vr_algo algo, const vr_camera* cam, const vr_lighting* lit,
                    const float translation[3], uint32_t scale, uint32_t width, uint32_t height,
                    uint32_t band_rows, uint32_t rank, uint32_t nranks, uint32_t* out_dev,
                    void* stream);
/* Number of uint32 words vr_render_bands writes per rank. */
uint64_t vr_band_buffer_words(uint32_t width, uint32_t height, uint32_t band_rows, uint32_t nranks);

/* The 2-D tile deal (vr_render_opts.tile_cols): every band_rows-row band of the frame is
 * cut into column blocks of tile_cols pixels, block j of band b -> rank (j + stride*b) %
 * nranks.  Row bands alone put a cluster of expensive rows (C5's crawl rows) on one or two
 * ranks; the deal gives every rank a share of every band while each 8x8 wave tile stays
 * whole.  out_dev: vr_tile_buffer_words(...) uint32 per rank (same for every rank). */
int vr_render_tiles(const vr_scene* s, vr_algo algo, const vr_camera* cam, const vr_lighting* lit,
                    const float translation[3], uint32_t scale, uint32_t width, uint32_t height,
                    uint32_t band_rows, uint32_t tile_cols, uint32_t rank, uint32_t nranks,
                    uint32_t* out_dev, void* stream);
uint64_t vr_tile_buffer_words(uint32_t width, uint32_t height, uint32_t band_rows, uint32_t tile_cols,
                              uint32_t nranks);
/* The stride the deal uses when deal_stride is 0: 3 (a knight's-move deal) unless it
 * shares a factor with nranks, else 1. */
uint32_t vr_deal_stride_default(uint32_t nranks);
/* Rank 0's reassembly after the gather: parts_dev holds the nranks tile buffers back to
 * back (each vr_tile_buffer_words(...) pixels of elem_bytes bytes: 4 for the packed words,
 * 3 for RGB8), frame_dev receives the width x height image (row-major, elem_bytes per
 * pixel).  deal_stride 0 = the default.  Asynchronous on `stream`. */
int vr_assemble_tiles(const void* parts_dev, void* frame_dev, uint32_t elem_bytes, uint32_t width,
                      uint32_t height, uint32_t band_rows, uint32_t tile_cols, uint32_t nranks,
                      uint32_t deal_stride, void* stream);

/* Kernel implementations behind vr_render*: all produce identical pixels.
 * (Value 2 was a persistent state-machine kernel, retired in round 3: it was
 * never the fastest; it is rejected with VR_E_INVALID.) */
typedef enum {
    VR_KERNEL_AUTO = 0,         /* the fastest measured for the (store, algorithm) pair */
    VR_KERNEL_TILE = 1,         /* one lane per pixel, one wave per 8x8 tile (vr_march.hip) */
    VR_KERNEL_TILE_REWALK = 3   /* the tile kernel whose crawl pass walks every deferred pixel
                                   from its start instead of resuming it (cross-check) */
} vr_kernel;

/* Full-control render (the other vr_render* calls are wrappers of this):
 * rows [row_begin,row_end) of the frame cut into bands of band_rows rows,
 * band b rendered when b % nranks == rank; out_dev gets this rank's bands
 * packed as in vr_render_bands.  bytes_dev (optional, device uint64,
 * caller-zeroed) accumulates the SURVEY.md 8(d) algorithmic bytes.
 *
 * Versioned by its leading size: set struct_size = sizeof(vr_render_opts)
 * (vr_render_opts_init does, with every other field at its default).  The
 * library rejects (VR_E_INVALID) a struct_size below VR_RENDER_OPTS_MIN_SIZE --
 * the layout before this field existed began with `kernel` (0..3), so a caller
 * built against it is refused instead of having fields read past its struct --
 * and treats fields that lie past struct_size as zero (callers built against
 * an older, shorter version of this layout keep working). */
typedef struct {
    uint32_t struct_size; /* sizeof(vr_render_opts) as the caller was compiled */
    uint32_t kernel;      /* vr_kernel */
    uint32_t row_begin, row_end;
    uint32_t band_rows;   /* 0 = one band covering [row_begin,row_end) */
    uint32_t rank, nranks;
    uint32_t defer_cap;   /* records in the crawl pass's deferral list: 0 = the default (16384);
                             smaller values exercise its overflow path (tests) */
    uint64_t* bytes_dev;
    uint32_t schedule;    /* vr_schedule: the tile pass's work order (pixels never depend on it) */
    uint32_t reserved;    /* 0 */
    /* (optional, device uint64[2], caller-zeroed; read only with bytes_dev) the part of
     * bytes_dev's count that the kernels credit without loading it: [0] cluster-skip crawl
     * iterations fast-forwarded in closed form (Renderer.cuh:290-306, performVoxelSpaceJump
     * :707-725), [1] the existence-read bytes credited without a load -- 4 per fast-forwarded
     * iteration and 4 per crawl-pass skip step answered from its LDS copy of the region's
     * cluster-existence bits.  bytes_dev - [1] = the bytes the kernels' own loads stand for. */
    uint64_t* stats_dev;
    /* (round 5) vr_occupancy: which occupancy variant of the tile pass renders.  The
     * uninstrumented cuckoo `original` and VCS `longestaxis` walks have a higher-occupancy
     * variant for frames in flight; AUTO takes it when another stream's launch is still
     * running on the device.  Pixels never depend on it.  Instrumented launches (bytes_dev)
     * always run the lone variant. */
    uint32_t occupancy;
    /* (round 5) 2-D tile deal.  0: bands of whole rows, band b -> rank b % nranks (the layout
     * described at vr_render_bands).  > 0: the rows [row_begin,row_end) are cut into bands of
     * band_rows rows (0 = one band) and every band into column blocks of tile_cols pixels; block
     * j of band b belongs to rank (j + stride * b) % nranks, stride = deal_stride (0 =
     * vr_deal_stride_default(nranks)).  out_dev then holds, for every band in order, this rank's
     * blocks of that band in increasing j, each band_rows x tile_cols, as rows of
     * ceil(ceil(width/tile_cols)/nranks) * tile_cols words (vr_tile_buffer_words); pixels past
     * the frame are written as 0.  Every rank gets a share of every band, so expensive rows
     * (long walks are spatially clustered) are spread over all ranks. */
    uint32_t tile_cols;
    uint32_t deal_stride;
    uint32_t reserved2;   /* 0 */
} vr_render_opts;
/* The smallest struct_size accepted: the layout up to and including `reserved`. */
#define VR_RENDER_OPTS_MIN_SIZE 48u

typedef enum {
    VR_OCCUPANCY_AUTO = 0,
    VR_OCCUPANCY_LONE = 1,        /* the lone-frame variant (7 waves/SIMD original, 6 longest axis) */
    VR_OCCUPANCY_IN_FLIGHT = 2    /* the frames-in-flight variant where one exists (a build knob:
                                     since round 6 every walk runs its lone kernel in flight too,
                                     VR_ORIG_WAVES_HI / VR_LONG_WAVES_HI in vr_march.hip) */
} vr_occupancy;

/* Defaults: struct_size = sizeof(vr_render_opts), kernel AUTO, rows [0, UINT32_MAX) --
 * clipped to the frame by the render call -- one band, rank 0 of 1, schedule AUTO,
 * occupancy AUTO, no tile deal. */
int vr_render_opts_init(vr_render_opts* opts);

/* Work order of the tile pass.  A frame's time alone is set by its slowest tiles:
 * dispatched heaviest first (costs recorded by an earlier launch of the same grid
 * size on the device) they no longer start late -- C2 alone 0.151 -> 0.125 ms.
 * With frames in flight on several streams the next frame fills the tail anyway and
 * grid order is faster (C2 0.1124 vs 0.1151 ms per frame).  AUTO picks heaviest
 * first when the device's previous launch was on the same stream (serialised: each
 * launch's time adds up) or has finished, grid order when it is still running on
 * another stream. */
typedef enum {
    VR_SCHEDULE_AUTO = 0,
    VR_SCHEDULE_GRID = 1,
    VR_SCHEDULE_HEAVIEST_FIRST = 2
} vr_schedule;
/* Learned orders (round 5).  Besides the work order, every launch (any schedule) deals the
 * pixels of each 16x16 block to the block's four waves heaviest first (the lane order: a
 * wave's lanes then walk about equally far) -- C2 per frame in flight 0.113 -> 0.101 ms.
 * Both are learned from the walk lengths of earlier launches of the SAME view (scene,
 * algorithm, camera, lights, transform, frame size, rows and band / tile deal) on the device
 * and used only for that view: a view's first launches, and a view that changes on every
 * launch, render with neither.  Neither ever changes a pixel.  A slot that has seen a view
 * defer no walk to the crawl pass skips that view's crawl pass (records carry their launch,
 * so a wrong skip could never shade another frame's pixels).  vr_forget_orders drops what a
 * device has learned, so the next launch renders as a first render (measurement). */
int vr_forget_orders(int device);
/* Test hook: the device's next launch skips its crawl pass as if its slot had seen the view
 * defer nothing.  For the crawl-skip safety net's test only (a launch that then defers a
 * pixel renders it as 0; the tile pass reports the deferral and the slot stops skipping, so
 * later launches are exact again).  Never needed by a renderer. */
int vr_debug_skip_next_crawl(int device);
/* Every vr_render* call returns VR_E_INVALID on a stream that is capturing a HIP graph
 * (its per-device slot ring and work-order bookkeeping are host state that a graph replay
 * would not repeat). */
int vr_render_ex(const vr_scene* s, vr_algo algo, const vr_camera* cam, const vr_lighting* lit,
                 const float translation[3], uint32_t scale, uint32_t width, uint32_t height,
                 const vr_render_opts* opts, uint32_t* out_dev, void* stream);

/* Same render as vr_render, plus the SURVEY.md 8(d) algorithmic byte count of
 * the launch accumulated into *bytes_dev (device uint64, caller-zeroed).
 * Instrumented variant for measurement; pixels are identical. */
int vr_render_count(const vr_scene* s, vr_algo algo, const vr_camera* cam, const vr_lighting* lit,
                    const float translation[3], uint32_t scale, uint32_t width, uint32_t height,
                    uint32_t row_begin, uint32_t row_end, uint32_t* out_dev,
                    uint64_t* bytes_dev, void* stream);

/* writeColorToFramebuffer (Renderer.cuh:1024-1031): packed words -> RGB8
 * (3 bytes per pixel, R = word >> 16 truncated to 8 bits), on the device. */
int vr_pack_rgb8(const uint32_t* words_dev, uint8_t* rgb_dev, uint64_t n_pixels, void* stream);

/* ImageWriter::writeImage(filename, image, width, height, colorChannels)
 * (ImageWriter.cpp:8-16, stbi_write_png with tightly packed rows): 8-bit PNG
 * of 1-4 channels from HOST memory. Row chunks are deflated on parallel
 * threads (level 0-9, out-of-range = 6). Pixels are what stb would store; the
 * compressed bytes differ. */
int vr_png_write(const char* path, const uint8_t* image, uint32_t width, uint32_t height, int channels, int level);

/* Same encoder into memory. out == NULL: sets *out_len to an upper bound of
 * the encoded size (no encoding); otherwise encodes and sets the actual size.
 * threads <= 0: hardware threads, at most 16. */
int vr_png_encode(const uint8_t* image, uint32_t width, uint32_t height, int channels, int level, int threads,
                  uint8_t* out, size_t capacity, size_t* out_len);

/* Synthetic scene: with xyz == NULL only counts (*n_out); otherwise writes up
 * to `capacity` voxels (3 int32 + 1 colour each) and sets *n_out. */
int vr_synth_generate(const vr_synth_params* p, int32_t* xyz, uint32_t* rgb, size_t capacity,
                      size_t* n_out);

/* .vox CSV reader/writer ("x,y,z,color" per line, VoxelFile.cuh:11-35).
 * Reader: two-phase like vr_synth_generate. */
int vr_vox_read(const char* path, int32_t* xyz, uint32_t* rgb, size_t capacity, size_t* n_out);
int vr_vox_write(const char* path, const int32_t* xyz, const uint32_t* rgb, size_t n);

/* .vxb binary scene sidecar: 32-byte header {"VRVXB001",
 * u64 count, u64 reserved[2]}, then int32 xyz[3*count], uint32 rgb[count]
 * (little endian, insertion order).  Same two-call protocol as vr_vox_read. */
int vr_vxb_read(const char* path, int32_t* xyz, uint32_t* rgb, size_t capacity, size_t* n_out);
int vr_vxb_write(const char* path, const int32_t* xyz, const uint32_t* rgb, size_t n);
/* Either format, detected by the .vxb magic. */
int vr_scene_file_read(const char* path, int32_t* xyz, uint32_t* rgb, size_t capacity, size_t* n_out);

const char* vr_last_error(void);
const char* vr_version(void);

#ifdef __cplusplus
}
#endif
#endif /* VR_H */
