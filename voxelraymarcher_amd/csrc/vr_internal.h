// vr_internal.h -- layouts shared by the host builder (vr_host.cpp) and the
// HIP kernels (vr_march.hip).  See DESIGN.md "Data layout in HBM".
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

namespace vr {

// Sets the thread's vr_last_error() message and returns `code` (vr_host.cpp).
int set_error(int code, const std::string& msg);

constexpr uint32_t kEmpty = 1u << 30;        // EMPTY_KEY == EMPTY_VAL (VoxelFunctions.cuh:20-21)
constexpr uint32_t kNone = 0xFFFFFFFFu;      // null region / null cluster in the tables
constexpr int32_t kBlock = 64;               // BLOCK_SIZE (VoxelFunctions.cuh:24)
// Iteration limits ("Walks that never finish").  The walks
// themselves have no budget: the reference runs every finite walk to its end.
//  kTileBudget : a tile-pass pixel whose walks exceed this many loop
//                iterations is handed to the crawl pass and walked there from
//                its start (normal pixels of every config take < 300; only
//                cluster-skip crawls run longer).
//  kCrawlBudget: the crawl pass's hang guard.  Walks that never finish are
//                detected exactly there (a loop iteration that leaves the
//                loop's state unchanged); the longest finite walk of any
//                config takes 1.4e6 iterations, ~770x below this.
constexpr uint32_t kTileBudget = 4096u;
constexpr uint32_t kCrawlBudget = 1u << 30;
// A tile-pass pixel that could not be deferred (the list was full) is written
// as kDeferMarker (no colour is >= 2^24) and counted in slot word 2; the crawl
// pass then finds it in the frame.
constexpr uint32_t kDeferMarker = 0xFFFFFFFFu;
// VCS walks address a region's cluster masks as a 32-bit byte offset from the
// scene's mask array (64 KB per occupied 64^3 region): at most 65536 occupied
// regions (4 GB of masks) per VCS scene; the builders reject larger scenes.  Cuckoo
// scenes have no such bound (as the reference's): their key-presence filter (32 KB per
// occupied region) is addressed with 64-bit offsets.
constexpr uint32_t kVcsMaxRegions = 65536u;
// words of a cuckoo region's key-presence filter (64^3 bits)
constexpr uint32_t kHashFilterWords = 8192u;

// Device view of one immutable scene.  All offsets are 32-bit word indices.
//  region_slot[D^3]          : region index r, or kNone (null StorageStructure*)
//  VCS   : vcs_mask[r*8192 + slot*16 + w]  (one 128-B record per cluster of an
//                              occupied region; VoxelClusterStore::deviceBlockMemAddress
//                              + the cluster's sorted keys, VoxelClusterStore.cuh:37-85)
//                              {bits, index}: bit b set <=> the voxel with in-cluster index
//                              q = 32w+b ((x&7)<<6|(y&7)<<3|z&7, the keys' order) is stored;
//                              index = vcs_vals position of the word's first stored voxel.
//                              Absent cluster: {0, kNone} in all 16 words.  slot =
//                              z-cluster<<6 | y-cluster<<3 | x-cluster (a permutation of the
//                              reference's cluster id x<<6|y<<3|z, so that the word of an
//                              in-region voxel is y2 | x<<1 | (y>>3)<<7 | (z>>3)<<10).
//          vcs_vals[]        : colours, cluster by cluster in key order.
//  Cuckoo: ht_meta[r]        : {base, M, prime, offset}
//          ht_slots[base+i]  : table 1 slot i {key, value};
//          ht_slots[base+M+i]: table 2 slot i {key, value}; empty key = kEmpty
//  VCS   : vcs_cbits[r*16 + w]: bit b set <=> cluster slot 32w+b of region r is present
//                              (derived from vcs_mask after either build; the crawl
//                              pass caches a region's 64 B in LDS)
//  Cuckoo: ht_filter[r*8192 + w]: key-presence bits of region r's tables, one bit per voxel
//                              of the 64^3 region in the VCS mask-word order: voxel (x,y,z)
//                              is word vcs_word_index(x,y,z), bit (y&3)<<3 | z&7 (derived
//                              from ht_slots after either build).  A probe whose key is not
//                              in the tables -- most of them -- is answered here; the
//                              tables are probed for the keys they hold.
struct KScene {
    const uint32_t* region_slot;
    const uint2* vcs_mask;
    const uint32_t* vcs_vals;
    const uint32_t* vcs_cbits;
    const uint4* ht_meta;
    const uint2* ht_slots;
    const uint32_t* ht_filter;
    uint32_t D;
    int32_t min_coord;
    uint32_t n_regions;
};

// Per-launch view: camera, lighting, scene transform and the row mapping.
// Local row l of the output maps to frame row
//   y = row0 + ((l / band_rows) * nranks + rank) * band_rows + (l % band_rows);
// rows with y >= row_limit (<= H) are written as 0.  The output's rows are LW words
// (= W, or the 2-D tile deal's local width).  2-D tile deal (tile_cols > 0; the row
// deal then has nranks = 1, rank = 0): local column x of band b = l / band_rows maps to
// frame column
//   X = ((x / tile_cols) * col_R + (col_rank - col_stride * b) mod col_R) * tile_cols + x % tile_cols;
// columns with X >= W are written as 0.
struct KView {
    float llc[3], hor[3], ver[3], org[3];
    float L[3], LC[3], LP[3];
    // the light direction's reciprocals RN(1 / L_i) (host division, correctly
    // rounded: exact in div_fast) and whether all three are in div_fast's divisor
    // domain -- kernel arguments, so the shadow walks keep them in SGPRs
    float Lr[3];
    uint32_t L_fast;
    // the light as a longest-axis walk sees it (Ray::convertRayToLongestAxisDirection,
    // Ray.cuh:19-71): axis order 0..5 (L,M,S = xyz, xzy, yxz, yzx, zxy, zyx), direction
    // k * L with k = 1 / |L_L| (xyz), its sign classes (bit 2a: > 0, bit 2a+1: < 0),
    // L_unit = that direction is (+-1, +-1, +-1) exactly and the order is zyx (equal
    // magnitudes), L_eq = L's three components are equal
    float Lw[3];
    uint32_t L_order, L_cls, L_unit, L_eq;
    float translation[3];
    float scale_f;
    int32_t use_point_light, use_shadows;
    uint32_t W, H;
    uint32_t row0, band_rows, rank, nranks, local_rows, row_limit;
    uint32_t band_minv;       // floor(2^32 / band_rows) (2^32 - 1 for 1): l / band_rows by a multiply-high
    uint32_t LW;              // output row stride in words (local columns)
    uint32_t tile_cols;       // 0: whole rows (no column deal)
    uint32_t tile_minv;       // floor(2^32 / tile_cols) (2^32 - 1 for 1)
    uint32_t col_R, col_rank, col_stride;   // 2-D deal: ranks, this rank, stride (< col_R)
    // ---- end of the view's identity.  Everything above `out` is hashed, with the scene and
    // the algorithm, into the view key (vr_host.cpp view_key) under which the learned orders
    // and the crawl-pass skip are kept: a field that changes any pixel, or which pixels the
    // tile pass defers to the crawl pass, MUST sit above this line.  Everything below is a
    // per-launch buffer or a launch knob that changes neither (checked by the static_assert
    // after the struct: adding a field below fails the build until it is reviewed here).
    // (The deferral's other inputs are compile-time: kTileBudget, and the walk itself.)
    uint32_t* out;
    unsigned long long* bytes;
    // (COUNT launches, optional) [0] crawl iterations the crawl pass fast-forwarded in
    // closed form, [1] the existence-read bytes credited for them (part of *bytes, never loaded)
    unsigned long long* stats;
    uint32_t* defer;         // crawl deferral slot: [count, done, overflow, 0, records (kDeferRecWords each)...]
    uint32_t defer_cap;
    uint32_t crawl_rewalk;    // 1: deferred crawls are walked from the pixel's start (VR_KERNEL_TILE_REWALK)
    uint32_t crawl_rpw;       // crawl records per wave (0 = 4): 2 for a lone frame, 8 with frames in flight
    uint32_t* defer_stat;     // host-mapped word: the crawl pass writes its record count there (grid sizing)
    // Tile-pass work order ("Heaviest tiles first"): workgroup i of the grid
    // renders tile order[i] = (tile row << 16 | tile column) -- a permutation of the grid
    // made from an earlier launch's costs -- or, when null, tile i in grid order.  cost
    // (or null): each wave writes its walk length (the max over its lanes of the pixel's
    // loop iterations) to cost[tile * kWavesPerTileGroup + wave], tile = row * columns + column.
    const uint32_t* order;
    uint32_t* cost;
    // Lane order (round 5, vr_march.hip lane_pixel): per pixel block (16x16 by default) the slot
    // of each pixel, dealing them to the block's waves heaviest first (or null: 8x8 tiles;
    // vr::perm_bytes(gx, gy) bytes); pcost (or null): each lane
    // writes its pixel's walk lengths at [l * LW + x] (primary << 16 | shadow, each saturated at
    // 0xFFFF; loop iterations), for the next lane order.
    const uint8_t* perm;
    uint32_t* pcost;
    // (or null) the launch slot's host-mapped crawl report: the crawl pass writes
    // {launch_id, records deferred} there in one 8-B store (the host's crawl-pass skip);
    // a tile pass that defers a pixel writes {launch_id, 1} there first (deferral_report:
    // on a launch whose crawl pass the host skipped, the report ends the skipping)
    uint32_t* slot_stat;
    uint32_t launch_id;
};
// The per-launch tail of KView (see "end of the view's identity" above): out, bytes, stats,
// defer, defer_cap, crawl_rewalk, crawl_rpw, defer_stat, order, cost, perm, pcost, slot_stat,
// launch_id.  defer_cap and crawl_rewalk change only how deferred pixels are resumed, never
// which ones defer; the crawl-pass skip keys them anyway (vr_host.cpp crawl_key).
// (10 pointers, 4 words, padding: 104 bytes)
static_assert(sizeof(KView) - offsetof(KView, out) == 104,
              "a KView field was added after `out`: review whether it belongs to the view identity");

// Rays that start a cluster-skip crawl (see vr_march.hip crawl_steps) in the
// tile pass, and pixels that exceed kTileBudget, are deferred to a second pass
// over a per-launch list.
// A slot is [count, done, overflow, 0] and kDeferCap records of kDeferRecWords
// words: the crawling walk's state at the crawl (vr_march.hip, grid_original_rt),
// from which the crawl pass resumes it, or just the pixel (flag 4: walk it from
// its start).  Record words:
//   0 pixel (row << 16 | x)   1 flags (1 shadow walk, 2 longest-axis shadow, 4 walk from the start)
//   2-4 stepped position      5-7 region         8 unused (0)
//   9 iterations so far       10 counted bytes so far
//   11-13 tX, tY, tZ of the last voxel step (hit normal; 0 for shadow walks)
//   14 reserved (0)           15-17 the crawl iteration's voxel (filled in by the crawl pass)
//   18 lit colour             19 unused
// A slot is used by one launch at a time (vr_host.cpp SlotRing).
constexpr uint32_t kDeferCap = 16384;
constexpr uint32_t kDeferRecWords = 20;
constexpr uint32_t kDeferWords = 4 + kDeferCap * kDeferRecWords;

// Launch one render (defined in vr_march.hip): the tile pass and the crawl pass on
// `stream`, the crawl pass with `crawl_wgs` workgroups (any number is correct).
// in_flight: another stream's launch is still running on the device (the tile pass then
// takes its higher-occupancy variant where one exists, vr_march.hip TileWaves)
hipError_t launch_march(int store, int algo, bool count, const KScene& s, const KView& v,
                        hipStream_t stream, uint32_t crawl_wgs, bool in_flight, bool crawl = true);
// Crawl-pass grid for a launch that expects about `records` deferred pixels.
uint32_t crawl_grid(uint32_t records, uint32_t rpw);
// vcs_cbits of a VCS scene from its mask records (one thread per 32 cluster slots).
hipError_t launch_cluster_bits(const uint2* vcs_mask, uint32_t n_regions, uint32_t* cbits, hipStream_t stream);
// ht_filter of a cuckoo scene from its tables (one workgroup per region).
hipError_t launch_hash_filter(const uint4* ht_meta, const uint2* ht_slots, uint32_t n_regions, uint32_t* filter,
                              hipStream_t stream);
hipError_t launch_pack_rgb8(const uint32_t* words, uint8_t* rgb, uint64_t n, hipStream_t stream);
// The 2-D tile deal's layout (vr_render_opts.tile_cols) for rank 0's reassembly: the frame
// W x H, bands of band_rows rows, column blocks of tile_cols, R ranks dealt with `stride`;
// LW = local row width (words), rank_words = one rank's buffer (pixels).
struct TileLayout {
    uint32_t W, H, band_rows, tile_cols, R, stride, LW;
    uint64_t rank_words;
};
// frame[y][x] <- parts[rank][local pixel] for every frame pixel, elem_bytes (1..4) per pixel.
hipError_t launch_assemble_tiles(const void* parts, void* frame, uint32_t elem_bytes, const TileLayout& t,
                                 hipStream_t stream);
// The tile pass's grid for a view (columns, rows of workgroups) and its waves per workgroup.
void march_grid(const KView& v, uint32_t& columns, uint32_t& rows);
constexpr uint32_t kWavesPerTileGroup = 2;
// Heaviest-first work order of a grid of `columns` x `n / columns` workgroups from the
// costs a launch wrote (KView::cost): one workgroup, a counting sort by cost.
hipError_t launch_order(const uint32_t* cost, uint32_t n, uint32_t columns, uint32_t* order, hipStream_t stream);
// The lane orders of a grid of gx x gy tile groups (gx x ceil(gy / 2) 16x16 blocks) from the
// per-pixel walk lengths a launch wrote (KView::pcost, rows x LW words); with cost non-null
// also the waves' walk lengths under the new lane order (KView::cost's layout).
size_t perm_bytes(uint32_t gx, uint32_t gy);   // the lane order of a gx x gy grid
hipError_t launch_perm(const uint32_t* pcost, uint32_t LW, uint32_t rows, uint32_t gx, uint32_t gy, uint8_t* perm,
                       uint32_t* cost, hipStream_t stream);

}  // namespace vr
