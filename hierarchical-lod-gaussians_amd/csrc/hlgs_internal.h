// hlgs_internal.h -- buffer layouts and kernel launchers shared by the translation units of libhlgs.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/hlgs.h"

namespace hlgs {

constexpr int kScanItems = 2048;    // elements per scan block (256 threads x 8)
constexpr int kSortCap = 4096;      // largest per-tile list sorted in one LDS pass
constexpr int kWaveSortCap = 1024;  // longest per-tile list sorted in registers by one wave
constexpr size_t kAlign = 256;

// Gaussians per binning block: 4,096 or 1,024 chosen per launch (raster_fwd.hip bin_gauss), on 1,024 threads
constexpr int kBinMaxTiles = 16384; // tile grids up to this use LDS histograms (2 x 64 KiB)

// The blend backward splits each tile's list into up to kBwdSplits + 1 chunks of bwd_chunk_len(count) entries (a
// multiple of the 64-splat batch, at least kBwdChunk) and runs one wave per (tile, chunk), so a launch holds ~3x
// more, shorter waves than tiles.  A chunk that is not the tile's last starts from the per-pixel state the forward
// sampled at the chunk's end (Img::split_state): the transmittance there, and the colour and inverse depth blended
// behind it (final - sampled), which give the back-to-front recursion's accumulators without replaying the back part.
// Chunks of at least 192 entries (round 3; 128 before): a configs[1] tile (~300 entries) then has one boundary instead
// of two, which halves the split state the forward writes (its write traffic was 137 MB per view, 83 MB of it split
// state) at no measured cost (blend pair 538.6-538.9 against 535.2-536.7 us).
constexpr int kBwdChunk = 192;
constexpr int kBwdSplits = 2;
constexpr int kSplitFloats = 4 * 5 * 64;  // per (tile, split): [quadrant][T, dC r, g, b, dD][lane]
__host__ __device__ inline uint32_t bwd_chunk_len(uint32_t cnt)
{
    const uint32_t even = ((cnt + kBwdSplits) / (kBwdSplits + 1) + 63u) & ~63u;
    return even > (uint32_t)kBwdChunk ? even : (uint32_t)kBwdChunk;
}

inline size_t align_up(size_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }
size_t scan_scratch_elems(size_t n);

// Per-Gaussian state written by the forward preprocess and read by the backward
// (the reference's GeometryState, rasterizer_impl.h:29-45).
struct Geom {
    float* depths;            // P
    uint32_t* clamped;        // P, bit c = colour channel c clamped at 0
    float2* means2D;          // P, pixel-space centre
    float* cov3D;             // P x 6
    uint32_t* tiles_touched;  // P
    uint32_t* point_offsets;  // P, inclusive scan of tiles_touched
    int2* rects;              // P, per-axis 3-sigma extent in pixels
    float4* splat;            // P x 4: the blend kernels' per-Gaussian record (see SplatRec)
    uint32_t* qmask;          // P: footprint quadrant masks of the first rect tiles (rect_quad_masks), written by the
                              // preprocess for the visible Gaussians when pack_entries; read by the key scatter
    int pack;                 // FrameOpts::pack of the frame this buffer is carved for (0 when carved without options)
    int drop;                 // FrameOpts::drop: instances whose quadrant mask is 0 are not binned
    uint32_t polls;           // FrameOpts::polls: bound on each look-back poll of the fused plan
    float* sh_jac;            // P x 9: d colour / d view direction (dRGBdx, dRGBdy, dRGBdz), written by k_preprocess_sh
                              // for the visible Gaussians when sh_jac_written(); the SH backward then reads no SH rows
    uint32_t* scan_tmp;
};

// 64-byte per-Gaussian record read by the blend kernels: one half cache line per (tile, Gaussian)
// instance instead of one line per attribute array.
//   [0] x, y, conic.a, conic.b      [1] conic.c, opacity, r, g
//   [2] b, 1/depth, t, 1/num_kids    [3] unused, first tile x | y << 16, rect width (int bits),
//                                        alpha threshold on e2 (alpha_e2_threshold)
// All written by the preprocess.  The Gaussian's record-slot base (the exclusive scan of the rect sizes) is read by
// the blend backward from point_offsets[idx - 1]: writing it into the record after the scan cost the key scatter a
// partial-line write per visible Gaussian.
// lds_binning(P, gx, gy): the LDS-histogram binning plan applies (raster_fwd.hip)
bool lds_binning(int P, int gx, int gy);

// Tile-list entries (point_list, and the low word of the sort keys) are idx << kEntryShift | quadrant mask whenever
// the Gaussian count leaves the room (P < 2^28): bit q of the mask says the splat's alpha >= 1/255 footprint reaches
// 8x8 quadrant q of the tile (quad_mask), decided once by the key scatter so that the blends read it instead of
// testing the footprint in every quadrant wave.  Otherwise the entry is idx and the blends test it themselves.
// The low bits do not change the sort order: within a tile the (depth, idx) pairs are already distinct.
// pack_entries(P) is decided on the host (capi.hip; hlgs_set_entry_packing turns it off for tests), once per frame
// (FrameOpts), and reaches the kernels as Geom::pack / their flags argument.
constexpr int kEntryShift = 4;
constexpr int kMiscPack = 3;  // Img::misc word holding the frame's FrameOpts::pack
constexpr int kMiscDrop = 4;  // Img::misc word holding the frame's FrameOpts::drop
constexpr int kMiscFail = 5;  // Img::misc word: a block of the fused plan timed out in its look-back (k_tile_offsets_plan)
constexpr int kMiscDone = 6;  // Img::misc word: blocks of the fused plan done with their ranges
constexpr uint32_t kPlanPolls = 1u << 20;  // default bound on each look-back poll of the fused plan (~0.1 s)
// drop_empty(P): with packed entries, an instance whose quadrant mask is 0 (its footprint reaches none of the tile's
// four 8x8 quadrants, so no pixel of the tile blends it) is not binned: the tile lists, the sort and the blends' staging
// skip it.  Its record slot stays (point_offsets and num_rendered are unchanged) and is never written; k_gauss_bwd
// skips the slots whose mask is 0 (their records would be zero).  On by default; hlgs_set_drop_empty(0) bins every
// instance, so point_list and n_contrib are laid out exactly as the reference's binning lays them out.
// k_plan's words for the host (R, longest list, record slots) in the pinned read-back slot: three 64-bit words, each
// carrying the frame's sequence number in its high half, written by single-copy-atomic 64-bit stores, so the host
// waits until all three carry it and the kernel needs no system-scope release (a write-back of the whole L2).
bool pack_entries(int P);
bool drop_empty(int P);
// The frame's binning options, read once from the process-wide test switches (atomics, hlgs_set_entry_packing /
// hlgs_set_drop_empty / hlgs_set_plan_polls) when the frame starts; nothing inside a frame reads the switches again,
// so a thread that flips one while another renders changes only later frames.  The plan kernels write pack and drop
// into Img::misc[kMiscPack], [kMiscDrop] and the host reports them in hlgs_frame_info (entry_shift, drops_empty).
struct FrameOpts {
    int pack = 0, drop = 0;
    uint32_t polls = 0;
    uint32_t flags() const { return (uint32_t)pack | (uint32_t)drop << 1; }  // the plan kernels' flags argument
};
FrameOpts frame_opts(int P);
// Does the forward's preprocess (k_preprocess_sh2) leave Geom::sh_jac for the SH backward?  Same condition as its launch.
inline bool sh_jac_written(const hlgs_raster_args& a)
{
    const int gx = (a.W + 15) / 16, gy = (a.H + 15) / 16;
    return !a.indices && !a.colors_precomp && a.shs && a.M > 0 && a.M <= 16 && lds_binning(a.P, gx, gy);
}
Geom carve_geom(void* base, int P, size_t* total, const FrameOpts& o = FrameOpts());

// Per-pixel / per-tile state (ImageState, rasterizer_impl.h:47-54) plus binning counters.
struct Img {
    float* final_T;        // N
    uint32_t* n_contrib;   // N
    uint2* ranges;         // T: [start, end) into point_list
    uint32_t* tile_count;  // T
    uint32_t* tile_cursor; // T
    uint32_t* misc;        // 16: [0] = binned instances, [1] = longest per-tile list, [2] = record slots (point_offsets[P-1]),
                           // [kMiscPack], [kMiscDrop] = the frame's FrameOpts (the backward reads pack here, not a switch),
                           // [kMiscFail], [kMiscDone]: the fused plan's failure and completion words
    uint32_t* scan_tmp;
    float* split_state;    // T x kBwdSplits x kSplitFloats (see bwd_chunk_len)
};
Img carve_img(void* base, int W, int H, size_t* total);

// Per-instance state (BinningState).  keys = depth_bits << 32 | gaussian index, grouped by tile.
struct Bin {
    uint64_t* keys;
    uint64_t* keys2;
    uint32_t* point_list;  // R, tile-major then front-to-back
};
Bin carve_bin(void* base, int R, size_t* total);

// Backward scratch: one 48-byte gradient record per (tile, Gaussian) instance, stored Gaussian-major at the
// Gaussian's point_offsets slot so the per-Gaussian reduction reads contiguous rows; one slot is three float4s
// (one contiguous write per instance instead of three partial lines in three arrays):
//   rec[3 s]     dmean2D.x, dmean2D.y, dconic.x, dconic.y
//   rec[3 s + 1] dconic.w, dopacity, dcolor.r, dcolor.g
//   rec[3 s + 2] dcolor.b, dinvdepth, -, -
struct BwdScratch {
    float4* rec;
    float* parent_dmean;  // P x 3 (hierarchy mode only)
};
BwdScratch carve_bwd(void* base, int P, int R, size_t* total);

// Buffers the preprocess clears on its way (instead of separate memsets before it): the per-tile counts the
// binning adds into and the caller's `seen` flags.  Null members are skipped.
struct ZeroJob {
    uint32_t* tile_count;
    int T;
    int* seen;
    int P;
};
__device__ __forceinline__ void zero_prelude(const ZeroJob& z, int tid, int nthreads)
{
    if (z.seen)
        for (int i = tid; i < z.P; i += nthreads) z.seen[i] = 0;
    if (z.tile_count)
        for (int i = tid; i < z.T; i += nthreads) z.tile_count[i] = 0;
}

// Speculative render (hlgs_rasterize_forward): the render kernels are queued before the host has read
// R and the longest tile list; each exits at once when they exceed what the launch was sized for.
struct Guard {
    const uint32_t* misc;  // Img::misc (R, longest list) or nullptr = no check
    uint32_t cap_R, cap_n;
};
__device__ __forceinline__ bool guard_fail(const Guard& gd)
{
    return gd.misc && (gd.misc[0] > gd.cap_R || gd.misc[1] > gd.cap_n);
}

// Upper-tree cut (stream.hip).  Per level the frontier (the reference's `stack`) is filtered by the cull;
// leaves go to the cut, then the non-leaves whose LOD condition is false, each group in frontier order; the
// next frontier is the first children of the expanded nodes in order, then their first children's next
// siblings in order (scene/gaussian_model.py:364-404).
constexpr int kCutLevelLaunches = 8;  // wide-level launches queued after the narrow walk (stream.hip)
constexpr int kCutMaxBlocks = 64;      // workgroups of one wide level (all resident at once)
struct CutState {          // the walk's state between k_upper_cut and the k_cut_level launches
    int size, total, parity, overflow;
};
struct CutFlat {           // the flat cut's placement state between k_cut_flat_place and k_cut_flat_write
    uint64_t leaf[1024], stop[1024];            // per thread run: the alive leaves / condition-false nodes
    int2 off[1024];                             // per run: leaves and condition-false nodes before it
    int2 lev[HLGS_CUT_FLAT_MAX_LEVELS + 1];     // per level: (leaves, condition-false nodes) before its first entry
};
struct CutArgs {
    int N;
    const int* nodes;      // N x 6 HierarchyNode rows: 2 child_count, 3 first_child, 4 next_sibling
    const float* xyz;
    const float* bounds;
    const float* min_dist2;
    const float* planes;   // nviews x 4 x (nx, ny, nz, d), normalised as extract_frustum_planes does
    const float* campos;   // nviews x 3
    float dmul;
    int use_frustum, use_lod;
    int nviews;            // >= 1: the cut serves the union of the views (visible in any frustum, LOD of the nearest)
    int* front_a;
    int* front_b;
    int capacity;          // entries of cut
    int* cut;
    int* count;            // [0] = cut size, [1] = overflow flag
    CutState* state;
    unsigned* arrive;      // kCutLevelLaunches arrival counters
    int* level_counts;     // 3 x kCutMaxBlocks
    CutFlat* flat;
};
size_t upper_cut_state_bytes();

// SPT cache bookkeeping of one streaming step (stream.hip, train_post.py:346-430)
struct CacheArgs {
    int n_cut;                // the cut's length, or its capacity when n_cut_dev is set
    const int* n_cut_dev;     // [count, overflow] of the device-side upper cut, or NULL
    const int* cut;           // coarse cut of the upper tree
    const int* nodes;         // upper-tree HierarchyNode rows
    const float* xyz;
    const float* campos;      // nviews x 3: an SPT's distance is that of the nearest camera
    int nviews;
    float dmul;
    int num_spts;
    int m;                    // previous step's SPTs
    const int* prev_idx;
    const float* prev_dist;
    const int* prev_counts;
    int R;                    // len(render_indices)
    int tail_end;             // len(render_indices) - len(load_from_disk_indices)
    float rtol, atol;
    // scratch
    int* flag;                // num_spts, zero on entry
    int* spt_idx;             // n_cut
    float* spt_dist;          // n_cut
    int* diff;                // R + 1, zero on entry
    int* sizes;               // device: n_kept, n_load, n_upper, prefix
    // outputs
    int* keep_idx;
    float* keep_dist;
    int* keep_counts;
    int* load_idx;
    float* load_dist;
    int* upper;
};
void launch_cache_lists(const CacheArgs& a, hipStream_t s);
void launch_cache_keep(int R, int sky, const uint32_t* diff_incl, uint32_t* keep, hipStream_t s);
void launch_cache_split(int R, const int* render, const uint32_t* keep_incl, int* keep_rows, int* render_kept,
                        int* wb_rows, int* wb_indices, hipStream_t s);
struct RowCopy {
    const void* src;
    void* dst;
    int64_t row_bytes;
    int device_only;          // both sides in device memory: 16-byte accesses at 4-byte alignment are used
};
constexpr int kMaxRowTables = 32;
void launch_rows_multi(int T, const RowCopy* tabs, int64_t n, const int* src_rows, const int* dst_rows,
                       hipStream_t s);
constexpr int kPackSlots = 4;  // packed host rows of up to 4 x 64 words (1 KiB)
void launch_rows_packed(int T, float* const* tabs, const int* words, int64_t n, const int* dev_rows,
                        const int* host_rows, float* host, int hw, bool to_host, hipStream_t s,
                        const float* const* resident = nullptr, const int* resident_of = nullptr);
// optim.hip: one dense Adam step over up to kMaxRowTables tensors (OurAdam._single_tensor_adam2)
struct AdamTensor {
    float* param;
    float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    int64_t numel;
    int64_t row_elems;        // elements per Gaussian row (skybox rows have their gradient zeroed)
    float neg_step_size;      // -lr / (1 - beta1^step)
};
void launch_adam_multi(int T, const AdamTensor* t, int sky, float b1, float a1, float b2, float a2, float bc2_sqrt,
                       float eps, hipStream_t s);

// scan.hip
void scan_inclusive_u32(const uint32_t* in, uint32_t* out, size_t n, uint32_t* tmp, hipStream_t s);

// stage timing (capi.cpp)
void stage_mark(hipStream_t s, int stage, bool begin);

}  // namespace hlgs
