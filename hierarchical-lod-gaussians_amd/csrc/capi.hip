// capi.hip -- the C ABI of libhlgs.so (declared in include/hlgs.h) and the host orchestration of the
// rasterizer stages.  Mirrors CudaRasterizer::Rasterizer::forward/backward
// (submodules/hierarchy-rasterizer/cuda_rasterizer/rasterizer_impl.cu:203-517) and the LOD entry
// points of gaussianhierarchy/runtime_switching.cu, re-planned for gfx950.
//
// Re-entrancy: no device memory is allocated here and no scratch is static; every buffer is passed
// in.  The only process-wide state is the opt-in stage-timing instrumentation used by bench.py.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "hlgs_internal.h"

namespace hlgs {
// The process-wide test switches, read once per frame (frame_opts) and never inside one.
static std::atomic<int> g_entry_packing{1};       // hlgs_set_entry_packing
static std::atomic<int> g_drop_empty{1};          // hlgs_set_drop_empty
static std::atomic<uint32_t> g_plan_polls{kPlanPolls};  // hlgs_set_plan_polls
bool pack_entries(int P) { return g_entry_packing.load(std::memory_order_relaxed) && P < (1 << (32 - kEntryShift)); }
bool drop_empty(int P) { return g_drop_empty.load(std::memory_order_relaxed) && pack_entries(P); }
FrameOpts frame_opts(int P)
{
    FrameOpts o;
    o.pack = pack_entries(P) ? 1 : 0;
    o.drop = o.pack && g_drop_empty.load(std::memory_order_relaxed) ? 1 : 0;
    o.polls = g_plan_polls.load(std::memory_order_relaxed);
    return o;
}
void launch_preprocess(const hlgs_raster_args& a, const Geom& g, int* radii, uint32_t* tile_count, int gx, int gy,
                       const ZeroJob& z,
                       hipStream_t s);
void launch_tile_ranges(const Img& im, int T, const uint32_t* point_offsets, int P, uint32_t flags, hipStream_t s);
void launch_plan(int P, const Geom& g, const Img& im, int gx, int gy, uint32_t* host, uint32_t seq, hipStream_t s,
                 bool fused);
bool lds_binning(int P, int gx, int gy);
uint32_t* bin_histogram(const Img& im, int P, int gx, int gy);
void launch_count_tiles(int P, const int* radii, const Geom& g, const Img& im, int gx, int gy, bool alt,
                        hipStream_t s, uint32_t* hist, bool fused);
void launch_binning(const hlgs_raster_args& a, const int* radii, const Geom& g, const Img& im, const Bin& b, int gx,
                    int gy, uint32_t max_count, hipStream_t s, bool timing, Guard gd);
void launch_blend_fwd(const hlgs_raster_args& a, const Geom& g, const Img& im, const Bin& b, int gx, int gy,
                      float* out_color, float* out_invdepth, int* seen, hipStream_t s, Guard gd);
void launch_blend_bwd(const hlgs_raster_args& a, const Geom& g, const Img& im, const Bin& b, const BwdScratch& rs,
                      int gx, int gy, const float* dL_dpix, const float* dL_dinv, hipStream_t s);
void launch_gauss_bwd(const hlgs_raster_args& a, const int* radii, const Geom& g, const BwdScratch& rs,
                      const hlgs_grads& o, bool has_depth, hipStream_t s, hipStream_t late, hipEvent_t ev,
                      const uint32_t* misc);
void launch_mark_visible(int P, const float* means, const float* view, uint8_t* present, hipStream_t s);
void launch_sh_from_colour(int P, int V, int D, int M, bool alt, const float* means, const float* campos,
                           const float* drgb, int64_t stride, float scale, float* dsh, float* ddc, hipStream_t s);
void launch_relocation(int P, const float* oo, const float* so, const int* N, const float* binoms, int n_max,
                       float* on, float* sn, hipStream_t s);
size_t ssim_partials(int C, int H, int W);
void launch_ssim_forward(int C, int H, int W, const float* img1, const float* img2, int valid, float* abc,
                         float* partial, float* out, hipStream_t s, bool clamp1);
void launch_ssim_backward(int C, int H, int W, const float* img1, const float* img2, const float* abc,
                          const float* coef, float* grad1, hipStream_t s, bool clamp1);
int depth_l1_blocks(long n);
void launch_depth_l1_forward(long n, const float* inv, const float* mono, const float* mask, float* partial,
                             float* out, hipStream_t s);
void launch_depth_l1_backward(long n, const float* inv, const float* mono, const float* mask, const float* coef,
                              float* grad, hipStream_t s);
void launch_upper_cut(const CutArgs& a, hipStream_t s);
void launch_upper_cut_flat(const CutArgs& a, const int* order, hipStream_t s);
void launch_rows(bool gather, long n, int row_bytes, const int64_t* idx, const void* src, void* dst, hipStream_t s);
void launch_act_fwd(int64_t n, const float* op_raw, const float* sc_raw, const float* rot_raw, float* op, float* sc,
                    float* rot, hipStream_t s);
void launch_act_bwd(int64_t n, const float* op, const float* sc, const float* rot_raw, const float* g_op,
                    const float* g_sc, const float* g_rot, float* d_op, float* d_sc, float* d_rot, hipStream_t s);
void launch_morton(int P, const float* xyz, const float* mn, const float* mx, int64_t* codes, hipStream_t s);
void launch_adam(float* param, const float* grad, float* m, float* v, const uint8_t* vis, float lr, float b1, float b2,
                 float eps, uint32_t N, uint32_t M, hipStream_t s);
void launch_expand_dynamic(int N, float target, const int* nodes, const float* pos, const float* scales,
                           const float* vp, const float* vd, int* ri, int* pi, int* ni, uint32_t* counts,
                           uint32_t* incl, uint32_t* tmp, hipStream_t s);
void launch_weights_dynamic(int n, const int* idx, float target, const int* nodes, const float* pos,
                            const float* scales, const float* vp, float* ts, int* kids, hipStream_t s);
void launch_expand_static(int N, float target, const int* nodes, const float* boxes, const float* vp, int* ri,
                          int* pi, int* ni, uint32_t* counts, uint32_t* incl, uint32_t* tmp, hipStream_t s);
void launch_weights_static(int n, const int* idx, float target, const int* nodes, const float* boxes,
                           const float* vp, float* ts, int* kids, hipStream_t s);
void launch_spt_prepare(int s_, const int* starts, const float* smax, const int* sidx, const float* sdist,
                        uint32_t* sizes, uint32_t* incl, uint32_t* tmp, hipStream_t s);
void launch_spt_finish(int s_, int E, int n, const int* gidx, const int* starts, const float* smin, const int* sidx,
                       const float* sdist, int compat, const uint32_t* sizes, const uint32_t* incl, uint32_t* counts,
                       uint32_t* counts_incl, uint32_t* tmp_s, int* result, uint32_t* keep, uint32_t* keep_incl,
                       uint32_t* tmp_n, int* cut, int* counts_prefix, hipStream_t s);
void launch_lod_interp_fwd(int S, int n, int M3, const int* ridx, const int* pidx, const float* w, const float* means,
                           const float* scales, const float* rots, const float* opac, const float* shs, float* om,
                           float* osc, float* orot, float* oop, float* osh, hipStream_t s);
size_t lerp_bwd_scratch_elems(int P, int n);
void launch_lod_interp_bwd(int P, int S, int n, int M3, const int* ridx, const int* pidx, const float* w,
                           const float* rots, const float* gm, const float* gsc, const float* grot, const float* gop,
                           const float* gsh, float* dm, float* dsc, float* drot, float* dop, float* dsh, void* scratch,
                           hipStream_t s);

// ---------------------------------------------------------------- buffer carving
template <typename T>
static T* take(char*& p, size_t count)
{
    T* r = reinterpret_cast<T*>(p);
    p += align_up(count * sizeof(T));
    return r;
}

Geom carve_geom(void* base, int P, size_t* total, const FrameOpts& o)
{
    char* p = static_cast<char*>(base);
    Geom g;
    g.depths = take<float>(p, P);
    g.clamped = take<uint32_t>(p, P);
    g.means2D = take<float2>(p, P);
    g.cov3D = take<float>(p, 6 * (size_t)P);
    g.tiles_touched = take<uint32_t>(p, P);
    g.point_offsets = take<uint32_t>(p, P);
    g.rects = take<int2>(p, P);
    g.splat = take<float4>(p, 4 * (size_t)P);
    g.sh_jac = take<float>(p, 9 * (size_t)P);
    g.qmask = take<uint32_t>(p, (size_t)P);
    g.pack = o.pack;
    g.drop = o.drop;
    g.polls = o.polls;
    g.scan_tmp = take<uint32_t>(p, scan_scratch_elems(P));
    if (total) *total = (size_t)(p - static_cast<char*>(base));
    return g;
}

Img carve_img(void* base, int W, int H, size_t* total)
{
    const size_t N = (size_t)W * H;
    const int T = ((W + 15) / 16) * ((H + 15) / 16);
    char* p = static_cast<char*>(base);
    Img im;
    im.final_T = take<float>(p, N);
    im.n_contrib = take<uint32_t>(p, N);
    im.ranges = take<uint2>(p, T);
    im.tile_count = take<uint32_t>(p, T);
    im.tile_cursor = take<uint32_t>(p, T);
    im.misc = take<uint32_t>(p, 16);
    im.scan_tmp = take<uint32_t>(p, scan_scratch_elems(T));
    im.split_state = take<float>(p, (size_t)T * kBwdSplits * kSplitFloats);
    if (total) *total = (size_t)(p - static_cast<char*>(base));
    return im;
}

Bin carve_bin(void* base, int R, size_t* total)
{
    char* p = static_cast<char*>(base);
    Bin b;
    b.point_list = take<uint32_t>(p, R);  // first: its offset does not depend on R
    b.keys = take<uint64_t>(p, R);
    b.keys2 = take<uint64_t>(p, R);
    if (total) *total = (size_t)(p - static_cast<char*>(base));
    return b;
}

BwdScratch carve_bwd(void* base, int P, int R, size_t* total)
{
    char* p = static_cast<char*>(base);
    BwdScratch r;
    r.rec = take<float4>(p, 3 * (size_t)R);
    r.parent_dmean = take<float>(p, 3 * (size_t)P);
    if (total) *total = (size_t)(p - static_cast<char*>(base));
    return r;
}

// ---------------------------------------------------------------- errors & timing
static thread_local std::string g_err;

static int fail(int code, const std::string& msg)
{
    g_err = msg;
    return code;
}

int fail_msg(int code, const std::string& msg) { return fail(code, msg); }  // hier_io.cpp

#define HLGS_TRY_HIP(expr)                                                                            \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess) return fail(HLGS_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// After a group of launches: always surface launch errors; under `debug` also synchronise, as the
// reference's CHECK_CUDA does (auxiliary.h:23-30).
static int check_stage(hipStream_t s, bool debug, const char* stage)
{
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && debug) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return fail(HLGS_ERR_DEVICE, std::string("[HIP ERROR] in ") + stage + ": " + hipGetErrorString(e));
    return HLGS_OK;
}

enum Stage { ST_PRE = 0, ST_SCAN, ST_RANGES, ST_SCATTER, ST_SORT, ST_BLEND_FWD, ST_BLEND_BWD, ST_GAUSS_BWD,
             ST_COUNT_TILES, ST_COUNT };
static const char* kStageNames[ST_COUNT] = {"preprocess", "scan", "tile_ranges", "scatter", "tile_sort",
                                            "blend_fwd", "blend_bwd", "gauss_bwd", "count_tiles"};
static uint32_t g_timing_mask = 0;  // bit i: time stage i
static bool g_timing = false;
// event pool per stage: launch i of a stage uses pair i (grown on demand, reused after a reset)
static std::vector<hipEvent_t> g_ev[ST_COUNT][2];
static int g_calls[ST_COUNT];

void stage_mark(hipStream_t s, int stage, bool begin)
{
    if (!((g_timing_mask >> stage) & 1u)) return;
    const size_t i = (size_t)g_calls[stage];
    auto& pool = g_ev[stage][begin ? 0 : 1];
    if (pool.size() <= i) {
        hipEvent_t e;
        hipEventCreate(&e);
        pool.push_back(e);
    }
    hipEventRecord(pool[i], s);
    if (!begin) g_calls[stage]++;
}

static int validate(const hlgs_raster_args* a)
{
    if (!a) return fail(HLGS_ERR_ARG, "null args");
    if (a->P < 0 || a->W <= 0 || a->H <= 0) return fail(HLGS_ERR_ARG, "invalid P/W/H");
    if (a->variant != HLGS_VARIANT_HIERARCHY && a->variant != HLGS_VARIANT_ALT)
        return fail(HLGS_ERR_ARG, "unknown rasterizer variant");
    if (a->P == 0) return HLGS_OK;
    if (!a->means3D || !a->opacities || !a->viewmatrix || !a->projmatrix || !a->bg || !a->campos)
        return fail(HLGS_ERR_ARG, "missing required tensor (means3D/opacities/viewmatrix/projmatrix/bg/campos)");
    if (a->variant == HLGS_VARIANT_ALT) {
        // alt-rasterizer: SH as dc (degree 0) + shs (the M higher-order coefficients)
        if (!a->dc && !a->colors_precomp) return fail(HLGS_ERR_ARG, "For non-RGB, provide precomputed Gaussian colors!");
        if (a->indices || a->parent_indices || a->ts || a->kids)
            return fail(HLGS_ERR_ARG, "the alt rasterizer has no hierarchy mode");
        if (a->shs && (a->M <= 0 || a->M > 15)) return fail(HLGS_ERR_ARG, "shs rows must hold 1..15 coefficients");
        if (!a->colors_precomp && (a->D < 0 || a->D > 3 || (a->D + 1) * (a->D + 1) - 1 > (a->shs ? a->M : 0)))
            return fail(HLGS_ERR_ARG, "sh_degree needs more SH coefficients than given");
        if (!a->cov3D_precomp && (!a->scales || !a->rotations))
            return fail(HLGS_ERR_ARG, "provide scales+rotations or cov3D_precomp");
        if (a->P != a->P_full) return fail(HLGS_ERR_ARG, "P must equal P_full");
        return HLGS_OK;
    }
    if (!a->shs && !a->colors_precomp)
        return fail(HLGS_ERR_ARG, "For non-RGB, provide precomputed Gaussian colors!");
    if (a->shs && (a->M <= 0 || a->M > 16)) return fail(HLGS_ERR_ARG, "shs rows must hold 1..16 coefficients");
    if (!a->cov3D_precomp && (!a->scales || !a->rotations))
        return fail(HLGS_ERR_ARG, "provide scales+rotations or cov3D_precomp");
    if (a->D < 0 || a->D > 3) return fail(HLGS_ERR_ARG, "sh_degree must be in [0,3]");
    if (a->shs && (a->D + 1) * (a->D + 1) > a->M) return fail(HLGS_ERR_ARG, "sh_degree needs more SH coefficients than given");
    const bool h0 = a->indices != nullptr, h1 = a->parent_indices != nullptr;
    if (h0 != h1) return fail(HLGS_ERR_ARG, "render_indices and parent_indices must be given together");
    if ((a->ts != nullptr) != (a->kids != nullptr))
        return fail(HLGS_ERR_ARG, "interpolation_weights and num_node_kids must be given together");
    if (h1 && !a->ts) return fail(HLGS_ERR_ARG, "parent_indices requires interpolation_weights");
    if (!h0 && a->P != a->P_full) return fail(HLGS_ERR_ARG, "P must equal P_full without render_indices");
    return HLGS_OK;
}

}  // namespace hlgs

using namespace hlgs;

extern "C" {

const char* hlgs_last_error(void) { return g_err.c_str(); }
const char* hlgs_version(void) { return "hlgs 0.1 gfx950"; }

size_t hlgs_geom_buffer_size(int P)
{
    size_t t = 0;
    carve_geom(nullptr, P < 0 ? 0 : P, &t);
    return t + kAlign;
}
size_t hlgs_image_buffer_size(int W, int H)
{
    size_t t = 0;
    carve_img(nullptr, W, H, &t);
    return t + kAlign;
}
size_t hlgs_binning_buffer_size(int R)
{
    size_t t = 0;
    carve_bin(nullptr, R < 0 ? 0 : R, &t);
    return t + kAlign;
}
size_t hlgs_backward_scratch_size(int P, int R)
{
    size_t t = 0;
    carve_bwd(nullptr, P, R < 0 ? 0 : R, &t);
    return t + kAlign;
}

static void* aligned(const void* p) { return (void*)align_up((size_t)p); }

void hlgs_set_entry_packing(int on) { g_entry_packing.store(on ? 1 : 0, std::memory_order_relaxed); }
void hlgs_set_drop_empty(int on) { g_drop_empty.store(on ? 1 : 0, std::memory_order_relaxed); }
void hlgs_set_plan_polls(unsigned polls) { g_plan_polls.store(polls, std::memory_order_relaxed); }
int hlgs_point_list_entry_shift(int P) { return pack_entries(P) ? kEntryShift : 0; }
int hlgs_point_list_drops_empty(int P) { return drop_empty(P) ? 1 : 0; }

size_t hlgs_binning_point_list_offset(int R)
{
    Bin b = carve_bin(nullptr, R < 0 ? 0 : R, nullptr);
    return (size_t)b.point_list;
}
size_t hlgs_image_misc_offset(int W, int H)
{
    Img im = carve_img(nullptr, W, H, nullptr);
    return (size_t)im.misc;
}
size_t hlgs_geom_splat_offset(int P)
{
    Geom g = carve_geom(nullptr, P < 0 ? 0 : P, nullptr);
    return (size_t)g.splat;
}
size_t hlgs_image_ranges_offset(int W, int H)
{
    Img im = carve_img(nullptr, W, H, nullptr);
    return (size_t)im.ranges;
}

namespace hlgs {
static bool pack_entries_fit(int P) { return P < (1 << (32 - kEntryShift)); }
static void set_frame_flags(hlgs_frame_info* info, const FrameOpts& o)
{
    info->entry_shift = o.pack ? kEntryShift : 0;
    info->drops_empty = o.drop;
}
// Phase 1: preprocess, tile counts, scans, tile ranges (misc = R, longest list, record slots).  With LDS-histogram
// binning the preprocess also clears tile_count and `seen`, and one k_plan block does both scans and the ranges and
// mirrors misc into `host` (pinned, may be null); otherwise the generic path runs device-wide scans.
static int prepare_launch(const hlgs_raster_args* a, const FrameOpts& o, void* geom, void* img, int* radii, int* seen,
                          uint32_t* host, uint32_t seq, hipStream_t s, bool fused = true)
{
    const int gx = (a->W + 15) / 16, gy = (a->H + 15) / 16, T = gx * gy;
    Geom g = carve_geom(aligned(geom), a->P, nullptr, o);
    Img im = carve_img(aligned(img), a->W, a->H, nullptr);
    hipGetLastError();
    const bool lds_bins = lds_binning(a->P, gx, gy);
    const bool alt = a->variant == HLGS_VARIANT_ALT;
    int rc;
    if (lds_bins) {
        stage_mark(s, ST_PRE, true);
        launch_preprocess(*a, g, radii, nullptr, gx, gy, ZeroJob{im.tile_count, T, seen, a->P}, s);
        stage_mark(s, ST_PRE, false);
        stage_mark(s, ST_COUNT_TILES, true);
        launch_count_tiles(a->P, radii, g, im, gx, gy, alt, s, bin_histogram(im, a->P, gx, gy), fused);
        stage_mark(s, ST_COUNT_TILES, false);
        if ((rc = check_stage(s, a->debug, "preprocess"))) return rc;
        stage_mark(s, ST_SCAN, true);
        launch_plan(a->P, g, im, gx, gy, host, seq, s, fused);
        stage_mark(s, ST_SCAN, false);
        return check_stage(s, a->debug, "scan");
    }
    if (seen) HLGS_TRY_HIP(hipMemsetAsync(seen, 0, sizeof(int) * (size_t)a->P, s));
    HLGS_TRY_HIP(hipMemsetAsync(im.tile_count, 0, sizeof(uint32_t) * T, s));
    HLGS_TRY_HIP(hipMemsetAsync(im.misc, 0, sizeof(uint32_t) * 16, s));
    stage_mark(s, ST_PRE, true);
    launch_preprocess(*a, g, radii, im.tile_count, gx, gy, ZeroJob{nullptr, 0, nullptr, 0}, s);
    stage_mark(s, ST_PRE, false);
    if ((rc = check_stage(s, a->debug, "preprocess"))) return rc;
    stage_mark(s, ST_SCAN, true);
    scan_inclusive_u32(g.tiles_touched, g.point_offsets, (size_t)a->P, g.scan_tmp, s);
    stage_mark(s, ST_SCAN, false);
    stage_mark(s, ST_RANGES, true);
    scan_inclusive_u32(im.tile_count, im.tile_cursor, (size_t)T, im.scan_tmp, s);
    launch_tile_ranges(im, T, g.point_offsets, a->P, o.flags(), s);
    stage_mark(s, ST_RANGES, false);
    if ((rc = check_stage(s, a->debug, "scan"))) return rc;
    if (host) HLGS_TRY_HIP(hipMemcpyAsync(host, im.misc, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    return HLGS_OK;
}

// The binning plan again with the two launches that need no inter-block wait (k_tile_offsets + k_plan), for a frame
// whose fused plan reported a timed-out look-back (k_tile_offsets_plan: R = ~0u).  The preprocess outputs are intact;
// the count kernel rewrites the histogram rows the failed plan had partly turned into offsets.
static int replan_launch(const hlgs_raster_args* a, const FrameOpts& o, void* geom, void* img, const int* radii,
                         uint32_t* host, uint32_t seq, hipStream_t s)
{
    const int gx = (a->W + 15) / 16, gy = (a->H + 15) / 16;
    Geom g = carve_geom(aligned(geom), a->P, nullptr, o);
    Img im = carve_img(aligned(img), a->W, a->H, nullptr);
    hipGetLastError();
    launch_count_tiles(a->P, radii, g, im, gx, gy, a->variant == HLGS_VARIANT_ALT, s, bin_histogram(im, a->P, gx, gy),
                       false);
    launch_plan(a->P, g, im, gx, gy, host, seq, s, false);
    return check_stage(s, a->debug, "re-plan");
}

static int render_launch(const hlgs_raster_args* a, const FrameOpts& o, const int* radii, void* geom, void* img,
                         void* binning, int R_carve, uint32_t max_count, float* out_color, float* out_invdepth, int* seen,
                         hipStream_t s, Guard gd)
{
    const int gx = (a->W + 15) / 16, gy = (a->H + 15) / 16;
    Geom g = carve_geom(aligned(geom), a->P, nullptr, o);
    Img im = carve_img(aligned(img), a->W, a->H, nullptr);
    Bin b = carve_bin(aligned(binning), R_carve, nullptr);
    hipGetLastError();
    launch_binning(*a, radii, g, im, b, gx, gy, max_count, s, g_timing, gd);
    int rc;
    if ((rc = check_stage(s, a->debug, "binning"))) return rc;
    stage_mark(s, ST_BLEND_FWD, true);
    launch_blend_fwd(*a, g, im, b, gx, gy, out_color, out_invdepth, seen, s, gd);
    stage_mark(s, ST_BLEND_FWD, false);
    return check_stage(s, a->debug, "blend_fwd");
}

// Largest R whose binning layout fits in `bytes`.
static int binning_capacity(size_t bytes)
{
    if (bytes <= 4 * kAlign) return 0;
    long r = (long)((bytes - 4 * kAlign) / 20);
    while (r > 0 && hlgs_binning_buffer_size((int)r) > bytes) r--;
    return (int)std::min<long>(r, 0x7fffffff);
}

// Pinned read-back slot and event for the speculative forward, per thread and device.
struct Readback {
    uint32_t* host = nullptr;  // three 64-bit words: the frame's sequence number | R, longest list, record slots (k_plan)
    hipEvent_t ev = nullptr;
    uint32_t last_maxc = 0;  // longest tile list of the previous frame (plans the speculative sort)
    uint32_t seq = 0;
};
// Wait until k_plan has mirrored the frame's words (host[3] == seq), polling the coherent pinned words rather than
// synchronising on an event recorded after k_plan: an event is a queue barrier, ~6 us of idle GPU before the binning.
// A stream that drains or fails without the words reports an error instead of spinning forever.
// words[i] = the three tagged 64-bit words' low halves once all of them carry seq (plan_host_words, raster_fwd.hip).
static bool plan_words_ready(const uint32_t* host, uint32_t seq, uint32_t* words)
{
    const uint64_t* h = reinterpret_cast<const uint64_t*>(host);
    for (int i = 0; i < 3; i++) {
        const uint64_t v = __atomic_load_n(&h[i], __ATOMIC_ACQUIRE);
        if ((uint32_t)(v >> 32) != seq) return false;
        words[i] = (uint32_t)v;
    }
    return true;
}
static int wait_plan_words(const uint32_t* host, uint32_t seq, hipStream_t s, uint32_t* words)
{
    for (uint32_t n = 1;; n++) {
        if (plan_words_ready(host, seq, words)) return HLGS_OK;
        if ((n & 1023u) == 0u && hipStreamQuery(s) != hipErrorNotReady) {
            if (plan_words_ready(host, seq, words)) return HLGS_OK;
            return fail(HLGS_ERR_DEVICE, "the binning plan did not report its sizes");
        }
        __builtin_ia32_pause();
    }
}
static int readback_for(hipStream_t s, Readback** out)
{
    static thread_local Readback rb[64];
    int dev = 0;
    HLGS_TRY_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return fail(HLGS_ERR_DEVICE, "device index out of range");
    Readback& r = rb[dev];
    if (!r.host) HLGS_TRY_HIP(hipHostMalloc((void**)&r.host, 16 * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent));
    if (!r.ev) HLGS_TRY_HIP(hipEventCreateWithFlags(&r.ev, hipEventDisableTiming));
    (void)s;
    *out = &r;
    return HLGS_OK;
}
}  // namespace hlgs

int hlgs_rasterize_forward_prepare(const hlgs_raster_args* a, void* geom, void* img, int* radii,
                                   hlgs_frame_info* info, void* stream)
{
    int rc = validate(a);
    if (rc) return rc;
    info->num_rendered = 0;
    info->max_tile_count = 0;
    info->rendered = 0;
    info->num_binned = 0;
    const FrameOpts o = frame_opts(a->P);  // the frame's options, handed to _render through *info
    set_frame_flags(info, o);
    if (a->P == 0) return HLGS_OK;
    hipStream_t s = (hipStream_t)stream;
    if ((rc = prepare_launch(a, o, geom, img, radii, nullptr, nullptr, 0u, s))) return rc;
    Img im = carve_img(aligned(img), a->W, a->H, nullptr);
    uint32_t misc[3];
    HLGS_TRY_HIP(hipMemcpyAsync(misc, im.misc, sizeof(misc), hipMemcpyDeviceToHost, s));
    HLGS_TRY_HIP(hipStreamSynchronize(s));
    if (misc[0] == ~0u) {  // the fused plan's look-back timed out: plan again without inter-block waits
        if ((rc = replan_launch(a, o, geom, img, radii, nullptr, 0u, s))) return rc;
        HLGS_TRY_HIP(hipMemcpyAsync(misc, im.misc, sizeof(misc), hipMemcpyDeviceToHost, s));
        HLGS_TRY_HIP(hipStreamSynchronize(s));
        if (misc[0] == ~0u) return fail(HLGS_ERR_DEVICE, "the binning plan failed twice");
    }
    info->num_binned = (int)misc[0];
    info->max_tile_count = (int)misc[1];
    info->num_rendered = (int)misc[2];
    return HLGS_OK;
}

int hlgs_rasterize_forward_render(const hlgs_raster_args* a, const int* radii, void* geom, void* img, void* binning,
                                  const hlgs_frame_info* info, float* out_color, float* out_invdepth, int* seen,
                                  void* stream)
{
    int rc = validate(a);
    if (rc) return rc;
    const int R = info->num_binned;
    if (a->P == 0) return HLGS_OK;
    // rasterizer_impl.cu:332-333: the hierarchy rasterizer's output stays 0; the alt rasterizer blends anyway (bg)
    if (R == 0 && a->variant != HLGS_VARIANT_ALT) return HLGS_OK;
    FrameOpts o = frame_opts(a->P);  // the options _prepare ran with (info), not the switches' state now
    o.pack = info->entry_shift == kEntryShift ? 1 : 0;
    o.drop = info->drops_empty ? 1 : 0;
    if ((info->entry_shift != 0 && info->entry_shift != kEntryShift) || (o.pack && !pack_entries_fit(a->P)) ||
        (o.drop && !o.pack))
        return fail(HLGS_ERR_ARG, "hlgs_frame_info does not come from hlgs_rasterize_forward_prepare of this frame");
    return render_launch(a, o, radii, geom, img, binning, R, (uint32_t)info->max_tile_count, out_color, out_invdepth,
                         seen, (hipStream_t)stream, Guard{nullptr, 0u, 0u});
}

int hlgs_rasterize_forward(const hlgs_raster_args* a, void* geom, void* img, int* radii, void* binning,
                           size_t binning_bytes, hlgs_frame_info* info, float* out_color, float* out_invdepth,
                           int* seen, void* stream)
{
    int rc = validate(a);
    if (rc) return rc;
    info->num_rendered = 0;
    info->max_tile_count = 0;
    info->rendered = 0;
    info->num_binned = 0;
    const FrameOpts o = frame_opts(a->P);  // read once: every launch of this frame uses these
    set_frame_flags(info, o);
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    const size_t HW = (size_t)a->W * a->H;
    const bool alt = a->variant == HLGS_VARIANT_ALT;
    if (a->P == 0) {
        HLGS_TRY_HIP(hipMemsetAsync(out_color, 0, 3 * sizeof(float) * HW, s));
        if (out_invdepth) HLGS_TRY_HIP(hipMemsetAsync(out_invdepth, 0, sizeof(float) * HW, s));
        info->rendered = 1;
        return HLGS_OK;
    }
    Readback* rb;
    if ((rc = readback_for(s, &rb))) return rc;
    if (++rb->seq == 0u) rb->seq = 1u;
    const uint32_t seq = rb->seq;
    if ((rc = prepare_launch(a, o, geom, img, radii, seen, rb->host, seq, s))) return rc;
    Img im = carve_img(aligned(img), a->W, a->H, nullptr);
    // the LDS-binning plan (k_plan) mirrors its words with the sequence number; the generic path copies them
    const bool polled = lds_binning(a->P, (a->W + 15) / 16, (a->H + 15) / 16);
    if (!polled) HLGS_TRY_HIP(hipEventRecord(rb->ev, s));
    // Queue the render before knowing R: it is sized for the caller's buffer and for lists the one-wave and
    // block sorts handle; the kernels exit at once if the frame exceeds either (Guard).
    const int capR = binning ? binning_capacity(binning_bytes) : 0;
    const bool spec = capR > 0;
    // the queued sorts are the ones the previous frame's longest list needed
    const uint32_t cap_n = rb->last_maxc <= (uint32_t)kWaveSortCap ? (uint32_t)kWaveSortCap : (uint32_t)kSortCap;
    if (spec && (rc = render_launch(a, o, radii, geom, img, binning, capR, cap_n, out_color, out_invdepth, seen, s,
                                    Guard{im.misc, (uint32_t)capR, cap_n})))
        return rc;
    uint32_t words[3];
    if (polled) {
        if ((rc = wait_plan_words(rb->host, seq, s, words))) return rc;
    } else {
        HLGS_TRY_HIP(hipEventSynchronize(rb->ev));
        for (int i = 0; i < 3; i++) words[i] = rb->host[i];
    }
    bool replanned = false;
    if (words[0] == ~0u) {
        // The fused plan's look-back timed out (k_tile_offsets_plan): the speculative render exited at once (R exceeds
        // every capacity); plan again with the two launches that need no inter-block wait, then render.
        if (++rb->seq == 0u) rb->seq = 1u;
        if ((rc = replan_launch(a, o, geom, img, radii, rb->host, rb->seq, s))) return rc;
        if ((rc = wait_plan_words(rb->host, rb->seq, s, words))) return rc;
        if (words[0] == ~0u) return fail(HLGS_ERR_DEVICE, "the binning plan failed twice");
        replanned = true;
    }
    const uint32_t R = words[0], maxc = words[1];
    rb->last_maxc = maxc;
    info->num_binned = (int)R;
    info->num_rendered = (int)words[2];
    info->max_tile_count = (int)maxc;
    if (R == 0 && !alt) {  // rasterizer_impl.cu:332-333: the output stays 0 (not bg)
        HLGS_TRY_HIP(hipMemsetAsync(out_color, 0, 3 * sizeof(float) * HW, s));
        if (out_invdepth) HLGS_TRY_HIP(hipMemsetAsync(out_invdepth, 0, sizeof(float) * HW, s));
        info->rendered = 1;
        return HLGS_OK;
    }
    if (R > (uint32_t)capR) return HLGS_OK;  // caller allocates hlgs_binning_buffer_size(R), calls _render
    if (!spec || maxc > cap_n || replanned) {
        if ((rc = render_launch(a, o, radii, geom, img, binning, capR, maxc, out_color, out_invdepth, seen, s,
                                Guard{nullptr, 0u, 0u})))
            return rc;
    }
    info->rendered = 1;
    return HLGS_OK;
}

// one hand-over event per thread (a stream wait captures the event's state when it is enqueued, so the event is
// free for the next call at once)
static hipEvent_t handover_event()
{
    thread_local hipEvent_t ev = nullptr;
    if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) ev = nullptr;
    return ev;
}

int hlgs_rasterize_backward(const hlgs_raster_args* a, const int* radii, const void* geom, const void* img,
                            const void* binning, int R, void* scratch, const float* dL_dcolor,
                            const float* dL_dinvdepth, const hlgs_grads* out, void* stream)
{
    return hlgs_rasterize_backward_split(a, radii, geom, img, binning, R, scratch, dL_dcolor, dL_dinvdepth, out, stream,
                                         nullptr);
}

int hlgs_rasterize_backward_split(const hlgs_raster_args* a, const int* radii, const void* geom, const void* img,
                                  const void* binning, int R, void* scratch, const float* dL_dcolor,
                                  const float* dL_dinvdepth, const hlgs_grads* out, void* stream, void* late_stream)
{
    int rc = validate(a);
    if (rc) return rc;
    if (!out || !out->dmean2D || !out->dcolor || !out->dopacity || !out->dmean3D || !out->dscale ||
        !out->drot || (a->M > 0 && !out->dsh) || (a->variant == HLGS_VARIANT_ALT && !out->ddc))
        return fail(HLGS_ERR_ARG, "missing gradient output");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    const size_t Pf = (size_t)a->P_full;
    if (a->indices || a->P == 0) {
        // hierarchy mode writes only the rendered rows: clear everything first (rasterize_points.cu:182-190)
        HLGS_TRY_HIP(hipMemsetAsync(out->dmean2D, 0, 12 * Pf, s));
        HLGS_TRY_HIP(hipMemsetAsync(out->dcolor, 0, 12 * Pf, s));
        HLGS_TRY_HIP(hipMemsetAsync(out->dopacity, 0, 4 * Pf, s));
        HLGS_TRY_HIP(hipMemsetAsync(out->dmean3D, 0, 12 * Pf, s));
        if (out->dcov3D) HLGS_TRY_HIP(hipMemsetAsync(out->dcov3D, 0, 24 * Pf, s));
        if (out->dsh && a->M > 0) HLGS_TRY_HIP(hipMemsetAsync(out->dsh, 0, 12 * (size_t)a->M * Pf, s));
        if (out->ddc) HLGS_TRY_HIP(hipMemsetAsync(out->ddc, 0, 12 * Pf, s));
        HLGS_TRY_HIP(hipMemsetAsync(out->dscale, 0, 12 * Pf, s));
        HLGS_TRY_HIP(hipMemsetAsync(out->drot, 0, 16 * Pf, s));
    }
    if (a->P == 0) return check_stage(s, a->debug, "backward");
    const int gx = (a->W + 15) / 16, gy = (a->H + 15) / 16;
    Geom g = carve_geom(aligned(geom), a->P, nullptr);
    Img im = carve_img(aligned(img), a->W, a->H, nullptr);
    BwdScratch rs = carve_bwd(aligned(scratch), a->P, R, nullptr);
    if (R > 0) {
        Bin b = carve_bin(aligned(binning), R, nullptr);
        stage_mark(s, ST_BLEND_BWD, true);
        launch_blend_bwd(*a, g, im, b, rs, gx, gy, dL_dcolor, dL_dinvdepth, s);
        stage_mark(s, ST_BLEND_BWD, false);
        if ((rc = check_stage(s, a->debug, "blend_bwd"))) return rc;
    }
    hipStream_t late = (hipStream_t)late_stream;
    hipEvent_t ev = nullptr;
    if (late && !(ev = handover_event())) return fail(HLGS_ERR_DEVICE, "hipEventCreateWithFlags failed");
    stage_mark(s, ST_GAUSS_BWD, true);
    launch_gauss_bwd(*a, radii, g, rs, *out, dL_dinvdepth != nullptr, s, late, ev, R > 0 ? im.misc : nullptr);
    stage_mark(s, ST_GAUSS_BWD, false);
    if (late && (rc = check_stage(late, a->debug, "sh_bwd"))) return rc;
    return check_stage(s, a->debug, "gauss_bwd");
}

int hlgs_sh_grad_from_colour(int P, int V, int D, int M, int variant, const float* means3D, const float* campos,
                             const float* drgb, int64_t view_stride, float scale, float* dsh, float* ddc, void* stream)
{
    const bool alt = variant == HLGS_VARIANT_ALT;
    if (P < 0 || V < 1 || D < 0 || D > 3 || M < 0 || M > 16 - (alt ? 1 : 0) || (V > 1 && view_stride < 3 * (int64_t)P))
        return fail(HLGS_ERR_ARG, "sh_grad_from_colour: bad P, V, D or M");
    if (P == 0 || M == 0 && !alt) return HLGS_OK;
    if (!means3D || !campos || !drgb || (M > 0 && !dsh) || (alt && !ddc))
        return fail(HLGS_ERR_ARG, "sh_grad_from_colour: missing buffer");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_sh_from_colour(P, V, D, M, alt, means3D, campos, drgb, view_stride, scale, dsh, ddc, s);
    return check_stage(s, false, "sh_grad_from_colour");
}

int hlgs_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                      uint8_t* present, void* stream)
{
    (void)projmatrix;
    if (P < 0) return fail(HLGS_ERR_ARG, "P < 0");
    if (P == 0) return HLGS_OK;
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_mark_visible(P, means3D, viewmatrix, present, s);
    return check_stage(s, false, "mark_visible");
}

int hlgs_compute_relocation(int P, const float* opacity_old, const float* scale_old, const int* N,
                            const float* binoms, int n_max, float* opacity_new, float* scale_new, void* stream)
{
    if (P < 0) return fail(HLGS_ERR_ARG, "P < 0");
    if (P == 0) return HLGS_OK;
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_relocation(P, opacity_old, scale_old, N, binoms, n_max, opacity_new, scale_new, s);
    return check_stage(s, false, "compute_relocation");
}

int hlgs_activate_forward(int64_t n, const float* opacity_raw, const float* scaling_raw, const float* rotation_raw,
                          float* opacity, float* scales, float* rotations, void* stream)
{
    if (n <= 0) return HLGS_OK;
    if (!opacity_raw || !scaling_raw || !rotation_raw || !opacity || !scales || !rotations)
        return fail(HLGS_ERR_ARG, "missing tensor");
    if ((reinterpret_cast<uintptr_t>(rotation_raw) | reinterpret_cast<uintptr_t>(rotations)) & 15u)
        return fail(HLGS_ERR_ARG, "rotation rows must be 16-byte aligned");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_act_fwd(n, opacity_raw, scaling_raw, rotation_raw, opacity, scales, rotations, s);
    return check_stage(s, false, "activate_forward");
}

int hlgs_activate_backward(int64_t n, const float* opacity, const float* scales, const float* rotation_raw,
                           const float* g_opacity, const float* g_scales, const float* g_rotations, float* d_opacity_raw,
                           float* d_scaling_raw, float* d_rotation_raw, void* stream)
{
    if (n <= 0) return HLGS_OK;
    if ((g_opacity && (!opacity || !d_opacity_raw)) || (g_scales && (!scales || !d_scaling_raw)) ||
        (g_rotations && (!rotation_raw || !d_rotation_raw)))
        return fail(HLGS_ERR_ARG, "missing tensor");
    if ((reinterpret_cast<uintptr_t>(rotation_raw) | reinterpret_cast<uintptr_t>(g_rotations) |
         reinterpret_cast<uintptr_t>(d_rotation_raw)) & 15u)
        return fail(HLGS_ERR_ARG, "rotation rows must be 16-byte aligned");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_act_bwd(n, opacity, scales, rotation_raw, g_opacity, g_scales, g_rotations, d_opacity_raw, d_scaling_raw,
                   d_rotation_raw, s);
    return check_stage(s, false, "activate_backward");
}

int hlgs_adam_update(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, const uint8_t* visible,
                     float lr, float b1, float b2, float eps, uint32_t N, uint32_t M, void* stream)
{
    if ((uint64_t)N * M == 0) return HLGS_OK;
    if (!param || !grad || !exp_avg || !exp_avg_sq || !visible) return fail(HLGS_ERR_ARG, "missing tensor");
    if ((uint64_t)N * M > 0xffffffffull) return fail(HLGS_ERR_ARG, "N * M exceeds 2^32 elements");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_adam(param, grad, exp_avg, exp_avg_sq, visible, lr, b1, b2, eps, N, M, s);
    return check_stage(s, false, "adam_update");
}

int hlgs_morton_codes(int P, const float* xyz, const float* mn, const float* mx, int64_t* codes, void* stream)
{
    if (P < 0) return fail(HLGS_ERR_ARG, "P < 0");
    if (P == 0) return HLGS_OK;
    if (!xyz || !mn || !mx || !codes) return fail(HLGS_ERR_ARG, "missing tensor");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_morton(P, xyz, mn, mx, codes, s);
    return check_stage(s, false, "morton_codes");
}

// ---------------------------------------------------------------- SPT streaming (stream.hip)
size_t hlgs_upper_cut_scratch_size(int N)
{
    const size_t cap = 2 * (size_t)(N > 0 ? N : 0) + 2;
    return 2 * align_up(sizeof(int) * cap) + align_up(2 * sizeof(int)) + align_up(upper_cut_state_bytes()) + kAlign;
}

static int upper_cut_launch(int N, const int* nodes, const float* xyz, const float* bounds, const float* min_dist2,
                            int nviews, const float* planes, const float* campos, float distance_multiplier,
                            int use_frustum, int use_lod, void* scratch, int* cut, int* count_out, hipStream_t s,
                            int** count_dev, const void* order = nullptr)
{
    if (nviews < 1) return fail(HLGS_ERR_ARG, "n_views < 1");
    if (!nodes || !xyz || !cut || !scratch || (use_frustum && (!bounds || !planes)) ||
        (use_lod && (!min_dist2 || !campos)))
        return fail(HLGS_ERR_ARG, "missing tensor");
    hipGetLastError();
    const int cap = 2 * N + 2;
    char* p = static_cast<char*>(aligned(scratch));
    CutArgs a{N, nodes, xyz, bounds, min_dist2, planes, campos, distance_multiplier, use_frustum, use_lod, nviews,
              take<int>(p, cap), take<int>(p, cap), N, cut, nullptr, nullptr, nullptr, nullptr};
    a.count = take<int>(p, 2);
    if (count_out) a.count = count_out;
    char* q = take<char>(p, upper_cut_state_bytes());
    a.state = reinterpret_cast<CutState*>(q);
    a.arrive = reinterpret_cast<unsigned*>(q + sizeof(CutState));
    a.level_counts = reinterpret_cast<int*>(a.arrive + kCutLevelLaunches);
    a.flat = reinterpret_cast<CutFlat*>(q + align_up(sizeof(CutState) + sizeof(unsigned) * kCutLevelLaunches +
                                                     sizeof(int) * 3 * kCutMaxBlocks));
    if (order) launch_upper_cut_flat(a, static_cast<const int*>(order), s);
    else launch_upper_cut(a, s);
    *count_dev = a.count;
    return check_stage(s, false, "upper_tree_cut");
}

int hlgs_upper_tree_cut(int N, const int* nodes, const float* xyz, const float* bounds, const float* min_dist2,
                        const float* planes, const float* campos, float distance_multiplier, int use_frustum,
                        int use_lod, void* scratch, int* cut, int* count, void* stream)
{
    *count = 0;
    if (N < 0) return fail(HLGS_ERR_ARG, "N < 0");
    if (N == 0) return HLGS_OK;
    hipStream_t s = (hipStream_t)stream;
    int* dev = nullptr;
    int rc = upper_cut_launch(N, nodes, xyz, bounds, min_dist2, 1, planes, campos, distance_multiplier, use_frustum,
                              use_lod, scratch, cut, nullptr, s, &dev);
    if (rc) return rc;
    int host[2];
    HLGS_TRY_HIP(hipMemcpyAsync(host, dev, sizeof(host), hipMemcpyDeviceToHost, s));
    HLGS_TRY_HIP(hipStreamSynchronize(s));
    if (host[1]) return fail(HLGS_ERR_ARG, "upper-tree cut outgrew the node count (not a tree?)");
    *count = host[0];
    return HLGS_OK;
}

int hlgs_upper_tree_cut_views_device(int N, const int* nodes, const float* xyz, const float* bounds,
                                     const float* min_dist2, int n_views, const float* planes, const float* campos,
                                     float distance_multiplier, int use_frustum, int use_lod, void* scratch, int* cut,
                                     int* count_device, void* stream)
{
    if (N < 0) return fail(HLGS_ERR_ARG, "N < 0");
    if (!count_device) return fail(HLGS_ERR_ARG, "missing count");
    hipStream_t s = (hipStream_t)stream;
    if (N == 0) {
        HLGS_TRY_HIP(hipMemsetAsync(count_device, 0, 2 * sizeof(int), s));
        return HLGS_OK;
    }
    int* dev = nullptr;
    return upper_cut_launch(N, nodes, xyz, bounds, min_dist2, n_views, planes, campos, distance_multiplier,
                            use_frustum, use_lod, scratch, cut, count_device, s, &dev);
}

int hlgs_upper_tree_cut_views_ordered_device(int N, const int* nodes, const void* order, const float* xyz,
                                             const float* bounds, const float* min_dist2, int n_views,
                                             const float* planes, const float* campos, float distance_multiplier,
                                             int use_frustum, int use_lod, void* scratch, int* cut, int* count_device,
                                             void* stream)
{
    if (N < 0) return fail(HLGS_ERR_ARG, "N < 0");
    if (!count_device) return fail(HLGS_ERR_ARG, "missing count");
    hipStream_t s = (hipStream_t)stream;
    if (N == 0) {
        HLGS_TRY_HIP(hipMemsetAsync(count_device, 0, 2 * sizeof(int), s));
        return HLGS_OK;
    }
    int* dev = nullptr;
    return upper_cut_launch(N, nodes, xyz, bounds, min_dist2, n_views, planes, campos, distance_multiplier,
                            use_frustum, use_lod, scratch, cut, count_device, s, &dev, order);
}

int hlgs_upper_tree_cut_device(int N, const int* nodes, const float* xyz, const float* bounds, const float* min_dist2,
                               const float* planes, const float* campos, float distance_multiplier, int use_frustum,
                               int use_lod, void* scratch, int* cut, int* count_device, void* stream)
{
    return hlgs_upper_tree_cut_views_device(N, nodes, xyz, bounds, min_dist2, 1, planes, campos, distance_multiplier,
                                            use_frustum, use_lod, scratch, cut, count_device, stream);
}

int hlgs_gather_rows(int64_t n, int row_bytes, const int64_t* idx, const void* src, void* dst, void* stream)
{
    if (n < 0 || row_bytes < 0 || row_bytes % 4) return fail(HLGS_ERR_ARG, "row size must be a multiple of 4 bytes");
    if (n == 0 || row_bytes == 0) return HLGS_OK;
    if (!idx || !src || !dst) return fail(HLGS_ERR_ARG, "missing tensor");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_rows(true, n, row_bytes, idx, src, dst, s);
    return check_stage(s, false, "gather_rows");
}

int hlgs_scatter_rows(int64_t n, int row_bytes, const int64_t* idx, const void* src, void* dst, void* stream)
{
    if (n < 0 || row_bytes < 0 || row_bytes % 4) return fail(HLGS_ERR_ARG, "row size must be a multiple of 4 bytes");
    if (n == 0 || row_bytes == 0) return HLGS_OK;
    if (!idx || !src || !dst) return fail(HLGS_ERR_ARG, "missing tensor");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_rows(false, n, row_bytes, idx, src, dst, s);
    return check_stage(s, false, "scatter_rows");
}

size_t hlgs_spt_cache_scratch_size(int n_cut, int m, int R, int num_spts)
{
    const size_t c = n_cut > 0 ? n_cut : 0, r = R > 0 ? R : 0, ns = num_spts > 0 ? num_spts : 0;
    (void)m;
    return align_up(4 * ns) + 2 * align_up(4 * c) + 2 * align_up(4 * (r + 1)) + 2 * align_up(4 * r) +
           align_up(4 * scan_scratch_elems(r + 1)) + align_up(4 * 8) + kAlign;
}

int hlgs_spt_cache_plan(const hlgs_cache_args* a, hlgs_cache_plan* pl, void* scratch, void* stream)
{
    if (!a || !pl) return fail(HLGS_ERR_ARG, "missing argument");
    pl->n_kept = pl->n_load = pl->n_upper = pl->n_keep_rows = pl->prefix = 0;
    if (a->n_cut < 0 || a->m < 0 || a->R < 0 || a->num_spts < 0) return fail(HLGS_ERR_ARG, "negative size");
    if (!scratch || (a->n_cut && (!a->cut || !a->upper_nodes || !a->upper_xyz || !a->campos)) ||
        (a->m && (!a->prev_spt_indices || !a->prev_spt_distances || !a->prev_spt_counts)) ||
        (a->R && !a->render_indices))
        return fail(HLGS_ERR_ARG, "missing tensor");
    if ((a->m && (!pl->keep_spt_indices || !pl->keep_spt_distances || !pl->keep_spt_counts)) ||
        (a->n_cut && (!pl->load_spt_indices || !pl->load_spt_distances || !pl->upper_render)) ||
        (a->R && (!pl->keep_rows || !pl->render_kept || !pl->write_back_rows || !pl->write_back_indices)))
        return fail(HLGS_ERR_ARG, "missing output");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    const int R = a->R;
    char* p = static_cast<char*>(aligned(scratch));
    CacheArgs c{};
    c.n_cut = a->n_cut;
    c.n_cut_dev = a->n_cut_device;
    c.cut = a->cut;
    c.nodes = a->upper_nodes;
    c.xyz = a->upper_xyz;
    c.campos = a->campos;
    c.nviews = a->n_views > 1 ? a->n_views : 1;
    c.dmul = a->distance_multiplier;
    c.num_spts = a->num_spts;
    c.m = a->m;
    c.prev_idx = a->prev_spt_indices;
    c.prev_dist = a->prev_spt_distances;
    c.prev_counts = a->prev_spt_counts;
    c.R = R;
    c.tail_end = R - a->n_loaded_prev;
    c.rtol = a->rtol;
    c.atol = a->atol;
    c.flag = take<int>(p, a->num_spts);
    c.spt_idx = take<int>(p, a->n_cut);
    c.spt_dist = take<float>(p, a->n_cut);
    c.diff = take<int>(p, (size_t)R + 1);
    uint32_t* diff_incl = take<uint32_t>(p, (size_t)R + 1);
    uint32_t* keep = take<uint32_t>(p, R);
    uint32_t* keep_incl = take<uint32_t>(p, R);
    uint32_t* tmp = take<uint32_t>(p, scan_scratch_elems((size_t)R + 1));
    c.sizes = take<int>(p, 8);
    c.keep_idx = pl->keep_spt_indices;
    c.keep_dist = pl->keep_spt_distances;
    c.keep_counts = pl->keep_spt_counts;
    c.load_idx = pl->load_spt_indices;
    c.load_dist = pl->load_spt_distances;
    c.upper = pl->upper_render;
    if (a->num_spts) HLGS_TRY_HIP(hipMemsetAsync(c.flag, 0, sizeof(int) * a->num_spts, s));
    HLGS_TRY_HIP(hipMemsetAsync(c.diff, 0, sizeof(int) * ((size_t)R + 1), s));
    HLGS_TRY_HIP(hipMemsetAsync(c.sizes, 0, sizeof(int) * 8, s));
    launch_cache_lists(c, s);
    if (R > 0) {
        scan_inclusive_u32(reinterpret_cast<const uint32_t*>(c.diff), diff_incl, R, tmp, s);
        launch_cache_keep(R, a->skybox_points, diff_incl, keep, s);
        scan_inclusive_u32(keep, keep_incl, R, tmp, s);
        launch_cache_split(R, a->render_indices, keep_incl, pl->keep_rows, pl->render_kept, pl->write_back_rows,
                           pl->write_back_indices, s);
        HLGS_TRY_HIP(hipMemcpyAsync(c.sizes + 4, keep_incl + (R - 1), sizeof(int), hipMemcpyDeviceToDevice, s));
    }
    int rc = check_stage(s, false, "spt_cache_plan");
    if (rc) return rc;
    int host[6];
    HLGS_TRY_HIP(hipMemcpyAsync(host, c.sizes, sizeof(host), hipMemcpyDeviceToHost, s));
    HLGS_TRY_HIP(hipStreamSynchronize(s));
    if (host[5]) return fail(HLGS_ERR_ARG, "upper-tree cut outgrew the node count (not a tree?)");
    pl->n_kept = host[0];
    pl->n_load = host[1];
    pl->n_upper = host[2];
    pl->prefix = host[3];
    pl->n_keep_rows = host[4];
    return HLGS_OK;
}

static bool is_device_memory(const void* p)
{
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeDevice;
}

int hlgs_copy_rows(int T, const hlgs_row_copy* tables, int64_t n, const int* src_rows, const int* dst_rows,
                   void* stream)
{
    if (T < 0 || T > kMaxRowTables) return fail(HLGS_ERR_ARG, "at most 32 tables");
    if (n < 0) return fail(HLGS_ERR_ARG, "n < 0");
    if (T == 0 || n == 0) return HLGS_OK;
    if (!tables) return fail(HLGS_ERR_ARG, "missing tables");
    RowCopy rc_[kMaxRowTables];
    for (int t = 0; t < T; t++) {
        if (tables[t].row_bytes < 0 || tables[t].row_bytes % 4) return fail(HLGS_ERR_ARG, "row size must be a multiple of 4 bytes");
        if (tables[t].row_bytes && (!tables[t].src || !tables[t].dst)) return fail(HLGS_ERR_ARG, "missing tensor");
        rc_[t] = RowCopy{tables[t].src, tables[t].dst, tables[t].row_bytes, is_device_memory(tables[t].src) &&
                                                                             is_device_memory(tables[t].dst)};
    }
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_rows_multi(T, rc_, n, src_rows, dst_rows, s);
    return check_stage(s, false, "copy_rows");
}

int hlgs_copy_rows_packed(int T, const hlgs_row_copy* tables, int64_t n, const int* dev_rows, const int* host_rows,
                          void* host, int64_t host_row_bytes, int to_host, void* stream)
{
    if (T < 0 || T > kMaxRowTables) return fail(HLGS_ERR_ARG, "at most 32 tables");
    if (n < 0) return fail(HLGS_ERR_ARG, "n < 0");
    if (host_row_bytes <= 0 || host_row_bytes % 64 || host_row_bytes > 64 * 4 * kPackSlots)
        return fail(HLGS_ERR_ARG, "host row size must be a multiple of 64 bytes, at most 1024");
    if (T == 0 || n == 0) return HLGS_OK;
    if (!tables || !host) return fail(HLGS_ERR_ARG, "missing tables or host storage");
    float* tabs[kMaxRowTables];
    int words[kMaxRowTables];
    int64_t used = 0;
    for (int t = 0; t < T; t++) {
        if (tables[t].row_bytes < 0 || tables[t].row_bytes % 4) return fail(HLGS_ERR_ARG, "row size must be a multiple of 4 bytes");
        if (tables[t].row_bytes && !tables[t].src) return fail(HLGS_ERR_ARG, "missing tensor");
        tabs[t] = (float*)tables[t].src;
        words[t] = (int)(tables[t].row_bytes / 4);
        used += tables[t].row_bytes;
    }
    if (used > host_row_bytes) return fail(HLGS_ERR_ARG, "the tables' rows exceed the host row");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_rows_packed(T, tabs, words, n, dev_rows, host_rows, (float*)host, (int)(host_row_bytes / 4), to_host != 0, s);
    return check_stage(s, false, "copy_rows_packed");
}

int hlgs_load_rows_packed(int T, const hlgs_row_copy* tables, int64_t n, const int* host_rows, const int* resident_of,
                          const void* host, int64_t host_row_bytes, void* stream)
{
    if (T < 0 || T > kMaxRowTables) return fail(HLGS_ERR_ARG, "at most 32 tables");
    if (n < 0) return fail(HLGS_ERR_ARG, "n < 0");
    if (host_row_bytes <= 0 || host_row_bytes % 64 || host_row_bytes > 64 * 4 * kPackSlots)
        return fail(HLGS_ERR_ARG, "host row size must be a multiple of 64 bytes, at most 1024");
    if (T == 0 || n == 0) return HLGS_OK;
    if (!tables || !host || !host_rows) return fail(HLGS_ERR_ARG, "missing tables, rows or host storage");
    float* dst[kMaxRowTables];
    const float* res[kMaxRowTables];
    int words[kMaxRowTables];
    int64_t used = 0;
    for (int t = 0; t < T; t++) {
        if (tables[t].row_bytes < 0 || tables[t].row_bytes % 4) return fail(HLGS_ERR_ARG, "row size must be a multiple of 4 bytes");
        if (tables[t].row_bytes && (!tables[t].dst || (resident_of && !tables[t].src))) return fail(HLGS_ERR_ARG, "missing tensor");
        dst[t] = (float*)tables[t].dst;
        res[t] = (const float*)tables[t].src;
        words[t] = (int)(tables[t].row_bytes / 4);
        used += tables[t].row_bytes;
    }
    if (used > host_row_bytes) return fail(HLGS_ERR_ARG, "the tables' rows exceed the host row");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_rows_packed(T, dst, words, n, nullptr, host_rows, (float*)host, (int)(host_row_bytes / 4), false, s, res,
                       resident_of);
    return check_stage(s, false, "load_rows_packed");
}

int hlgs_adam_step(int T, const hlgs_adam_tensor* tensors, int64_t step, int skybox_rows, double beta1, double beta2,
                   double eps, void* stream)
{
    if (T < 0 || T > kMaxRowTables) return fail(HLGS_ERR_ARG, "at most 32 tensors");
    if (T == 0) return HLGS_OK;
    if (!tensors) return fail(HLGS_ERR_ARG, "missing tensors");
    if (step < 1) return fail(HLGS_ERR_ARG, "step must be >= 1");
    // Python-float scalars as _single_tensor_adam2 forms them (OurAdam.py:425-432), each rounded to float32
    // where torch hands it to a float32 kernel
    const double bc1 = 1.0 - std::pow(beta1, (double)step);
    const double bc2 = 1.0 - std::pow(beta2, (double)step);
    AdamTensor at[kMaxRowTables];
    for (int t = 0; t < T; t++) {
        const hlgs_adam_tensor& x = tensors[t];
        if (x.numel < 0 || x.row_elems < 0) return fail(HLGS_ERR_ARG, "negative size");
        if (x.numel && (!x.param || !x.grad || !x.exp_avg || !x.exp_avg_sq)) return fail(HLGS_ERR_ARG, "missing tensor");
        at[t] = AdamTensor{x.param, x.grad, x.exp_avg, x.exp_avg_sq, x.numel, x.row_elems, (float)(-(x.lr / bc1))};
    }
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_adam_multi(T, at, skybox_rows < 0 ? 0 : skybox_rows, (float)beta1, (float)(1.0 - beta1), (float)beta2,
                      (float)(1.0 - beta2), (float)std::sqrt(bc2), (float)eps, s);
    return check_stage(s, false, "adam_step");
}

// ---------------------------------------------------------------- losses
size_t hlgs_ssim_scratch_size(int C, int H, int W)
{
    if (C <= 0 || H <= 0 || W <= 0) return kAlign;
    return align_up(2 * sizeof(float) * ssim_partials(C, H, W)) + kAlign;
}

int hlgs_ssim_forward_ex(int C, int H, int W, const float* img1, const float* img2, int flags, float* dmaps,
                         void* scratch, float* out, void* stream)
{
    const int valid = flags & HLGS_SSIM_VALID;
    if (C <= 0 || H <= 0 || W <= 0) return fail(HLGS_ERR_ARG, "empty image");
    if (flags & ~(HLGS_SSIM_VALID | HLGS_SSIM_CLAMP1)) return fail(HLGS_ERR_ARG, "unknown SSIM flags");
    if (valid && (H <= 10 || W <= 10)) return fail(HLGS_ERR_ARG, "padding='valid' needs images larger than 10x10");
    if (!img1 || !img2 || !scratch || !out) return fail(HLGS_ERR_ARG, "missing tensor");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_ssim_forward(C, H, W, img1, img2, valid, dmaps, static_cast<float*>(aligned(scratch)), out, s,
                        (flags & HLGS_SSIM_CLAMP1) != 0);
    return check_stage(s, false, "ssim_forward");
}

int hlgs_ssim_forward(int C, int H, int W, const float* img1, const float* img2, int valid, float* dmaps,
                      void* scratch, float* out, void* stream)
{
    return hlgs_ssim_forward_ex(C, H, W, img1, img2, valid ? HLGS_SSIM_VALID : 0, dmaps, scratch, out, stream);
}

int hlgs_ssim_backward_ex(int C, int H, int W, const float* img1, const float* img2, int flags, const float* dmaps,
                          const float* coef, float* grad_img1, void* stream)
{
    if (C <= 0 || H <= 0 || W <= 0) return fail(HLGS_ERR_ARG, "empty image");
    if (flags & ~(HLGS_SSIM_VALID | HLGS_SSIM_CLAMP1)) return fail(HLGS_ERR_ARG, "unknown SSIM flags");
    if (!img1 || !img2 || !dmaps || !coef || !grad_img1) return fail(HLGS_ERR_ARG, "missing tensor");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_ssim_backward(C, H, W, img1, img2, dmaps, coef, grad_img1, s, (flags & HLGS_SSIM_CLAMP1) != 0);
    return check_stage(s, false, "ssim_backward");
}

int hlgs_ssim_backward(int C, int H, int W, const float* img1, const float* img2, const float* dmaps,
                       const float* coef, float* grad_img1, void* stream)
{
    return hlgs_ssim_backward_ex(C, H, W, img1, img2, 0, dmaps, coef, grad_img1, stream);
}

size_t hlgs_depth_l1_scratch_size(int64_t n)
{
    return align_up(sizeof(float) * (size_t)depth_l1_blocks(n > 0 ? n : 1)) + kAlign;
}

int hlgs_depth_l1_forward(int64_t n, const float* invdepth, const float* mono, const float* mask, void* scratch,
                          float* out, void* stream)
{
    if (n <= 0) return fail(HLGS_ERR_ARG, "empty depth map");
    if (!invdepth || !mono || !scratch || !out) return fail(HLGS_ERR_ARG, "missing tensor");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_depth_l1_forward(n, invdepth, mono, mask, static_cast<float*>(aligned(scratch)), out, s);
    return check_stage(s, false, "depth_l1_forward");
}

int hlgs_depth_l1_backward(int64_t n, const float* invdepth, const float* mono, const float* mask, const float* coef,
                           float* grad, void* stream)
{
    if (n <= 0) return fail(HLGS_ERR_ARG, "empty depth map");
    if (!invdepth || !mono || !coef || !grad) return fail(HLGS_ERR_ARG, "missing tensor");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_depth_l1_backward(n, invdepth, mono, mask, coef, grad, s);
    return check_stage(s, false, "depth_l1_backward");
}

// ---------------------------------------------------------------- LOD
size_t hlgs_lod_scratch_size(int N)
{
    const size_t n = N < 0 ? 0 : (size_t)N;
    return align_up(4 * n) * 2 + align_up(4 * scan_scratch_elems(n)) + kAlign;
}

struct LodScratch {
    uint32_t *counts, *incl, *tmp;
};
static LodScratch carve_lod(void* base, int N)
{
    char* p = static_cast<char*>(aligned(base));
    LodScratch l;
    l.counts = take<uint32_t>(p, N);
    l.incl = take<uint32_t>(p, N);
    l.tmp = take<uint32_t>(p, scan_scratch_elems(N));
    return l;
}

static int read_count(const uint32_t* dev, int* count, hipStream_t s)
{
    uint32_t c = 0;
    HLGS_TRY_HIP(hipMemcpyAsync(&c, dev, sizeof(c), hipMemcpyDeviceToHost, s));
    HLGS_TRY_HIP(hipStreamSynchronize(s));
    *count = (int)c;
    return HLGS_OK;
}

int hlgs_expand_to_size_dynamic(int N, float target_size, const int* nodes, const float* positions,
                                const float* scales, const float* viewpoint, const float* viewdir_host,
                                int* render_indices, int* parent_indices, int* nodes_for_render_indices,
                                void* scratch, int* count, void* stream)
{
    *count = 0;
    if (N < 0) return fail(HLGS_ERR_ARG, "N < 0");
    if (N == 0) return HLGS_OK;
    if (!render_indices || !parent_indices || !nodes_for_render_indices || !viewdir_host)
        return fail(HLGS_ERR_ARG, "missing output buffer");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    LodScratch l = carve_lod(scratch, N);
    launch_expand_dynamic(N, target_size, nodes, positions, scales, viewpoint, viewdir_host, render_indices,
                          parent_indices, nodes_for_render_indices, l.counts, l.incl, l.tmp, s);
    int rc = check_stage(s, false, "expand_to_size_dynamic");
    if (rc) return rc;
    return read_count(l.incl + (N - 1), count, s);
}

int hlgs_get_interpolation_weights_dynamic(int n, const int* node_indices, float target_size, const int* nodes,
                                           const float* positions, const float* scales,
                                           const float* viewpoint_host, const float* viewdir_host, float* ts,
                                           int* kids, void* stream)
{
    (void)viewdir_host;
    if (n < 0) return fail(HLGS_ERR_ARG, "n < 0");
    if (n == 0) return HLGS_OK;
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_weights_dynamic(n, node_indices, target_size, nodes, positions, scales, viewpoint_host, ts, kids, s);
    return check_stage(s, false, "get_interpolation_weights_dynamic");
}

int hlgs_expand_to_size(int N, float target_size, const int* nodes, const float* boxes, const float* viewpoint,
                        const float* viewdir_host, int* render_indices, int* parent_indices,
                        int* nodes_for_render_indices, void* scratch, int* count, void* stream)
{
    (void)viewdir_host;
    *count = 0;
    if (N < 0) return fail(HLGS_ERR_ARG, "N < 0");
    if (N == 0) return HLGS_OK;
    if (!render_indices) return fail(HLGS_ERR_ARG, "missing output buffer");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    LodScratch l = carve_lod(scratch, N);
    launch_expand_static(N, target_size, nodes, boxes, viewpoint, render_indices, parent_indices,
                         nodes_for_render_indices, l.counts, l.incl, l.tmp, s);
    int rc = check_stage(s, false, "expand_to_size");
    if (rc) return rc;
    return read_count(l.incl + (N - 1), count, s);
}

int hlgs_get_interpolation_weights(int n, const int* node_indices, float target_size, const int* nodes,
                                   const float* boxes, const float* viewpoint_host, const float* viewdir_host,
                                   float* ts, int* kids, void* stream)
{
    (void)viewdir_host;
    if (n < 0) return fail(HLGS_ERR_ARG, "n < 0");
    if (n == 0) return HLGS_OK;
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_weights_static(n, node_indices, target_size, nodes, boxes, viewpoint_host, ts, kids, s);
    return check_stage(s, false, "get_interpolation_weights");
}

// ---------------------------------------------------------------- SPT cut
struct SptScratch {
    uint32_t *sizes, *incl, *counts, *counts_incl, *tmp;
};
static SptScratch carve_spt(void* base, int s_, size_t* total)
{
    char* p = static_cast<char*>(aligned(base));
    char* p0 = p;
    SptScratch r;
    r.sizes = take<uint32_t>(p, s_);
    r.incl = take<uint32_t>(p, s_);
    r.counts = take<uint32_t>(p, s_);
    r.counts_incl = take<uint32_t>(p, s_);
    r.tmp = take<uint32_t>(p, scan_scratch_elems(s_));
    if (total) *total = (size_t)(p - p0);
    return r;
}
struct SptWork {
    int* result;
    uint32_t *keep, *keep_incl, *tmp;
};
static SptWork carve_spt_work(void* base, int n, size_t* total)
{
    char* p = static_cast<char*>(aligned(base));
    char* p0 = p;
    SptWork w;
    w.result = take<int>(p, n);
    w.keep = take<uint32_t>(p, n);
    w.keep_incl = take<uint32_t>(p, n);
    w.tmp = take<uint32_t>(p, scan_scratch_elems(n));
    if (total) *total = (size_t)(p - p0);
    return w;
}

size_t hlgs_spt_scratch_size(int s_)
{
    size_t t = 0;
    carve_spt(nullptr, s_ < 0 ? 0 : s_, &t);
    return t + kAlign;
}
size_t hlgs_spt_work_size(int n)
{
    size_t t = 0;
    carve_spt_work(nullptr, n < 0 ? 0 : n, &t);
    return t + kAlign;
}

int hlgs_spt_cut_prepare(int s_, const int* SPT_starts, const float* SPT_max, const int* SPT_indices,
                         const float* SPT_distances, void* scratch, int* n_candidates, void* stream)
{
    *n_candidates = 0;
    if (s_ < 0) return fail(HLGS_ERR_ARG, "number_of_SPTs < 0");
    if (s_ == 0) return HLGS_OK;
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    SptScratch r = carve_spt(scratch, s_, nullptr);
    launch_spt_prepare(s_, SPT_starts, SPT_max, SPT_indices, SPT_distances, r.sizes, r.incl, r.tmp, s);
    int rc = check_stage(s, false, "spt_cut_prepare");
    if (rc) return rc;
    return read_count(r.incl + (s_ - 1), n_candidates, s);
}

int hlgs_spt_cut_finish(int s_, int E, int n_candidates, const int* gaussian_indices, const int* SPT_starts,
                        const float* SPT_min, const int* SPT_indices, const float* SPT_distances, int compat,
                        void* scratch, void* work, int* cut, int* counts_prefix, int* count, void* stream)
{
    *count = 0;
    if (s_ <= 0) return HLGS_OK;
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    SptScratch r = carve_spt(scratch, s_, nullptr);
    SptWork w = carve_spt_work(work, n_candidates, nullptr);
    launch_spt_finish(s_, E, n_candidates, gaussian_indices, SPT_starts, SPT_min, SPT_indices, SPT_distances, compat,
                      r.sizes, r.incl, r.counts, r.counts_incl, r.tmp, w.result, w.keep, w.keep_incl, w.tmp, cut,
                      counts_prefix, s);
    int rc = check_stage(s, false, "spt_cut_finish");
    if (rc) return rc;
    if (n_candidates == 0) return HLGS_OK;
    return read_count(w.keep_incl + (n_candidates - 1), count, s);
}

int hlgs_lod_interp_forward(int S, int n, int M3, const int* ridx, const int* pidx, const float* w,
                            const float* means, const float* scales, const float* rots, const float* opac,
                            const float* shs, float* o_means, float* o_scales, float* o_rots, float* o_opac,
                            float* o_shs, void* stream)
{
    if (S < 0 || n < 0 || M3 < 0) return fail(HLGS_ERR_ARG, "negative size");
    if (S + n == 0) return HLGS_OK;
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_lod_interp_fwd(S, n, M3, ridx, pidx, w, means, scales, rots, opac, M3 ? shs : nullptr, o_means, o_scales,
                          o_rots, o_opac, M3 ? o_shs : nullptr, s);
    return check_stage(s, false, "lod_interp_forward");
}

size_t hlgs_lod_interp_scratch_size(int P, int n)
{
    return 4 * lerp_bwd_scratch_elems(P < 0 ? 0 : P, n < 0 ? 0 : n) + kAlign;
}

int hlgs_lod_interp_backward(int P, int S, int n, int M3, const int* ridx, const int* pidx, const float* w,
                             const float* rots, const float* g_means, const float* g_scales, const float* g_rots,
                             const float* g_opac, const float* g_shs, float* d_means, float* d_scales,
                             float* d_rots, float* d_opac, float* d_shs, void* scratch, void* stream)
{
    if (P < 0 || S < 0 || n < 0 || M3 < 0) return fail(HLGS_ERR_ARG, "negative size");
    if (M3 > 64) return fail(HLGS_ERR_ARG, "SH rows of more than 64 floats");
    if (S > P) return fail(HLGS_ERR_ARG, "skybox prefix longer than the gradient rows");
    if (P == 0) return HLGS_OK;
    if (!scratch) return fail(HLGS_ERR_ARG, "missing scratch");
    hipStream_t s = (hipStream_t)stream;
    hipGetLastError();
    launch_lod_interp_bwd(P, S, n, M3, ridx, pidx, w, rots, g_means, g_scales, g_rots, g_opac, M3 ? g_shs : nullptr,
                          d_means, d_scales, d_rots, d_opac, M3 ? d_shs : nullptr, aligned(scratch), s);
    return check_stage(s, false, "lod_interp_backward");
}

// ---------------------------------------------------------------- timing hooks
void hlgs_set_stage_timing(int mask)
{
    g_timing_mask = (uint32_t)mask;
    g_timing = mask != 0;
    for (int i = 0; i < ST_COUNT; i++) g_calls[i] = 0;
}
int hlgs_stage_count(void) { return ST_COUNT; }
const char* hlgs_stage_name(int i) { return (i >= 0 && i < ST_COUNT) ? kStageNames[i] : ""; }
int hlgs_stage_stats(float* mean_ms, int* calls, int max)
{
    const int n = max < ST_COUNT ? max : ST_COUNT;
    for (int i = 0; i < n; i++) {
        double tot = 0.0;
        int k = 0;
        for (int c = 0; c < g_calls[i]; c++) {
            float t = 0.f;
            if (hipEventSynchronize(g_ev[i][1][c]) != hipSuccess) continue;
            if (hipEventElapsedTime(&t, g_ev[i][0][c], g_ev[i][1][c]) != hipSuccess) continue;
            tot += t;
            k++;
        }
        mean_ms[i] = k ? (float)(tot / k) : -1.f;
        calls[i] = k;
    }
    return n;
}

}  // extern "C"
