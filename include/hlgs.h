/*
 * hlgs.h -- C ABI of libhlgs.so, the MI355X (gfx950) differentiable Gaussian-splat rasterizer
 * with hierarchical level-of-detail selection.
 *
 * Drop-in boundary: every entry point below replaces one native function the reference binds
 * through pybind11 (paths relative to /root/reference):
 *
 *   hlgs_rasterize_forward_prepare/_render  <- RasterizeGaussiansCUDA
 *        submodules/hierarchy-rasterizer/rasterize_points.cu:36-139 (bound as _C.rasterize_gaussians,
 *        ext.cpp:16); split in two phases at the reference's own host sync (rasterizer_impl.cu:330-333)
 *        so that the caller allocates the binning buffer, as the reference's resize lambda did
 *        (rasterize_points.cu:28-34).
 *   hlgs_rasterize_backward[_split]         <- RasterizeGaussiansBackwardCUDA, rasterize_points.cu:141-245
 *   hlgs_mark_visible                       <- CudaRasterizer::Rasterizer::markVisible,
 *        rasterizer_impl.cu:145-157 (called as _C.mark_visible at diff_gaussian_rasterization/__init__.py:174)
 *   hlgs_compute_relocation                 <- ComputeRelocationCUDA, rasterize_points.cu:248-271
 *   hlgs_expand_to_size_dynamic             <- ExpandToSizeDynamic, gaussianhierarchy/torch/torch_interface.cpp:171-194
 *   hlgs_get_interpolation_weights_dynamic  <- GetTsIndexedDynamic, torch_interface.cpp:222-244
 *   hlgs_expand_to_size                     <- ExpandToSize, torch_interface.cpp:148-169
 *   hlgs_get_interpolation_weights          <- GetTsIndexed, torch_interface.cpp:200-220
 *   hlgs_spt_cut_prepare/_finish            <- GetSPTCut, torch_interface.cpp:287-316 (two phases at the
 *        reference's candidate-count sync, runtime_switching.cu:926-931)
 *   hlgs_lod_interp_forward/_backward       <- the Python child/parent lerp of render_post,
 *        gaussian_renderer/__init__.py:304-339 (interp_python=True), and its autograd
 *   hlgs_upper_tree_cut, hlgs_spt_cache_plan, hlgs_copy_rows, hlgs_adam_step, hlgs_spt_build
 *                                           <- the SPT streaming step of train_post.py:323-491, 786-812 and
 *        GaussianModel.build_hierarchical_SPT (scene/gaussian_model.py:184-352), which the reference runs as
 *        Python loops over torch ops
 *   hlgs_adam_update                        <- adamUpdate, submodules/alt-rasterizer/rasterize_points.cu:255-281
 *        (kernel cuda_rasterizer/adam.cu:9-36), bound as _C.adamUpdate (ext.cpp:19)
 *
 * The alt rasterizer (submodules/alt-rasterizer: RasterizeGaussiansCUDA rasterize_points.cu:44-137 and
 * RasterizeGaussiansBackwardCUDA :138-232) goes through the same rasterizer entry points with
 * variant = HLGS_VARIANT_ALT (see hlgs_raster_args).
 *
 * Conventions: all pointers are device pointers unless a parameter says "host"; float = IEEE fp32,
 * int = int32; every array is dense and contiguous in the reference's layout (means (P,3), rotations
 * (P,4) as [r,x,y,z], shs (P,M,3), view/proj 16 floats, color (3,H,W)).  Nothing is allocated inside
 * the library: the caller passes buffers sized by the *_size() queries.  Work is launched on `stream`
 * (a hipStream_t; NULL = legacy default stream).  Functions return HLGS_OK or an error code;
 * hlgs_last_error() returns the message for the calling thread.
 */
#ifndef HLGS_H
#define HLGS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HLGS_OK 0
#define HLGS_ERR_ARG 1
#define HLGS_ERR_DEVICE 2

/* Rasterizer variants (hlgs_raster_args.variant). */
#define HLGS_VARIANT_HIERARCHY 0 /* submodules/hierarchy-rasterizer (diff_gaussian_rasterization) */
#define HLGS_VARIANT_ALT 1       /* submodules/alt-rasterizer (alt_gaussian_rasterization): SH split into dc +
                                    rest, optional antialiasing, eigen-radius tile rect with exact per-tile
                                    culling (rasterizer_impl.cu:52-191), background rendered when nothing is
                                    binned, inverse depth always, and its backward (backward.cu:452-624) */

/* Arguments of one rasterizer call: the tensors RasterizeGaussiansCUDA receives. */
typedef struct hlgs_raster_args {
    int P;            /* Gaussians rasterised: indices.size(0) if non-empty, else means3D rows */
    int P_full;       /* means3D rows (gradients are P_full-sized, rasterize_points.cu:171) */
    int D;            /* active SH degree */
    int M;            /* SH coefficients per Gaussian (sh.size(1)), 0 when colors_precomp is used */
    int W, H;
    const float* bg;             /* 3 */
    const float* means3D;        /* P_full x 3 */
    const float* shs;            /* P_full x M x 3, or NULL */
    const float* colors_precomp; /* P x 3, or NULL */
    const float* opacities;      /* P_full */
    const float* scales;         /* P_full x 3 (activated), or NULL with cov3D_precomp */
    const float* rotations;      /* P_full x 4, or NULL with cov3D_precomp */
    const float* cov3D_precomp;  /* P x 6, or NULL */
    const float* viewmatrix;     /* 16 */
    const float* projmatrix;     /* 16 */
    const float* campos;         /* 3 */
    float scale_modifier, tanfovx, tanfovy;
    const int* indices;          /* in-kernel hierarchy mode (all four non-NULL) or NULL */
    const int* parent_indices;
    const float* ts;
    const int* kids;
    int prefiltered;
    int debug;                   /* synchronise + check after every stage (auxiliary.h:23-30) */
    const float* dc;             /* HLGS_VARIANT_ALT: P x 3 degree-0 SH coefficient; shs then holds the M
                                    higher-order ones (P x M x 3).  NULL otherwise. */
    int antialiasing;            /* EWA opacity compensation; the hierarchy rasterizer always applies it */
    int variant;                 /* HLGS_VARIANT_* */
} hlgs_raster_args;

/* Gradient outputs, all P_full rows; written completely by hlgs_rasterize_backward (no pre-zeroing). */
typedef struct hlgs_grads {
    float* dmean2D;   /* P_full x 3 (z stays 0) */
    float* dcolor;    /* P_full x 3 */
    float* dopacity;  /* P_full */
    float* dmean3D;   /* P_full x 3 */
    float* dcov3D;    /* P_full x 6, or NULL: not written (a caller without cov3D_precomp has nothing to return it for) */
    float* dsh;       /* P_full x M x 3 (may be NULL when M == 0) */
    float* dscale;    /* P_full x 3 */
    float* drot;      /* P_full x 4 */
    float* ddc;       /* HLGS_VARIANT_ALT: P_full x 3, else NULL */
    float* drgb;      /* NULL, or P_full x 3: the colour-factored SH gradient (hlgs_sh_grad_from_colour) -- the SH
                         backward then writes dL/dRGB with the clamp mask applied (zero rows for Gaussians it skips)
                         here instead of dsh / ddc, and still adds its view-direction term to dmean3D */
} hlgs_grads;

const char* hlgs_last_error(void);
const char* hlgs_version(void);

/* ---- rasterizer buffer sizing (bytes) ---- */
size_t hlgs_geom_buffer_size(int P);
size_t hlgs_image_buffer_size(int W, int H);
size_t hlgs_binning_buffer_size(int R);
size_t hlgs_backward_scratch_size(int P, int R);

/* Host-side result of phase 1. */
typedef struct hlgs_frame_info {
    int num_rendered;    /* the reference's num_rendered: Gaussian/tile instances over every tile rect (the alt
                            variant counts its culled instances too); sizes hlgs_backward_scratch_size */
    int max_tile_count;  /* longest per-tile list (selects the binning plan) */
    int rendered;        /* hlgs_rasterize_forward: 1 when phase 2 ran inside the call */
    int num_binned;      /* instances actually binned into the per-tile lists (== num_rendered for the
                            hierarchy rasterizer); sizes hlgs_binning_buffer_size */
    int entry_shift;     /* this frame's point_list entries are (index << entry_shift) | quadrant mask (0: plain
                            indices); the switches are read once when the frame starts (hlgs_set_entry_packing) */
    int drops_empty;     /* 1 if this frame's lists drop the instances whose quadrant mask is 0 (hlgs_set_drop_empty);
                            _prepare sets both and _render runs with them */
} hlgs_frame_info;

/* Phase 1: preprocess + scans.  Writes radii (P), fills geom/img and *info (host).  One host
 * synchronisation, as the reference has (rasterizer_impl.cu:330-331). */
int hlgs_rasterize_forward_prepare(const hlgs_raster_args* a, void* geom, void* img, int* radii,
                                   hlgs_frame_info* info, void* stream);
/* Phase 2: binning (per-tile depth sort) + front-to-back blend.  Every pixel of out_color (3,H,W) and
 * out_invdepth (H,W, or NULL when do_depth is off) is written; seen (P, or NULL for the alt variant) must
 * be zero-initialised by the caller.  With nothing binned this is a no-op for the hierarchy rasterizer
 * (the caller's zeroed output stays 0, not bg: rasterizer_impl.cu:332-333); the alt variant renders bg. */
int hlgs_rasterize_forward_render(const hlgs_raster_args* a, const int* radii, void* geom, void* img,
                                  void* binning, const hlgs_frame_info* info, float* out_color,
                                  float* out_invdepth, int* seen, void* stream);
/* Both phases in one call, with one host synchronisation and no return to the caller between them:
 * prepare, then -- when hlgs_binning_buffer_size(num_rendered) <= binning_bytes -- render into
 * `binning` and set info->rendered = 1.  Otherwise info->rendered = 0 and the caller allocates a
 * binning buffer of the reported size and calls hlgs_rasterize_forward_render.  seen is cleared here;
 * out_color / out_invdepth need no initialisation (with R == 0 they are set to 0).
 * Replaces the forward of RasterizeGaussiansCUDA (rasterize_points.cu:36-139). */
int hlgs_rasterize_forward(const hlgs_raster_args* a, void* geom, void* img, int* radii, void* binning,
                           size_t binning_bytes, hlgs_frame_info* info, float* out_color, float* out_invdepth,
                           int* seen, void* stream);
/* Backward: blend backward (per-tile partial sums, no float atomics) + fused covariance / SH / scale-
 * rotation backward.  dL_dinvdepth may be NULL (rasterize_points.cu:195-201).  R = info.num_rendered. */
int hlgs_rasterize_backward(const hlgs_raster_args* a, const int* radii, const void* geom, const void* img,
                            const void* binning, int R, void* scratch, const float* dL_dcolor,
                            const float* dL_dinvdepth, const hlgs_grads* out, void* stream);
/* hlgs_rasterize_backward with the kernels after the covariance backward (the SH backward, which completes dmean3D,
 * dsh and ddc, and the hierarchy-mode parent mean add) launched on late_stream behind an event on stream, and NOT
 * joined back: dopacity, dscale, drot, dcov3D, dmean2D and dcolor are final in stream order, dmean3D / dsh / ddc in
 * late_stream order.  The caller joins (waits on late_stream) before reading those three.  A view-data-parallel
 * exchange uses it to start the collective over the early gradients while the SH backward runs.
 * late_stream = NULL is hlgs_rasterize_backward. */
int hlgs_rasterize_backward_split(const hlgs_raster_args* a, const int* radii, const void* geom, const void* img,
                                  const void* binning, int R, void* scratch, const float* dL_dcolor,
                                  const float* dL_dinvdepth, const hlgs_grads* out, void* stream, void* late_stream);

/* The averaged SH gradient of a view-data-parallel step, rebuilt from each view's colour gradient.
 * One view's SH gradient is an outer product per Gaussian, dL/dsh[c] = basis_c(dir) * dL/dRGB with the clamp mask
 * applied (computeColorFromSH backward, backward.cu:23-142; alt-rasterizer backward.cu:23-146), so ranks exchange the
 * 3-float dL/dRGB rows (hlgs_grads.drgb) instead of the (D+1)^2 x 3 SH rows, and each rank forms
 *   dsh[p][c - OFF][ch] = scale * sum_v basis_c(normalize(mean_p - campos_v)) * drgb[v][p][ch]
 * in view order v = 0..V-1.  View v's campos (3 floats) and drgb (P x 3) start view_stride floats after view v-1's
 * (an exchange gathers them as one row per rank: [campos, pad | drgb]); means3D: P x 3 (device).  dsh: P x M x 3 holds
 * coefficients OFF..OFF+M-1 (OFF = 1 for HLGS_VARIANT_ALT, whose coefficient 0 goes to ddc: P x 3; OFF = 0 and ddc
 * NULL otherwise); coefficients at or above (D+1)^2 are zero. */
int hlgs_sh_grad_from_colour(int P, int V, int D, int M, int variant, const float* means3D, const float* campos,
                             const float* drgb, int64_t view_stride, float scale, float* dsh, float* ddc, void* stream);

/* z > 0.2 visibility (auxiliary.h:164-189); present is P bytes (bool) */
int hlgs_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                      uint8_t* present, void* stream);
/* MCMC relocation, utils.cu:6-36.  scale_new is 3P floats. */
int hlgs_compute_relocation(int P, const float* opacity_old, const float* scale_old, const int* N,
                            const float* binoms, int n_max, float* opacity_new, float* scale_new, void* stream);

/* Sparse Adam step of SparseGaussianAdam (alt_gaussian_rasterization/__init__.py:244-271, adam.cu:9-36):
 * for every element p of the N x M parameter whose Gaussian p / M is visible (visible: N bytes),
 * m = b1 m + (1 - b1) g, v = b2 v + (1 - b2) g^2, param -= lr m / (sqrt(v) + eps).  No bias correction and
 * no step counter, as the reference. */
int hlgs_adam_update(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, const uint8_t* visible,
                     float lr, float b1, float b2, float eps, uint32_t N, uint32_t M, void* stream);

/* ---- hierarchical LOD ---- */
size_t hlgs_lod_scratch_size(int N);
/* nodes: N x 6 int32 HierarchyNode rows; viewpoint: device float3; viewdir: host float[3].
 * Writes the first *count entries of render_indices / parent_indices / nodes_for_render_indices
 * (parent_indices is left untouched for roots, runtime_switching.cu:104-107). */
int hlgs_expand_to_size_dynamic(int N, float target_size, const int* nodes, const float* positions,
                                const float* scales, const float* viewpoint, const float* viewdir_host,
                                int* render_indices, int* parent_indices, int* nodes_for_render_indices,
                                void* scratch, int* count, void* stream);
/* viewpoint_host / viewdir_host: host float[3] (torch_interface.cpp:240-241) */
int hlgs_get_interpolation_weights_dynamic(int n, const int* node_indices, float target_size, const int* nodes,
                                           const float* positions, const float* scales,
                                           const float* viewpoint_host, const float* viewdir_host, float* ts,
                                           int* kids, void* stream);
/* static (.hier) variant: nodes N x 7 int32, boxes N x 8 float (minn xyzw, maxx xyzw) */
int hlgs_expand_to_size(int N, float target_size, const int* nodes, const float* boxes, const float* viewpoint,
                        const float* viewdir_host, int* render_indices, int* parent_indices,
                        int* nodes_for_render_indices, void* scratch, int* count, void* stream);
int hlgs_get_interpolation_weights(int n, const int* node_indices, float target_size, const int* nodes,
                                   const float* boxes, const float* viewpoint_host, const float* viewdir_host,
                                   float* ts, int* kids, void* stream);

/* SPT cut (runtime_switching.cu:878-994).  prepare() computes per-SPT candidate intervals into
 * scratch (hlgs_spt_scratch_size(s) bytes) and returns the candidate total in *n_candidates (host);
 * finish() needs work >= hlgs_spt_work_size(n_candidates) bytes and writes the kept Gaussian indices to
 * cut[0..*count) and the exclusive prefix of per-SPT kept counts to counts_prefix (s).  compat != 0
 * reproduces the reference bit for bit (App. A-10 boundary attribution + dropping index 0). */
size_t hlgs_spt_scratch_size(int s);
size_t hlgs_spt_work_size(int n_candidates);
int hlgs_spt_cut_prepare(int s, const int* SPT_starts, const float* SPT_max, const int* SPT_indices,
                         const float* SPT_distances, void* scratch, int* n_candidates, void* stream);
int hlgs_spt_cut_finish(int s, int E, int n_candidates, const int* gaussian_indices, const int* SPT_starts,
                        const float* SPT_min, const int* SPT_indices, const float* SPT_distances, int compat,
                        void* scratch, void* work, int* cut, int* counts_prefix, int* count, void* stream);

/* LOD interpolation (render_post lerp).  M3 = floats of SH per Gaussian (0: no SH).  Outputs have
 * S + n rows: rows [0,S) copy the skybox prefix, row S+i lerps child ridx[i] with parent pidx[i]. */
int hlgs_lod_interp_forward(int S, int n, int M3, const int* ridx, const int* pidx, const float* w,
                            const float* means, const float* scales, const float* rots, const float* opac,
                            const float* shs, float* o_means, float* o_scales, float* o_rots, float* o_opac,
                            float* o_shs, void* stream);
/* Gradient of the lerp (the autograd of render_post's block, gaussian_renderer/__init__.py:304-339) into the
 * P-row gradient arrays d_*: every row is written (zeros where no output row depends on it), so no
 * initialisation is needed; contributions are gathered per node in a fixed order (bitwise deterministic).
 * scratch: hlgs_lod_interp_scratch_size(P, n) bytes.  M3 <= 64. */
size_t hlgs_lod_interp_scratch_size(int P, int n);
int hlgs_lod_interp_backward(int P, int S, int n, int M3, const int* ridx, const int* pidx, const float* w,
                             const float* rots, const float* g_means, const float* g_scales, const float* g_rots,
                             const float* g_opac, const float* g_shs, float* d_means, float* d_scales,
                             float* d_rots, float* d_opac, float* d_shs, void* scratch, void* stream);

/* Morton codes of P positions in the [mn, mx] box (device float3 each): get_morton_indices,
 * gaussianhierarchy/morton.cu:9-58 via torch_interface.cpp:246-260 (used by GaussianModel.sort_morton,
 * scene/gaussian_model.py:570-589). */
int hlgs_morton_codes(int P, const float* xyz, const float* mn, const float* mx, int64_t* codes, void* stream);

/* ---- SPT streaming around the SPT cut (train_post.py:323-491) ---- */
/* Coarse cut of the upper tree (GaussianModel.cut_hierarchy_on_condition with root 0, no upper-tree output,
 * leave_out_of_cut_condition = frustum_cull_spheres: scene/gaussian_model.py:364-404, 67-100, as train_post.py
 * :326-343 calls it).  nodes: N x 6 int32 upper-tree HierarchyNode rows; xyz N x 3; bounds N (sphere radii);
 * min_dist2 N; planes: 4 x 4 floats (nx, ny, nz, d) from extract_frustum_planes; campos 3.  A node survives the
 * cull unless n.p + d + r < 0 for one plane (use_frustum); it is cut if it is a leaf or (use_lod) if not
 * min_dist2 > |campos - p|^2 * distance_multiplier, else its first child and that child's next sibling are
 * visited.  cut (device, N entries) receives the nodes in the reference's order; *count (host) their number.
 * scratch: hlgs_upper_cut_scratch_size(N) bytes.  One host synchronisation (the reference's len()). */
size_t hlgs_upper_cut_scratch_size(int N);
/* The same cut without the host read: the count and an overflow flag land in count_device[0..1] (device memory),
 * for hlgs_spt_cache_plan's n_cut_device, which reads them in its own single host synchronisation. */
int hlgs_upper_tree_cut_device(int N, const int* nodes, const float* xyz, const float* bounds, const float* min_dist2,
                               const float* planes, const float* campos, float distance_multiplier, int use_frustum,
                               int use_lod, void* scratch, int* cut, int* count_device, void* stream);
int hlgs_upper_tree_cut(int N, const int* nodes, const float* xyz, const float* bounds, const float* min_dist2,
                        const float* planes, const float* campos, float distance_multiplier, int use_frustum,
                        int use_lod, void* scratch, int* cut, int* count, void* stream);
/* The cut for a batch of n_views training views (one per rank of a view-data-parallel step): planes
 * n_views x 4 x 4, campos n_views x 3.  A node survives the cull if its sphere reaches into ANY view's frustum, and
 * expands if min_dist2 > min over views |campos_g - p|^2 * distance_multiplier (the nearest camera decides).  With
 * n_views = 1 this is hlgs_upper_tree_cut_device, bit for bit.  Every rank computing it from the same gathered views
 * obtains the same cut (no train_post.py counterpart: the reference trains one view per step). */
int hlgs_upper_tree_cut_views_device(int N, const int* nodes, const float* xyz, const float* bounds,
                                     const float* min_dist2, int n_views, const float* planes, const float* campos,
                                     float distance_multiplier, int use_frustum, int use_lod, void* scratch, int* cut,
                                     int* count_device, void* stream);
/* The same cut from a precomputed walk order (round 5): two launches (every node's state in parallel, then one
 * workgroup that places the surviving nodes) instead of one per level, with the result of
 * hlgs_upper_tree_cut_views_device bit for bit.  order (device): the blob hlgs_upper_tree_order wrote for these
 * nodes, or NULL for the level walk.  Same scratch. */
int hlgs_upper_tree_cut_views_ordered_device(int N, const int* nodes, const void* order, const float* xyz,
                                             const float* bounds, const float* min_dist2, int n_views,
                                             const float* planes, const float* campos, float distance_multiplier,
                                             int use_frustum, int use_lod, void* scratch, int* cut, int* count_device,
                                             void* stream);
/* Host: the walk order of an upper tree (nodes: N x 6 HierarchyNode rows, host memory) into order_host
 * (hlgs_upper_tree_order_size(N) bytes).  Word 3 holds N: the flat cut refuses (count_device[1] = 1) a blob built for
 * another node count.  Word 2 of the blob is 1 when the flat cut can use it: the nodes form a
 * tree as the reference walks it (root 0; first child, then that child's next sibling) with at most 65,535 nodes
 * on it over at most 64 levels; otherwise use the level walk (order = NULL above). */
#define HLGS_CUT_ORDER_HEADER 80       /* words before the per-entry arrays of the order blob */
#define HLGS_CUT_FLAT_MAX_ENTRIES 65535
#define HLGS_CUT_FLAT_MAX_LEVELS 64
size_t hlgs_upper_tree_order_size(int N);
int hlgs_upper_tree_order(int N, const int* nodes_host, void* order_host);
/* SPT construction (GaussianModel.build_hierarchical_SPT + get_min_distance, scene/gaussian_model.py:184-352), host
 * code over host arrays: nodes G x 6 (HierarchyNode), xyz G x 3, log_scales G x 3 (unactivated, as _scaling);
 * root = the hierarchy root (the reference's default root_node 100000 is its skybox size).  The result is an
 * opaque handle: query the sizes, copy into caller buffers (any pointer may be NULL), free.
 *   starts (n_spt + 1), smax / smin / gidx (n_entries): the SPT arrays get_spt_cut_cuda takes;
 *   roots (n_spt): hierarchy ids of the SPT roots; up_nodes (n_upper x 6), up_xyz, up_scaling (n_upper x 3),
 *   min_d2, radii (n_upper): the upper tree (radii only with use_bounding_spheres). */
typedef struct hlgs_spt_result hlgs_spt_result;
int hlgs_spt_build(int G, const int* nodes, const float* xyz, const float* log_scales, int root, float spt_root_volume,
                   float target_granularity, int min_spt_size, int use_bounding_spheres, hlgs_spt_result** out);
int hlgs_spt_result_sizes(const hlgs_spt_result* r, int* n_spt, int* n_entries, int* n_upper);
int hlgs_spt_result_copy(const hlgs_spt_result* r, int* starts, float* smax, float* smin, int* gidx, int* roots,
                         int* up_nodes, float* up_xyz, float* up_scaling, float* min_d2, float* radii);
void hlgs_spt_result_free(hlgs_spt_result* r);
/* Row gather dst[i] = src[idx[i]] and scatter dst[idx[i]] = src[i] for n rows of row_bytes (a multiple of 4):
 * the streaming cache's storage[idx].cuda() loads and write-backs (train_post.py:439-488).  src / dst may be
 * pinned host memory (read and written by the GPU over the host link). */
int hlgs_gather_rows(int64_t n, int row_bytes, const int64_t* idx, const void* src, void* dst, void* stream);
int hlgs_scatter_rows(int64_t n, int row_bytes, const int64_t* idx, const void* src, void* dst, void* stream);

/* One bookkeeping pass of train_post.py's SPT cache (the body of the budget loop, :346-430): given the view's
 * coarse cut and the previous step's SPT state, decide which SPTs are reused, which are loaded, and which
 * resident Gaussians stay or are written back.  All arrays are device int32/float32 unless noted. */
typedef struct hlgs_cache_args {
    int n_cut;                         /* coarse cut (hlgs_upper_tree_cut) */
    const int* cut;
    const int* upper_nodes;            /* upper tree, n_upper x 6 */
    const float* upper_xyz;            /* n_upper x 3 */
    const float* campos;               /* 3 */
    float distance_multiplier;         /* SPT distances are |xyz - campos| * distance_multiplier */
    int num_spts;                      /* SPT ids are in [0, num_spts) */
    int m;                             /* prev_SPT_indices / _distances / _counts, m each */
    const int* prev_spt_indices;
    const float* prev_spt_distances;
    const int* prev_spt_counts;
    int R;                             /* len(render_indices) */
    const int* render_indices;
    int n_loaded_prev;                 /* len(load_from_disk_indices) of the previous pass */
    int skybox_points;
    float rtol, atol;                  /* isclose of the reused distances (Reuse_SPT_Tolerarance, 0.05) */
    const int* n_cut_device;           /* NULL, or the [count, overflow] words of hlgs_upper_tree_cut_device: the
                                          cut's length is then read on the device and n_cut is its capacity */
    int n_views;                       /* 0 or 1: campos is one camera; > 1: campos is n_views x 3 and each SPT's
                                          distance is that of the nearest camera (hlgs_upper_tree_cut_views_device) */
} hlgs_cache_args;
typedef struct hlgs_cache_plan {
    int* keep_spt_indices;             /* m: keep_SPT_indices */
    float* keep_spt_distances;         /* m: prev_SPT_distances[SPT_keep_counts_indices] */
    int* keep_spt_counts;              /* m: SPT_counts_new[:n_kept] */
    int* load_spt_indices;             /* n_cut: load_SPT_indices (for hlgs_spt_cut_*) */
    float* load_spt_distances;         /* n_cut */
    int* upper_render;                 /* n_cut: upper_tree_nodes_to_render */
    int* keep_rows;                    /* R: nonzero(keep_gaussians_mask) */
    int* render_kept;                  /* R: render_indices[keep_gaussians_mask] */
    int* write_back_rows;              /* R: nonzero(write_back_mask) */
    int* write_back_indices;           /* R: render_indices[write_back_mask] */
    int n_kept, n_load, n_upper;       /* host outputs: list lengths */
    int n_keep_rows;                   /* R - n_keep_rows rows are written back */
    int prefix;                        /* the prefix the loaded SPTs' counts are shifted by (plus skybox_points) */
} hlgs_cache_plan;
/* scratch: hlgs_spt_cache_scratch_size bytes; one host synchronisation for all the sizes. */
size_t hlgs_spt_cache_scratch_size(int n_cut, int m, int R, int num_spts);
int hlgs_spt_cache_plan(const hlgs_cache_args* a, hlgs_cache_plan* plan, void* scratch, void* stream);
/* dst_t[dst_rows[i]] = src_t[src_rows[i]] for i < n and every table t < T (at most 32); a NULL row list is the
 * identity.  row_bytes a multiple of 4; src / dst may be pinned host memory.  All of a cache step's parameter
 * and Adam-moment traffic (train_post.py:439-479) in one launch per direction. */
typedef struct hlgs_row_copy {
    const void* src;
    void* dst;
    int64_t row_bytes;
} hlgs_row_copy;
int hlgs_copy_rows(int T, const hlgs_row_copy* tables, int64_t n, const int* src_rows, const int* dst_rows,
                   void* stream);
/* The host legs of the same traffic with packed host storage: host row h (host_row_bytes bytes, a multiple of 64,
 * at most 1024; pinned host memory) holds the T device tables' rows back to back -- table t's row at the sum of the
 * earlier tables' row_bytes -- then zero padding.  tables[t].src is the device table (dst is ignored), float32
 * rows.  to_host != 0: host[host_rows[i]] = (dev_0[dev_rows[i]], dev_1[dev_rows[i]], ..., 0...) -- whole host
 * rows, padding included;  to_host == 0: dev_t[dev_rows[i]] = the table's part of host[host_rows[i]].  NULL row
 * lists are the identity.  Every store or load the GPU issues to host memory covers whole 64-byte lines, where
 * per-tensor host storage takes one 12-180-byte fragment per tensor and row (train_post.py:439-479). */
int hlgs_copy_rows_packed(int T, const hlgs_row_copy* tables, int64_t n, const int* dev_rows, const int* host_rows,
                          void* host, int64_t host_row_bytes, int to_host, void* stream);
/* The load leg of a cache step with rows that are still resident (train_post.py:446-479 after the write-back of
 * :439-444): dst_t[i] = the table's part of host[host_rows[i]] for i < n, except that a host row h with
 * resident_of[h] = r >= 0 is taken from src_t[r] (tables[t].src, the resident table) instead of over the host
 * link -- the step's write-back has just stored the same bits at h.  tables[t].dst is the destination table;
 * resident_of is indexed by host row (NULL: every row from the host). */
int hlgs_load_rows_packed(int T, const hlgs_row_copy* tables, int64_t n, const int* host_rows, const int* resident_of,
                          const void* host, int64_t host_row_bytes, void* stream);
/* Dense Adam step of the cached training loop (train_post.py:786-812: skybox gradient rows zeroed, then
 * OurAdam._single_tensor_adam2, scene/OurAdam.py:357-448, with state step = step) over T (at most 32) tensors in
 * one launch.  The scalars follow torch: lr, betas and eps are the caller's doubles; step_size =
 * lr / (1 - beta1^step) and sqrt(1 - beta2^step) are formed in double, then every tensor op runs in float32. */
typedef struct hlgs_adam_tensor {
    float* param;
    float* grad;                       /* rows < skybox_rows are set to 0 before the update */
    float* exp_avg;
    float* exp_avg_sq;
    int64_t numel;
    int64_t row_elems;                 /* elements per Gaussian row */
    double lr;
} hlgs_adam_tensor;
int hlgs_adam_step(int T, const hlgs_adam_tensor* tensors, int64_t step, int skybox_rows, double beta1, double beta2,
                   double eps, void* stream);
/* The activations render() reads (scene/gaussian_model.py:44-56: get_opacity = sigmoid(_opacity), get_scaling =
 * exp(_scaling), get_rotation = normalize(_rotation), eps 1e-12) over n resident rows in one pass: opacity_raw n,
 * scaling_raw n x 3, rotation_raw n x 4 (16-byte aligned) -> opacity, scales, rotations (same shapes). */
int hlgs_activate_forward(int64_t n, const float* opacity_raw, const float* scaling_raw, const float* rotation_raw,
                          float* opacity, float* scales, float* rotations, void* stream);
/* Their gradients in one pass: d_opacity_raw = g (1 - o) o, d_scaling_raw = g s, d_rotation_raw through the norm.
 * opacity / scales are the forward's outputs; any (g, d) pair may be NULL to skip that tensor. */
int hlgs_activate_backward(int64_t n, const float* opacity, const float* scales, const float* rotation_raw,
                           const float* g_opacity, const float* g_scales, const float* g_rotations, float* d_opacity_raw,
                           float* d_scaling_raw, float* d_rotation_raw, void* stream);

/* ---- photometric losses of the training step (utils/loss_utils.py:17-63, train_single.py:106-121,
 *      train_post.py:558-559 with the un-vendored fused_ssim) ---- */
/* SSIM of C planes of H x W (11x11 Gaussian window, sigma 1.5, zero padding, C1 = 0.01^2, C2 = 0.03^2:
 * _ssim, loss_utils.py:44-63).  out (device, 2 floats) = (mean of the SSIM map -- over the interior
 * [5, H-5) x [5, W-5) when valid != 0, fused_ssim padding="valid" --, mean |img1 - img2| = l1_loss).
 * dmaps (C x 3 x H x W, or NULL when no gradient is needed) receives the map's derivatives with respect to the
 * window moments for hlgs_ssim_backward.  scratch: hlgs_ssim_scratch_size bytes. */
size_t hlgs_ssim_scratch_size(int C, int H, int W);
int hlgs_ssim_forward(int C, int H, int W, const float* img1, const float* img2, int valid, float* dmaps,
                      void* scratch, float* out, void* stream);
/* grad_img1 = coef[0] * d(sum of the SSIM map)/d img1 + coef[1] * sign(img1 - img2); coef is a device array so
 * the upstream gradient never needs a host read. */
int hlgs_ssim_backward(int C, int H, int W, const float* img1, const float* img2, const float* dmaps,
                       const float* coef, float* grad_img1, void* stream);
/* The same two with flags: HLGS_SSIM_VALID (= valid above) and HLGS_SSIM_CLAMP1 -- img1 enters as clamp(img1, 0, 1),
 * the rendered_image.clamp(0, 1) of the reference's renderers (gaussian_renderer/__init__.py:142, 612) folded into
 * the loss: the forward reads the clamped values, the backward gradient passes only where 0 <= img1 <= 1 (torch's
 * clamp backward), so the two clamp kernels of each direction disappear.  Pass the same flags to both. */
#define HLGS_SSIM_VALID 1
#define HLGS_SSIM_CLAMP1 2
int hlgs_ssim_forward_ex(int C, int H, int W, const float* img1, const float* img2, int flags, float* dmaps,
                         void* scratch, float* out, void* stream);
int hlgs_ssim_backward_ex(int C, int H, int W, const float* img1, const float* img2, int flags, const float* dmaps,
                          const float* coef, float* grad_img1, void* stream);
/* Depth term of train_single.py:111-118: out[0] = mean |(invdepth - mono) * mask| over n values (mask may be
 * NULL); backward grad = coef[0] * sign((invdepth - mono) * mask) * mask. */
size_t hlgs_depth_l1_scratch_size(int64_t n);
int hlgs_depth_l1_forward(int64_t n, const float* invdepth, const float* mono, const float* mask, void* scratch,
                          float* out, void* stream);
int hlgs_depth_l1_backward(int64_t n, const float* invdepth, const float* mono, const float* mask, const float* coef,
                           float* grad, void* stream);

/* ---- hierarchy files and traversal (host code, host buffers; gaussianhierarchy/hierarchy_loader.cpp,
 *      hierarchy_writer.cpp, traversal.cpp -- bound there as load_hierarchy, load_dynamic_hierarchy,
 *      write_hierarchy, write_dynamic_hierarchy, expand_to_target: ext.cpp:16-20) ---- */
#define HLGS_HIER_FULL 0    /* .hier, float32 (hierarchy_writer.cpp:33-57) */
#define HLGS_HIER_HALF 1    /* .hier, binary16 attributes (the default of WriteHierarchy, :58-110) */
#define HLGS_HIER_DYNAMIC 2 /* .dhier (HierarchyNode rows, :113-155) */
typedef struct hlgs_hier_info {
    int format;     /* HLGS_HIER_* */
    int G;          /* Gaussians */
    int N;          /* nodes (.dhier: == G, hierarchy_loader.cpp:185) */
    int sh_degree;  /* .dhier: stored degree (SH rows hold (deg+1)^2 coefficients); .hier: 3 (48 floats) */
} hlgs_hier_info;
/* Sizes of a hierarchy file; dynamic != 0 reads the .dhier header. */
int hlgs_hier_info_read(const char* path, int dynamic, hlgs_hier_info* info);
/* LoadHierarchy (torch_interface.cpp:9-40): pos G x 3, rot G x 4, log_scales G x 3, opacities G, shs G x 48,
 * nodes N x 7 int32 (Node), boxes N x 8 (minn xyzw, maxx xyzw); both the full and the half layout. */
int hlgs_hier_load(const char* path, float* pos, float* rot, float* log_scales, float* opacities, float* shs,
                   int* nodes, float* boxes);
/* WriteHierarchy (torch_interface.cpp:77-104); compressed != 0 writes the binary16 layout (the reference's
 * default) and fails with "Would lose information!" when a node count exceeds 32000. */
int hlgs_hier_write(const char* path, int G, int N, const float* pos, const float* shs, const float* opacities,
                    const float* log_scales, const float* rot, const int* nodes, const float* boxes, int compressed);
/* LoadDynamicHierarchy (torch_interface.cpp:43-74): shs G x (deg+1)^2 x 3, nodes G x 6 int32 (HierarchyNode). */
int hlgs_dhier_load(const char* path, float* pos, float* rot, float* log_scales, float* opacities, float* shs,
                    int* nodes);
/* WriteDynamicHierarchy (torch_interface.cpp:107-133): shs G x (deg+1)^2 x 3, nodes N x 6. */
int hlgs_dhier_write(const char* path, int G, int N, const float* pos, const float* shs, const float* opacities,
                     const float* log_scales, const float* rot, const int* nodes, int sh_degree);
/* ExpandToTarget (torch_interface.cpp:136-146, traversal.cpp:15-39): Gaussian indices of the cut at node depth
 * `target` over N static Nodes (host).  Writes min(count, capacity) entries to out (may be NULL to query). */
int hlgs_expand_to_target(int N, const int* nodes, int target, int* out, int capacity, int* count);

/* ---- inspection (tests): byte offsets of fields inside the caller's buffers, counted from the
 * buffer's first 256-byte-aligned address ---- */
size_t hlgs_binning_point_list_offset(int R);  /* uint32 point_list[R] */
/* point_list entries of a P-Gaussian forward started now are (Gaussian index << shift) | footprint quadrant mask: the
 * shift (a finished frame's own is hlgs_frame_info.entry_shift). */
int hlgs_point_list_entry_shift(int P);
/* The process-wide switches below are atomics, read once when a frame starts: a frame in flight keeps the options it
 * started with (reported in its hlgs_frame_info), so flipping a switch from another thread changes later frames only.
 * 1 if a P-Gaussian forward started now bins no instance whose quadrant mask is 0 (packed entries, dropping on): its tile
 * lists and n_contrib then match the oracle run with drop_empty (oracle/hlgs_oracle.c rect_quad_masks).  0: every
 * instance of the reference's binning (rasterizer_impl.cu:70-115) is listed, and point_list / n_contrib are laid out as
 * the reference lays them out. */
int hlgs_point_list_drops_empty(int P);
/* Tests: on = 0 makes every following frame use plain index entries (the P >= 2^28 path); 1 restores the default. */
void hlgs_set_entry_packing(int on);
/* on = 0: following frames bin every instance, including those whose footprint reaches none of their tile's quadrants
 * (the reference's tile lists and n_contrib; images and gradients are the same either way); 1 (default) drops them. */
void hlgs_set_drop_empty(int on);
/* Tests: the bound on each look-back poll of the fused binning plan (default 2^20 polls, ~0.1 s).  A plan whose
 * look-back times out is re-run with the two-launch plan that needs no inter-block wait; polls = 0 forces that path. */
void hlgs_set_plan_polls(unsigned polls);
size_t hlgs_image_ranges_offset(int W, int H);  /* uint2 ranges[tiles] */
/* uint32 misc[16]: [0] binned instances, [1] longest tile list, [2] record slots, [3] the frame's entry packing (1 when
 * entry_shift != 0), [4] the frame's drops_empty -- written on the device by the frame's binning plan */
size_t hlgs_image_misc_offset(int W, int H);
size_t hlgs_geom_splat_offset(int P);           /* float4 splat[P][4]: x, y, conic a, b | conic c, opacity, r, g |
                                                   b, 1/depth, t, 1/kids | record base, tile x0, y0, width */

/* ---- measurement hooks (bench.py) ---- */
/* Stage timing: every launch of each selected rasterizer stage (bit i of mask = stage i, -1 = all,
 * 0 = off) is bracketed by hipEvents on its launch stream.  hlgs_stage_stats returns, per stage, the
 * mean duration in ms over all launches recorded since the last hlgs_set_stage_timing call and the
 * number of launches (synchronises).  Off by default. */
void hlgs_set_stage_timing(int mask);
int hlgs_stage_count(void);
const char* hlgs_stage_name(int i);
int hlgs_stage_stats(float* mean_ms, int* calls, int max);

#ifdef __cplusplus
}
#endif
#endif
