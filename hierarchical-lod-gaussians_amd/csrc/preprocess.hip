// preprocess.hip -- the forward's per-Gaussian preprocess for gfx950.
//
// Reference semantics (submodules/hierarchy-rasterizer/cuda_rasterizer):
//   k_preprocess, k_preprocess_sh2  <- preprocessCUDA<3>   forward.cu:218-445
//                                      (+ per-tile instance counting for the generic binning path)
// Built with -ffp-contract=off (hlgs_core/build.py PER_FILE): every per-Gaussian value the blends read is computed in
// the oracle's operation order without contraction, so the splat records are bitwise equal to the oracle's
// (the shared arithmetic contract).
#include "hlgs_internal.h"
#include "hlgs_math.h"

namespace hlgs {

// ------------------------------------------------------------------------------------------------
// Preprocess: one thread per rasterised Gaussian.
// ------------------------------------------------------------------------------------------------
template <bool HIER, bool ALT>
__global__ void __launch_bounds__(256) k_preprocess(hlgs_raster_args a, Geom g, int* __restrict__ radii,
                                                    uint32_t* __restrict__ tile_count, int gx, int gy, float fx,
                                                    float fy, ZeroJob z)
{
    const int t_idx = blockIdx.x * 256 + threadIdx.x;
    zero_prelude(z, t_idx, gridDim.x * 256);
    if (t_idx >= a.P) return;
    const int r_idx = HIER ? a.indices[t_idx] : t_idx;
    radii[t_idx] = 0;
    g.tiles_touched[t_idx] = 0;
    g.rects[t_idx] = make_int2(0, 0);
    g.clamped[t_idx] = 0;

    bool use_parent = false;
    int p_idx = 0;
    float t = 0.f;
    f3 p_orig = mk(a.means3D[3 * r_idx], a.means3D[3 * r_idx + 1], a.means3D[3 * r_idx + 2]);
    if (HIER) {
        p_idx = a.parent_indices[t_idx];
        if (p_idx != -1) { use_parent = true; t = a.ts[t_idx]; }
        else p_idx = 0;
        if (use_parent) {
            f3 pa = mk(a.means3D[3 * p_idx], a.means3D[3 * p_idx + 1], a.means3D[3 * p_idx + 2]);
            p_orig = mk(t * p_orig.x + (1.0f - t) * pa.x, t * p_orig.y + (1.0f - t) * pa.y,
                        t * p_orig.z + (1.0f - t) * pa.z);
        }
    }
    const float* proj = a.projmatrix;
    const float* view = a.viewmatrix;
    float hx = proj[0] * p_orig.x + proj[4] * p_orig.y + proj[8] * p_orig.z + proj[12];
    float hy = proj[1] * p_orig.x + proj[5] * p_orig.y + proj[9] * p_orig.z + proj[13];
    float hw = xform44w(p_orig, proj);
    float p_w = 1.0f / (hw + 0.0000001f);
    float ppx = hx * p_w, ppy = hy * p_w;
    f3 p_view = xform43(p_orig, view);
    if (p_view.z <= 0.2f) return;

    float c3[6];
    const float* cov3D;
    if (a.cov3D_precomp == nullptr) {
        f3 scale = mk(a.scales[3 * r_idx], a.scales[3 * r_idx + 1], a.scales[3 * r_idx + 2]);
        float4 rq = reinterpret_cast<const float4*>(a.rotations)[r_idx];
        float rot[4] = {rq.x, rq.y, rq.z, rq.w};
        if (HIER && use_parent) {
            f3 ps = mk(a.scales[3 * p_idx], a.scales[3 * p_idx + 1], a.scales[3 * p_idx + 2]);
            scale = add(scl(t, scale), scl(1.0f - t, ps));
            float4 oq = reinterpret_cast<const float4*>(a.rotations)[p_idx];
            float orot[4] = {oq.x, oq.y, oq.z, oq.w};
            float dp = rot[0] * orot[0] + rot[1] * orot[1] + rot[2] * orot[2] + rot[3] * orot[3];
            if (dp < 0.0f)
                for (int i = 0; i < 4; i++) orot[i] = -orot[i];
            for (int i = 0; i < 4; i++) rot[i] = t * rot[i] + (1.0f - t) * orot[i];
        }
        cov3d_fwd(scale, a.scale_modifier, rot, c3);
        cov3D = c3;
    } else {
        // the reference leaves cov3D unassigned here; we take the evident intent.
        for (int i = 0; i < 6; i++) c3[i] = a.cov3D_precomp[6 * t_idx + i];
        cov3D = c3;
    }
    if (HIER) {  // the hierarchy-mode backward reads the lerped covariance; otherwise k_gauss_bwd recomputes it
        float2* c3o = reinterpret_cast<float2*>(g.cov3D + 6 * (size_t)t_idx);
        c3o[0] = make_float2(c3[0], c3[1]);
        c3o[1] = make_float2(c3[2], c3[3]);
        c3o[2] = make_float2(c3[4], c3[5]);
    }

    Cov2D k;
    cov2d_eval(p_orig, fx, fy, a.tanfovx, a.tanfovy, cov3D, view, k);
    float cx = k.cov.m[0][0], cy = k.cov.m[0][1], cz = k.cov.m[1][1];
    const float h_var = 0.3f;
    const float det_cov = cx * cz - cy * cy;
    cx += h_var;
    cz += h_var;
    const float det_h = cx * cz - cy * cy;
    float h_scale = sqrtf(fmaxf(0.000025f, det_cov / det_h));
    constexpr bool alt = ALT;
    if (alt && !a.antialiasing) h_scale = 1.0f;  // alt-rasterizer forward.cu:226-229
    const float det = det_h;
    if (det == 0.0f) return;
    const float det_inv = 1.f / det;
    const float conic_x = cz * det_inv, conic_y = -cy * det_inv, conic_z = cx * det_inv;
    const float mid = 0.5f * (cx + cz);
    const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    const float my_radius = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
    const float pix_x = ndc2pix(ppx, a.W), pix_y = ndc2pix(ppy, a.H);
    // per-axis 3-sigma rect (forward.cu:398-403); the alt rasterizer bins the eigen-radius square (its
    // forward.cu:249), whose tiles it then culls exactly (alt_tile_keep)
    const int ex = alt ? (int)my_radius : (int)ceilf(3.f * sqrtf(cx));
    const int ey = alt ? (int)my_radius : (int)ceilf(3.f * sqrtf(cz));
    g.rects[t_idx] = make_int2(ex, ey);
    int x0, y0, x1, y1;
    tile_rect(pix_x, pix_y, ex, ey, gx, gy, x0, y0, x1, y1);
    const uint32_t area = (uint32_t)(x1 - x0) * (uint32_t)(y1 - y0);
    if (area == 0) return;

    f3 col;
    if (a.colors_precomp) {
        col = mk(a.colors_precomp[3 * t_idx], a.colors_precomp[3 * t_idx + 1], a.colors_precomp[3 * t_idx + 2]);
    } else {
        const f3 campos = mk(a.campos[0], a.campos[1], a.campos[2]);
        const f3 mean_r = mk(a.means3D[3 * r_idx], a.means3D[3 * r_idx + 1], a.means3D[3 * r_idx + 2]);
        const float* sc = a.shs + (size_t)r_idx * a.M * 3;
        uint32_t cb = 0;
        f3 rgb;
        if (alt) {
            // alt-rasterizer forward.cu:23-75: coefficient 0 from dc, coefficient c >= 1 from shs[c - 1]
            const float* d0 = a.dc + 3 * (size_t)r_idx;
            rgb = sh_to_rgb(a.D, [&](int c) {
                return c == 0 ? mk(d0[0], d0[1], d0[2]) : mk(sc[3 * c - 3], sc[3 * c - 2], sc[3 * c - 1]);
            }, mean_r, campos, cb);
        } else if (!(HIER && use_parent)) {
            rgb = sh_to_rgb(a.D, [&](int c) { return mk(sc[3 * c], sc[3 * c + 1], sc[3 * c + 2]); }, mean_r, campos, cb);
        } else {
            // forward.cu:86-138: every coefficient lerped child<->parent, view direction from the child
            const float* sp = a.shs + (size_t)p_idx * a.M * 3;
            const float tt = t;
            rgb = sh_to_rgb(a.D, [&](int c) {
                return mk(tt * sc[3 * c] + (1.0f - tt) * sp[3 * c], tt * sc[3 * c + 1] + (1.0f - tt) * sp[3 * c + 1],
                          tt * sc[3 * c + 2] + (1.0f - tt) * sp[3 * c + 2]);
            }, mean_r, campos, cb);
        }
        g.clamped[t_idx] = cb;
        col = rgb;
    }
    g.depths[t_idx] = p_view.z;
    radii[t_idx] = (int)my_radius;
    g.means2D[t_idx] = make_float2(pix_x, pix_y);
    float opacity = a.opacities[r_idx];
    if (HIER && use_parent) opacity = t * opacity + (1.0f - t) * a.opacities[p_idx];
    g.tiles_touched[t_idx] = area;
    uint32_t masks = 0xFFFFFFFFu;
    {
        const float cr = col.x, cg = col.y, cbl = col.z;
        const bool interp = a.ts && a.kids;
        float4* rec = g.splat + 4 * (size_t)t_idx;
        rec[0] = make_float4(pix_x, pix_y, conic_x, conic_y);
        rec[1] = make_float4(conic_z, opacity * h_scale, cr, cg);
        const float tt = interp ? a.ts[t_idx] : 0.f, fr = interp ? 1.0f / (float)a.kids[t_idx] : 0.f;
        rec[2] = make_float4(cbl, 1.f / p_view.z, tt, fr);
        const float thr = alpha_e2_threshold(opacity * h_scale, interp, tt, fr);
        if (g.pack)
            masks = rect_quad_masks(pix_x, pix_y, make_float4(conic_x, conic_y, conic_z, opacity * h_scale), thr, x0, y0,
                                    x1, y1);
        if (g.pack) g.qmask[t_idx] = masks;
        rec[3] = make_float4(0.f, __int_as_float(x0 | (y0 << 16)), __int_as_float(x1 - x0), thr);
    }
    if (tile_count) {  // only when the tile grid is too large for the LDS-histogram binning
        const float4 co = make_float4(conic_x, conic_y, conic_z, opacity * h_scale);
        const AltKeep kthr = alt ? alt_keep_prep(co) : AltKeep{0.f, 0.f, 0.f};
        uint32_t r = 0;
        for (int y = y0; y < y1; y++)
            for (int x = x0; x < x1; x++, r++)
                if ((!alt || alt_tile_keep(pix_x, pix_y, co, kthr, x, y)) &&
                    !(g.drop && !rect_tile_mask(masks, r)))
                    atomicAdd(&tile_count[y * gx + x], 1u);
    }
}

// ------------------------------------------------------------------------------------------------
// Preprocess, common path (no hierarchy indices, SH coefficients given): k_preprocess_sh2 below.
// The geometry is per thread as in k_preprocess; the block's SH rows are copied into LDS with all 64 lanes on
// consecutive float4s, so the 192-byte SH rows (M = 16) stream from HBM in whole lines instead of 48 strided
// 4-byte loads per thread.  Every per-Gaussian output is bit-identical to k_preprocess (same arithmetic, same order).
// ------------------------------------------------------------------------------------------------
struct PreGeom {
    float pix_x, pix_y, depth, conic_x, conic_y, conic_z, h_scale, radius;
    int x0, y0, x1, y1;
    int ex, ey;  // the per-axis rect extents (Geom::rects); 0 when culled before they are formed
};

// The per-Gaussian inputs of the geometry, all loaded before the kernel's first global store: a load that follows a
// store waits for it too (vmcnt counts both), and the uniform camera matrices only go through the scalar path when no
// store in the kernel can precede them.
struct PreIn {
    f3 mean, scale;
    float4 rq;
    float opacity;
};

__device__ __forceinline__ PreIn preprocess_load(const hlgs_raster_args& a, int t_idx)
{
    PreIn in;
    in.opacity = a.opacities[t_idx];
    in.mean = mk(a.means3D[3 * t_idx], a.means3D[3 * t_idx + 1], a.means3D[3 * t_idx + 2]);
    in.scale = mk(0.f, 0.f, 0.f);
    in.rq = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.cov3D_precomp == nullptr) {
        in.scale = mk(a.scales[3 * t_idx], a.scales[3 * t_idx + 1], a.scales[3 * t_idx + 2]);
        in.rq = reinterpret_cast<const float4*>(a.rotations)[t_idx];
    }
    // pinned here, so all of them share one round trip (the compiler would sink scale and rotation below the
    // near-plane test, a second dependent round trip)
    asm volatile("" : "+v"(in.mean.x), "+v"(in.mean.y), "+v"(in.mean.z), "+v"(in.scale.x), "+v"(in.scale.y),
                 "+v"(in.scale.z), "+v"(in.opacity));
    asm volatile("" : "+v"(in.rq.x), "+v"(in.rq.y), "+v"(in.rq.z), "+v"(in.rq.w));
    return in;
}

// forward.cu:218-403 up to the colour; false = culled.  Stores nothing (the caller writes every output once).
template <bool ALT>
__device__ __forceinline__ bool preprocess_geom(const hlgs_raster_args& a, const PreIn& in, const float (&proj)[16],
                                                const float (&view)[16], int t_idx, int gx, int gy, float fx, float fy,
                                                PreGeom& o)
{
    o.ex = o.ey = 0;
    const f3 p_orig = in.mean;
    const float hx = proj[0] * p_orig.x + proj[4] * p_orig.y + proj[8] * p_orig.z + proj[12];
    const float hy = proj[1] * p_orig.x + proj[5] * p_orig.y + proj[9] * p_orig.z + proj[13];
    const float hw = xform44w(p_orig, proj);
    const float p_w = 1.0f / (hw + 0.0000001f);
    const float ppx = hx * p_w, ppy = hy * p_w;
    const f3 p_view = xform43(p_orig, view);
    if (p_view.z <= 0.2f) return false;
    float c3[6];
    if (a.cov3D_precomp == nullptr) {
        const float rot[4] = {in.rq.x, in.rq.y, in.rq.z, in.rq.w};
        cov3d_fwd(in.scale, a.scale_modifier, rot, c3);
    } else {
        for (int i = 0; i < 6; i++) c3[i] = a.cov3D_precomp[6 * t_idx + i];
    }
    // cov3D is not stored: k_gauss_bwd recomputes it bit-identically (cov3d_exact), 24 bytes per Gaussian saved
    // on each side
    Cov2D k;
    cov2d_eval(p_orig, fx, fy, a.tanfovx, a.tanfovy, c3, view, k);
    float cx = k.cov.m[0][0], cy = k.cov.m[0][1], cz = k.cov.m[1][1];
    const float h_var = 0.3f;
    const float det_cov = cx * cz - cy * cy;
    cx += h_var;
    cz += h_var;
    const float det_h = cx * cz - cy * cy;
    o.h_scale = sqrtf(fmaxf(0.000025f, det_cov / det_h));
    if (ALT && !a.antialiasing) o.h_scale = 1.0f;
    const float det = det_h;
    if (det == 0.0f) return false;
    const float det_inv = 1.f / det;
    o.conic_x = cz * det_inv;
    o.conic_y = -cy * det_inv;
    o.conic_z = cx * det_inv;
    const float mid = 0.5f * (cx + cz);
    const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    o.radius = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
    o.pix_x = ndc2pix(ppx, a.W);
    o.pix_y = ndc2pix(ppy, a.H);
    o.ex = ALT ? (int)o.radius : (int)ceilf(3.f * sqrtf(cx));
    o.ey = ALT ? (int)o.radius : (int)ceilf(3.f * sqrtf(cz));
    tile_rect(o.pix_x, o.pix_y, o.ex, o.ey, gx, gy, o.x0, o.y0, o.x1, o.y1);
    o.depth = p_view.z;
    return (uint32_t)(o.x1 - o.x0) * (uint32_t)(o.y1 - o.y0) != 0;
}

// Two waves per 64 Gaussians: wave 0 runs the geometry while wave 1 streams the block's 64 SH rows (contiguous in
// the AoS input, culled rows included) into LDS; after a barrier wave 1 evaluates the colour and the direction
// Jacobian from LDS while wave 0 classifies the footprint quadrants, and after a second barrier wave 0 writes the
// records.  The SH rows' HBM latency overlaps the geometry instead of following it, and one 12 KB LDS stage keeps two
// waves busy.  Same arithmetic, same outputs.
// The rows arrive through registers: every lane loads consecutive float4s of the block's contiguous rows (1 KiB per
// wave instruction) and stores them into LDS rows of odd stride (kShStride), so that each lane's own row walk hits
// distinct banks; degree-3 rows use the unpadded swizzled float4 layout of sh_rows_load_swz below instead.  (Round 5 measured LDS-DMA into a chunk-major image instead -- conflict-free b128 reads, no staging
// registers: 115 against 97 us, because the DMA's source side then reads 16 bytes per lane at the row stride, 64 lines
// per wave instruction instead of 8; preprocess_dma.hip, tools/variants/INDEX.md.)
template <int M3T>
__device__ __forceinline__ void sh_rows_load_contig(const float* gbase, float* lds, int n, int lane, int m3)
{
    if constexpr (M3T > 0 && M3T % 4 == 0) {
        constexpr int Q = M3T / 4;
        float4 v[Q];
#pragma unroll
        for (int k = 0; k < Q; k++) {
            const int f = lane + 64 * k;
            v[k] = f < n * Q ? reinterpret_cast<const float4*>(gbase)[f] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int k = 0; k < Q; k++) {
            const int f = lane + 64 * k;
            if (f < n * Q) {
                const int r = f / Q, q = f - r * Q;
                float* lp = lds + r * kShStride + 4 * q;
                lp[0] = v[k].x; lp[1] = v[k].y; lp[2] = v[k].z; lp[3] = v[k].w;
            }
        }
    } else {
        const int M3 = M3T ? M3T : m3;
        for (int f = lane; f < n * M3; f += 64) {
            const int r = f / M3, q = f - r * M3;
            lds[r * kShStride + q] = gbase[f];
        }
    }
}

// Degree-3 rows (48 floats, 12 float4s) are staged unpadded, float4 q of row r at slot 12 r + (q ^ sh_swz(r)): the
// staging stores (ds_write_b128, 8-lane groups), each lane's reads of its own row (ds_read_b128, 16-lane groups) and
// a copy back out all hit distinct banks, where the odd 49-float stride takes four b32 stores and four b32 reads per
// float4 with two-way store conflicts (a fifth of the kernel's LDS cycles were conflict cycles).
__device__ __forceinline__ int sh_swz(int r) { return (r >> 2) & 3; }
__device__ __forceinline__ void sh_rows_load_swz(const float* gbase, float* lds, int n, int lane)
{
    float4 v[12];
#pragma unroll
    for (int k = 0; k < 12; k++) {
        const int f = lane + 64 * k;
        v[k] = f < n * 12 ? reinterpret_cast<const float4*>(gbase)[f] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < 12; k++) {
        const int f = lane + 64 * k;
        if (f < n * 12) {
            const int r = f / 12, q = f - r * 12;
            reinterpret_cast<float4*>(lds)[12 * r + (q ^ sh_swz(r))] = v[k];
        }
    }
}

template <bool ALT, int M3T, bool INTERP>  // INTERP = a.ts && a.kids, host-dispatched: its threshold bisection in
                                          // double would otherwise set the register budget (90 VGPRs against 67)
__global__ void __launch_bounds__(128) k_preprocess_sh2(hlgs_raster_args a, Geom g, int* __restrict__ radii, int gx,
                                                        int gy, float fx, float fy, ZeroJob z)
{
    constexpr bool SWZ = M3T == 48;           // degree-3 rows: unpadded, swizzled float4 slots (sh_rows_load_swz)
    __shared__ __attribute__((aligned(16))) float s_rows[64 * (SWZ ? 48 : kShStride)];  // the SH rows; after the
                                                                                         // second barrier the records' stage
    __shared__ float4 s_col[64];              // r, g, b, clamp bits
    __shared__ int s_need[64];
    __shared__ float s_jac[64 * 9];           // the direction Jacobians' stage
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t0 = blockIdx.x * 64, t_idx = t0 + lane;
    const int n_grp = min(64, a.P - t0);      // Gaussians of this block
    const int M3 = 3 * a.M;
    const bool live = t_idx < a.P;
    PreGeom o;
    bool need = false;
    f3 mean_r = mk(0.f, 0.f, 0.f), dc0 = mk(0.f, 0.f, 0.f);
    PreIn in{};
    if (wave == 0) {
        float proj[16], view[16];
#pragma unroll
        for (int i = 0; i < 16; i++) {
            proj[i] = a.projmatrix[i];
            view[i] = a.viewmatrix[i];
        }
        if (live) in = preprocess_load(a, t_idx);
        need = live && preprocess_geom<ALT>(a, in, proj, view, t_idx, gx, gy, fx, fy, o);
        s_need[lane] = need;
    } else {
        const int n = min(64, a.P - t0);
        if constexpr (SWZ) sh_rows_load_swz(a.shs + (size_t)t0 * M3, s_rows, n, lane);
        else sh_rows_load_contig<M3T>(a.shs + (size_t)t0 * M3, s_rows, n, lane, M3);
        // the colour's own inputs in the same round trip as the rows (not behind the barrier)
        if (live) {
            mean_r = mk(a.means3D[3 * t_idx], a.means3D[3 * t_idx + 1], a.means3D[3 * t_idx + 2]);
            if (ALT) dc0 = mk(a.dc[3 * (size_t)t_idx], a.dc[3 * (size_t)t_idx + 1], a.dc[3 * (size_t)t_idx + 2]);
        }
    }
    __syncthreads();
    const f3 campos = mk(a.campos[0], a.campos[1], a.campos[2]);
    constexpr bool interp = INTERP;
    float thr = 0.f;
    const float opacity = in.opacity;
    if (wave == 1) {
        float* sj = s_jac + 9 * lane;  // odd stride: the 64 lanes' 4-byte writes hit distinct banks
        if (s_need[lane]) {
            // coefficient c of this lane's row (the full index: the alt rasterizer's 0 is dc)
            const float* row = s_rows + lane * kShStride;
            float rv[SWZ ? 48 : 1];  // SWZ: the lane's whole row, twelve ds_read_b128
            if constexpr (SWZ) {
                const float4* r4 = reinterpret_cast<const float4*>(s_rows) + 12 * lane;
                const int sw = sh_swz(lane);
#pragma unroll
                for (int j = 0; j < 12; j++) {
                    const float4 t = r4[(j & ~3) | ((j & 3) ^ sw)];
                    rv[4 * j] = t.x; rv[4 * j + 1] = t.y; rv[4 * j + 2] = t.z; rv[4 * j + 3] = t.w;
                }
            }
            auto rowf = [&](int f) -> float {
                if constexpr (SWZ) return rv[f];
                else return row[f];
            };
            auto shv = [&](int c) {
                if (ALT) return c == 0 ? dc0 : mk(rowf(3 * c - 3), rowf(3 * c - 2), rowf(3 * c - 1));
                return mk(rowf(3 * c), rowf(3 * c + 1), rowf(3 * c + 2));
            };
            uint32_t cb = 0;
            const f3 col = sh_to_rgb(a.D, shv, mean_r, campos, cb);
            s_col[lane] = make_float4(col.x, col.y, col.z, __uint_as_float(cb));
            {  // d colour / d view direction for the SH backward (Geom::sh_jac), from the coefficients in LDS
                const f3 d = sub(mean_r, campos);
                const float len = sqrtf(dot(d, d));
                f3 jx, jy, jz;
                sh_dir_jacobian(a.D, shv, d.x / len, d.y / len, d.z / len, jx, jy, jz);
                sj[0] = jx.x; sj[1] = jx.y; sj[2] = jx.z;
                sj[3] = jy.x; sj[4] = jy.y; sj[5] = jy.z;
                sj[6] = jz.x; sj[7] = jz.y; sj[8] = jz.z;
            }
        } else {
            for (int k = 0; k < 9; k++) sj[k] = 0.f;
        }
        // the block's Jacobians are contiguous in Geom::sh_jac: stored from the stage as whole float4s (the rows are
        // 36 bytes, so per-lane stores would write every line in pieces)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's own stage writes, before its reads
        {
            const int nf = 9 * n_grp;
            float* jb = g.sh_jac + 9 * (size_t)t0;  // 16-byte aligned: t0 is a multiple of 64
            for (int f4 = lane; 4 * f4 < nf; f4 += 64) {
                if (4 * f4 + 3 < nf) {
                    reinterpret_cast<float4*>(jb)[f4] = reinterpret_cast<const float4*>(s_jac)[f4];
                } else {
                    for (int e = 4 * f4; e < nf; e++) jb[e] = s_jac[e];
                }
            }
        }
        // the zeroing the next stages need (after this wave's loads, so no load waits for these stores)
        zero_prelude(z, t_idx, gridDim.x * 64);
    } else if (need) {
        const float tt = interp ? a.ts[t_idx] : 0.f, fr = interp ? 1.0f / (float)a.kids[t_idx] : 0.f;
        thr = alpha_e2_threshold(opacity * o.h_scale, interp, tt, fr);
        if (g.pack)
            g.qmask[t_idx] = rect_quad_masks(o.pix_x, o.pix_y, make_float4(o.conic_x, o.conic_y, o.conic_z,
                                                                           opacity * o.h_scale), thr, o.x0, o.y0, o.x1, o.y1);
    }
    __syncthreads();
    if (wave == 1) return;
    // the block's splat records through a stage (the row buffer, free now), stored as contiguous float4s: 4 KiB in
    // four 1 KiB wave instructions instead of four 16-byte pieces of every lane's 64-byte record (a culled Gaussian's
    // record is written as zeros; nothing reads it)
    float4* st = reinterpret_cast<float4*>(s_rows);
    float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0, r2 = r0, r3 = r0;
    if (live) {
        g.rects[t_idx] = make_int2(o.ex, o.ey);
        if (!need) {  // culled: the zero outputs (rects as far as they were formed, forward.cu:398-403)
            radii[t_idx] = 0;
            g.tiles_touched[t_idx] = 0;
            g.clamped[t_idx] = 0;
        } else {
            const float4 c = s_col[lane];
            g.clamped[t_idx] = __float_as_uint(c.w);
            g.depths[t_idx] = o.depth;
            radii[t_idx] = (int)o.radius;
            g.means2D[t_idx] = make_float2(o.pix_x, o.pix_y);
            g.tiles_touched[t_idx] = (uint32_t)(o.x1 - o.x0) * (uint32_t)(o.y1 - o.y0);
            const float tt = interp ? a.ts[t_idx] : 0.f, fr = interp ? 1.0f / (float)a.kids[t_idx] : 0.f;
            r0 = make_float4(o.pix_x, o.pix_y, o.conic_x, o.conic_y);
            r1 = make_float4(o.conic_z, opacity * o.h_scale, c.x, c.y);
            r2 = make_float4(c.z, 1.f / o.depth, tt, fr);
            r3 = make_float4(0.f, __int_as_float(o.x0 | (o.y0 << 16)), __int_as_float(o.x1 - o.x0), thr);
        }
    }
    // Word k of lane l's record goes to slot (k + l / 2) mod 4 of its 64-byte stage row: each ds_write_b128 group of 8
    // consecutive lanes then covers all 32 banks once (unrotated, lanes 0, 2, 4, 6 all hit banks 0-3: 4-way conflicts,
    // half of the kernel's SQ_LDS_BANK_CONFLICT cycles).  The reads stay linear (conflict-free); the global store puts
    // each word back in place within the same record, so every wave store still covers contiguous 1 KiB.
    const int rot = lane >> 1;
    st[4 * lane + (rot & 3)] = r0;
    st[4 * lane + ((rot + 1) & 3)] = r1;
    st[4 * lane + ((rot + 2) & 3)] = r2;
    st[4 * lane + ((rot + 3) & 3)] = r3;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's own stage writes, before its reads
    float4* rb = g.splat + 4 * (size_t)t0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int f4 = 64 * k + lane, rec = f4 >> 2;
        if (f4 < 4 * n_grp) rb[4 * rec + (((f4 & 3) - (rec >> 1)) & 3)] = st[f4];
    }
}

void launch_preprocess(const hlgs_raster_args& a, const Geom& g, int* radii, uint32_t* tile_count, int gx, int gy,
                       const ZeroJob& z, hipStream_t s)
{
    const float fy = a.H / (2.0f * a.tanfovy);
    const float fx = a.W / (2.0f * a.tanfovx);
    const dim3 grid((a.P + 255) / 256);
    const bool alt = a.variant == HLGS_VARIANT_ALT;
    if (!a.indices && !a.colors_precomp && a.shs && a.M > 0 && !tile_count && a.M <= 16) {
        const dim3 g64((a.P + 63) / 64);
#define HLGS_PSH(AL, M3)                                                                                              \
    do {                                                                                                              \
        if (a.ts && a.kids)                                                                                           \
            hipLaunchKernelGGL((k_preprocess_sh2<AL, M3, true>), g64, dim3(128), 0, s, a, g, radii, gx, gy, fx, fy, z); \
        else                                                                                                          \
            hipLaunchKernelGGL((k_preprocess_sh2<AL, M3, false>), g64, dim3(128), 0, s, a, g, radii, gx, gy, fx, fy,   \
                               z);                                                                                    \
    } while (0)
        if (alt) {
            switch (a.M) {
            case 3: HLGS_PSH(true, 9); break;
            case 8: HLGS_PSH(true, 24); break;
            case 15: HLGS_PSH(true, 45); break;
            default: HLGS_PSH(true, 0); break;
            }
        } else {
            switch (a.M) {
            case 1: HLGS_PSH(false, 3); break;
            case 4: HLGS_PSH(false, 12); break;
            case 9: HLGS_PSH(false, 27); break;
            case 16: HLGS_PSH(false, 48); break;
            default: HLGS_PSH(false, 0); break;
            }
        }
#undef HLGS_PSH
        return;
    }
    if (a.indices)
        hipLaunchKernelGGL((k_preprocess<true, false>), grid, dim3(256), 0, s, a, g, radii, tile_count, gx, gy, fx, fy, z);
    else if (a.variant == HLGS_VARIANT_ALT)
        hipLaunchKernelGGL((k_preprocess<false, true>), grid, dim3(256), 0, s, a, g, radii, tile_count, gx, gy, fx, fy, z);
    else
        hipLaunchKernelGGL((k_preprocess<false, false>), grid, dim3(256), 0, s, a, g, radii, tile_count, gx, gy, fx, fy, z);
}

}  // namespace hlgs
