/*
 * hlgs_oracle.c -- CPU restatement of the reference hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or as the CPU baseline).  The product path (libhlgs.so) never calls it.
 *
 * Every function restates the algorithm of the reference CUDA sources
 * (FelixWindisch/hierarchical-LOD-gaussians, mounted read-only at
 * /root/reference) in plain, serial, single-threaded C with float32
 * arithmetic.  Citations are path:line relative to that tree:
 *   HR = submodules/hierarchy-rasterizer/cuda_rasterizer
 *   GH = submodules/gaussianhierarchy
 *
 * Parity status: the SH evaluation and camera conventions are pinned against
 * the reference's own importable Python helpers (utils/sh_utils.eval_sh,
 * utils/graphics_utils) by tests/golden fixtures; the backward formulas are
 * pinned against a float64 torch-autograd restatement (tests/test_oracle.py).
 * The reference ships no golden vectors for the rasterizer itself, so the
 * blend/binning stages are a line-faithful restatement ("partially pinned").
 *
 * glm conventions are reproduced: mat3 is column-major, m[c][r] = column c,
 * row r, and products are summed in glm's order.
 */
#include <math.h>
#include <float.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* The same source also builds the all-cores CPU baseline (oracle/build/libhlgs_oracle_omp.so, gcc -fopenmp):
 * preprocess and per-Gaussian backward over Gaussians, the blend and the blend backward over tiles, per-tile sorts
 * in parallel.  The blend backward sums each (tile, Gaussian) pair's contributions over the tile's pixels into a
 * record of its own (tile_records), and the records are added per Gaussian in tile order afterwards, serially: the
 * reference adds its per-pixel contributions with float atomics in no fixed order (HR/backward.cu:669-718), and this
 * fixed order makes the OpenMP build bitwise equal to the serial one (tests/test_oracle.py), so it can stand in for
 * it on full-size frames. */


/* Alpha decision mode:
 *   0 (default) -- the shared arithmetic contract (A-17): e2 = power log2(e) from the pre-scaled conic, G = exp2(e2),
 *                  keep iff e2 >= the per-Gaussian threshold computed in double; bit-identical to the HIP kernels;
 *   1           -- the reference's own float operation order: power = -0.5f (a dx dx + c dy dy) - b dx dy,
 *                  G = expf(power), keep iff alpha >= 1.0f / 255.0f (HR/forward.cu:538-560,
 *                  HR/backward.cu:614-643, AR/forward.cu:383-391, AR/backward.cu:594-600), evaluated without FMA
 *                  contraction.  Reported beside the contract so that divergence from the reference's float
 *                  behaviour stays visible. */
static int g_ref_order = 0;
void orc_set_alpha_mode(int reference_order) { g_ref_order = reference_order != 0; }
int orc_get_alpha_mode(void) { return g_ref_order; }
int orc_num_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

#define TILE 16
#define NCH 3

/* SH constants, HR/auxiliary.h:34-51 */
static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

typedef struct { float x, y, z; } v3;
typedef struct { float m[3][3]; } m3; /* m[col][row] */

static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vscale(float s, v3 a) { return V3(s * a.x, s * a.y, s * a.z); }
static inline float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

/* glm operator*(mat3, mat3): r[c][row] = a[0][row]*b[c][0] + a[1][row]*b[c][1] + a[2][row]*b[c][2] */
static m3 mmul(m3 a, m3 b)
{
    m3 r;
    for (int c = 0; c < 3; c++)
        for (int row = 0; row < 3; row++)
            r.m[c][row] = a.m[0][row] * b.m[c][0] + a.m[1][row] * b.m[c][1] + a.m[2][row] * b.m[c][2];
    return r;
}
static m3 mtrans(m3 a)
{
    m3 r;
    for (int c = 0; c < 3; c++)
        for (int row = 0; row < 3; row++) r.m[c][row] = a.m[row][c];
    return r;
}
/* glm::mat3(a0..a8): columns (a0,a1,a2), (a3,a4,a5), (a6,a7,a8) */
static m3 mcols(float a0, float a1, float a2, float a3, float a4, float a5, float a6, float a7, float a8)
{
    m3 r;
    r.m[0][0] = a0; r.m[0][1] = a1; r.m[0][2] = a2;
    r.m[1][0] = a3; r.m[1][1] = a4; r.m[1][2] = a5;
    r.m[2][0] = a6; r.m[2][1] = a7; r.m[2][2] = a8;
    return r;
}

/* HR/auxiliary.h:53-56 -- evaluated in double, as the reference does */
static inline float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }

/* HR/auxiliary.h:83-102 */
static inline v3 xform43(v3 p, const float *m)
{
    return V3(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
              m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}
static inline void xform44(v3 p, const float *m, float out[4])
{
    out[0] = m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12];
    out[1] = m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13];
    out[2] = m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14];
    out[3] = m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15];
}

static inline int imin(int a, int b) { return a < b ? a : b; }
/* float -> int32 with the GPU's saturating, NaN -> 0 conversion (cvt.rzi.s32.f32 / v_cvt_i32_f32) */
static inline int f2i(float f)
{
    if (f != f) return 0;
    if (f >= 2147483647.0f) return 2147483647;
    if (f <= -2147483648.0f) return (-2147483647 - 1);
    return (int)f;
}
static inline int imax(int a, int b) { return a > b ? a : b; }

/* HR/auxiliary.h:70-80 (rect variant; the torch path always passes rects) */
static void get_rect(float px, float py, int ex, int ey, int gx, int gy, int *x0, int *y0, int *x1, int *y1)
{
    *x0 = imin(gx, imax(0, f2i((px - ex) / TILE)));
    *y0 = imin(gy, imax(0, f2i((py - ey) / TILE)));
    *x1 = imin(gx, imax(0, f2i((px + ex + TILE - 1) / TILE)));
    *y1 = imin(gy, imax(0, f2i((py + ey + TILE - 1) / TILE)));
}

/* HR/forward.cu:25-76 (and the Interp variant :86-138 via the lerped sh pointer) */
static v3 sh_to_rgb(int deg, const float *sh /* M*3 */, v3 pos, v3 campos, uint8_t *clamp_bits)
{
    v3 dir = vsub(pos, campos);
    float len = sqrtf(vdot(dir, dir));
    dir = V3(dir.x / len, dir.y / len, dir.z / len);
#define SHV(k) V3(sh[3 * (k)], sh[3 * (k) + 1], sh[3 * (k) + 2])
    v3 res = vscale(SH_C0, SHV(0));
    if (deg > 0) {
        float x = dir.x, y = dir.y, z = dir.z;
        res = vsub(vadd(vsub(res, vscale(SH_C1 * y, SHV(1))), vscale(SH_C1 * z, SHV(2))), vscale(SH_C1 * x, SHV(3)));
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            res = vadd(res, vscale(SH_C2[0] * xy, SHV(4)));
            res = vadd(res, vscale(SH_C2[1] * yz, SHV(5)));
            res = vadd(res, vscale(SH_C2[2] * (2.0f * zz - xx - yy), SHV(6)));
            res = vadd(res, vscale(SH_C2[3] * xz, SHV(7)));
            res = vadd(res, vscale(SH_C2[4] * (xx - yy), SHV(8)));
            if (deg > 2) {
                res = vadd(res, vscale(SH_C3[0] * y * (3.0f * xx - yy), SHV(9)));
                res = vadd(res, vscale(SH_C3[1] * xy * z, SHV(10)));
                res = vadd(res, vscale(SH_C3[2] * y * (4.0f * zz - xx - yy), SHV(11)));
                res = vadd(res, vscale(SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy), SHV(12)));
                res = vadd(res, vscale(SH_C3[4] * x * (4.0f * zz - xx - yy), SHV(13)));
                res = vadd(res, vscale(SH_C3[5] * z * (xx - yy), SHV(14)));
                res = vadd(res, vscale(SH_C3[6] * x * (xx - 3.0f * yy), SHV(15)));
            }
        }
    }
#undef SHV
    res = V3(res.x + 0.5f, res.y + 0.5f, res.z + 0.5f);
    *clamp_bits = (uint8_t)((res.x < 0) | ((res.y < 0) << 1) | ((res.z < 0) << 2));
    return V3(fmaxf(res.x, 0.0f), fmaxf(res.y, 0.0f), fmaxf(res.z, 0.0f));
}

/* HR/forward.cu:181-215 -- quaternion used as given (no normalisation) */
static void cov3d_fwd(v3 scale, float mod, const float q[4], float out[6])
{
    m3 S = mcols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = mod * scale.x;
    S.m[1][1] = mod * scale.y;
    S.m[2][2] = mod * scale.z;
    float r = q[0], x = q[1], y = q[2], z = q[3];
    m3 R = mcols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                 2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                 2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    m3 M = mmul(S, R);
    m3 Sig = mmul(mtrans(M), M);
    out[0] = Sig.m[0][0]; out[1] = Sig.m[0][1]; out[2] = Sig.m[0][2];
    out[3] = Sig.m[1][1]; out[4] = Sig.m[1][2]; out[5] = Sig.m[2][2];
}

/* Shared by HR/forward.cu:141-176 and HR/backward.cu:176-204 */
typedef struct { v3 t; float txtz, tytz, limx, limy; m3 W, J, T, Vrk, cov; } cov2d_ctx;
static void cov2d_eval(v3 mean, float fx, float fy, float tanx, float tany, const float *c3, const float *view,
                       cov2d_ctx *k)
{
    v3 t = xform43(mean, view);
    k->limx = 1.3f * tanx;
    k->limy = 1.3f * tany;
    k->txtz = t.x / t.z;
    k->tytz = t.y / t.z;
    t.x = fminf(k->limx, fmaxf(-k->limx, k->txtz)) * t.z;
    t.y = fminf(k->limy, fmaxf(-k->limy, k->tytz)) * t.z;
    k->t = t;
    k->J = mcols(fx / t.z, 0.0f, -(fx * t.x) / (t.z * t.z), 0.0f, fy / t.z, -(fy * t.y) / (t.z * t.z), 0, 0, 0);
    k->W = mcols(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6], view[10]);
    k->T = mmul(k->W, k->J);
    k->Vrk = mcols(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
    k->cov = mmul(mmul(mtrans(k->T), mtrans(k->Vrk)), k->T);
}

/* Argument block shared by forward / backward (mirrors include/hlgs.h hlgs_raster_args) */
typedef struct {
    int P, D, M, W, H;
    const float *bg;            /* 3 */
    const float *means3D;       /* P_full x 3 */
    const float *shs;           /* P_full x M x 3 or NULL */
    const float *colors_precomp;/* P x 3 or NULL */
    const float *opacities;     /* P_full */
    const float *scales;        /* P_full x 3 or NULL */
    const float *rotations;     /* P_full x 4 or NULL */
    const float *cov3D_precomp; /* P x 6 or NULL */
    const float *viewmatrix;    /* 16 */
    const float *projmatrix;    /* 16 */
    const float *campos;        /* 3 */
    float scale_modifier, tanfovx, tanfovy;
    const int *indices;         /* hierarchy mode (P entries) or NULL */
    const int *parent_indices;
    const float *ts;
    const int *kids;
    /* alt-rasterizer variant (submodules/alt-rasterizer, AR below): SH split into dc (P x 3, degree 0) and
     * shs = the M higher-order coefficients; AA opacity scaling optional; radius rect with exact per-tile
     * culling; its own blend backward (AR/backward.cu:424-605). */
    const float *dc;
    int antialiasing;
    int alt;
    /* not the reference's: bin no instance whose quadrant mask (rect_quad_masks) is 0, as the HIP binning does with
     * packed entries and HLGS_DROP_EMPTY (hlgs_point_list_drops_empty).  Such an instance reaches no pixel of its tile
     * with alpha >= 1/255, so the images and gradients do not change; the tile lists and n_contrib positions do. */
    int drop_empty;
} orc_args;

/* Per-Gaussian geometry produced by the forward preprocess (HR/rasterizer_impl.h:29-45) */
typedef struct {
    float *depths;          /* P */
    uint8_t *clamped;       /* P bitmask (bit c = channel c clamped) */
    float *means2D;         /* P x 2 */
    float *cov3D;           /* P x 6 */
    float *conic_opacity;   /* P x 4 */
    float *rgb;             /* P x 3 */
    uint32_t *tiles_touched;/* P */
    uint32_t *point_offsets;/* P, inclusive scan */
    int *rects;             /* P x 2 */
    int *radii;             /* P */
} orc_geom;

/* HR/forward.cu:218-445 (preprocessCUDA<3>) for one Gaussian */
static void preprocess_one(const orc_args *a, const orc_geom *g, int t_idx, int gx, int gy)
{
    const float focal_y = a->H / (2.0f * a->tanfovy);
    const float focal_x = a->W / (2.0f * a->tanfovx);
    int r_idx = a->indices ? a->indices[t_idx] : t_idx;
    int use_parent = 0, p_idx = 0;
    float t = 0.f;
    g->radii[t_idx] = 0;
    g->tiles_touched[t_idx] = 0;
    v3 p_orig = V3(a->means3D[3 * r_idx], a->means3D[3 * r_idx + 1], a->means3D[3 * r_idx + 2]);
    if (a->parent_indices) {
        p_idx = a->parent_indices[t_idx];
        if (p_idx != -1) { use_parent = 1; t = a->ts[t_idx]; }
        else p_idx = 0;
    }
    if (use_parent) {
        v3 pa = V3(a->means3D[3 * p_idx], a->means3D[3 * p_idx + 1], a->means3D[3 * p_idx + 2]);
        p_orig = V3(t * p_orig.x + (1.0f - t) * pa.x, t * p_orig.y + (1.0f - t) * pa.y, t * p_orig.z + (1.0f - t) * pa.z);
    }
    float ph[4];
    xform44(p_orig, a->projmatrix, ph);
    float p_w = 1.0f / (ph[3] + 0.0000001f);
    float pp[3] = {ph[0] * p_w, ph[1] * p_w, ph[2] * p_w};
    v3 p_view = xform43(p_orig, a->viewmatrix);
    if (p_view.z <= 0.2f) return;

    const float *cov3D;
    if (a->cov3D_precomp == NULL) {
        v3 scale = V3(a->scales[3 * r_idx], a->scales[3 * r_idx + 1], a->scales[3 * r_idx + 2]);
        float rot[4] = {a->rotations[4 * r_idx], a->rotations[4 * r_idx + 1], a->rotations[4 * r_idx + 2],
                        a->rotations[4 * r_idx + 3]};
        if (use_parent) {
            v3 ps = V3(a->scales[3 * p_idx], a->scales[3 * p_idx + 1], a->scales[3 * p_idx + 2]);
            scale = vadd(vscale(t, scale), vscale(1.0f - t, ps));
            float orot[4] = {a->rotations[4 * p_idx], a->rotations[4 * p_idx + 1], a->rotations[4 * p_idx + 2],
                             a->rotations[4 * p_idx + 3]};
            float dp = rot[0] * orot[0] + rot[1] * orot[1] + rot[2] * orot[2] + rot[3] * orot[3];
            if (dp < 0.0) for (int i = 0; i < 4; i++) orot[i] = -orot[i];
            for (int i = 0; i < 4; i++) rot[i] = t * rot[i] + (1.0f - t) * orot[i];
        }
        cov3d_fwd(scale, a->scale_modifier, rot, g->cov3D + 6 * t_idx);
        cov3D = g->cov3D + 6 * t_idx;
    } else {
        /* A-3: the reference leaves cov3D unassigned here; we take the evident intent. */
        cov3D = a->cov3D_precomp + 6 * t_idx;
        memcpy(g->cov3D + 6 * t_idx, cov3D, 6 * sizeof(float));
    }
    cov2d_ctx k;
    cov2d_eval(p_orig, focal_x, focal_y, a->tanfovx, a->tanfovy, cov3D, a->viewmatrix, &k);
    float cx = k.cov.m[0][0], cy = k.cov.m[0][1], cz = k.cov.m[1][1];
    const float h_var = 0.3f;
    const float det_cov = cx * cz - cy * cy;
    cx += h_var;
    cz += h_var;
    const float det_h = cx * cz - cy * cy;
    float h_scale = sqrtf(fmaxf(0.000025f, det_cov / det_h));
    if (a->alt && !a->antialiasing) h_scale = 1.0f; /* AR/forward.cu:226-229 */
    const float det = det_h;
    if (det == 0.0f) return;
    float det_inv = 1.f / det;
    float conic[3] = {cz * det_inv, -cy * det_inv, cx * det_inv};
    float mid = 0.5f * (cx + cz);
    float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    float my_radius = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
    float pix[2] = {ndc2pix(pp[0], a->W), ndc2pix(pp[1], a->H)};
    int ex = f2i(ceilf(3.f * sqrtf(cx))), ey = f2i(ceilf(3.f * sqrtf(cz)));
    if (a->alt) ex = ey = f2i(my_radius); /* AR/forward.cu:249: getRect with the eigen radius */
    g->rects[2 * t_idx] = ex;
    g->rects[2 * t_idx + 1] = ey;
    int x0, y0, x1, y1;
    get_rect(pix[0], pix[1], ex, ey, gx, gy, &x0, &y0, &x1, &y1);
    if ((uint32_t)(x1 - x0) * (uint32_t)(y1 - y0) == 0) return;

    if (a->colors_precomp == NULL) {
        v3 campos = V3(a->campos[0], a->campos[1], a->campos[2]);
        v3 mean_r = V3(a->means3D[3 * r_idx], a->means3D[3 * r_idx + 1], a->means3D[3 * r_idx + 2]);
        v3 rgb;
        if (a->alt) {
            /* AR/forward.cu:23-75, 257: coefficient 0 from dc, coefficient k >= 1 from shs[k - 1] */
            float tmp[16 * 3];
            memset(tmp, 0, sizeof(tmp));
            memcpy(tmp, a->dc + 3 * (size_t)r_idx, 3 * sizeof(float));
            int nrest = a->M < 15 ? a->M : 15;
            if (a->shs) memcpy(tmp + 3, a->shs + (size_t)r_idx * a->M * 3, sizeof(float) * 3 * nrest);
            rgb = sh_to_rgb(a->D, tmp, mean_r, campos, &g->clamped[t_idx]);
        } else if (!use_parent) {
            rgb = sh_to_rgb(a->D, a->shs + (size_t)r_idx * a->M * 3, mean_r, campos, &g->clamped[t_idx]);
        } else {
            /* HR/forward.cu:86-138: lerp every coefficient, view dir from the child mean */
            float tmp[16 * 3];
            const float *sc = a->shs + (size_t)r_idx * a->M * 3, *sp = a->shs + (size_t)p_idx * a->M * 3;
            int ncoef = a->M < 16 ? a->M : 16;
            for (int i = 0; i < 3 * ncoef; i++) tmp[i] = t * sc[i] + (1.0f - t) * sp[i];
            rgb = sh_to_rgb(a->D, tmp, mean_r, campos, &g->clamped[t_idx]);
        }
        g->rgb[3 * t_idx] = rgb.x;
        g->rgb[3 * t_idx + 1] = rgb.y;
        g->rgb[3 * t_idx + 2] = rgb.z;
    }
    g->depths[t_idx] = p_view.z;
    g->radii[t_idx] = f2i(my_radius);
    g->means2D[2 * t_idx] = pix[0];
    g->means2D[2 * t_idx + 1] = pix[1];
    float opacity = a->opacities[r_idx];
    if (use_parent) opacity = t * opacity + (1.0f - t) * a->opacities[p_idx];
    g->conic_opacity[4 * t_idx] = conic[0];
    g->conic_opacity[4 * t_idx + 1] = conic[1];
    g->conic_opacity[4 * t_idx + 2] = conic[2];
    g->conic_opacity[4 * t_idx + 3] = opacity * h_scale;
    g->tiles_touched[t_idx] = (uint32_t)(y1 - y0) * (uint32_t)(x1 - x0);
}

/* Forward phase 1: preprocess + inclusive scan (HR/rasterizer_impl.cu:280-333). Returns R. */
int orc_forward_preprocess(const orc_args *a, orc_geom *g)
{
    int gx = (a->W + TILE - 1) / TILE, gy = (a->H + TILE - 1) / TILE;
    memset(g->clamped, 0, (size_t)a->P);
    memset(g->rgb, 0, sizeof(float) * 3 * (size_t)a->P);
    memset(g->rects, 0, sizeof(int) * 2 * (size_t)a->P);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < a->P; i++) preprocess_one(a, g, i, gx, gy);
    uint64_t acc = 0;
    for (int i = 0; i < a->P; i++) { acc += g->tiles_touched[i]; g->point_offsets[i] = (uint32_t)acc; }
    return a->P ? (int)g->point_offsets[a->P - 1] : 0;
}

typedef struct { uint64_t key; uint32_t pos; uint32_t val; } kv;
static int kv_cmp(const void *pa, const void *pb)
{
    const kv *x = (const kv *)pa, *y = (const kv *)pb;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->pos < y->pos ? -1 : (x->pos > y->pos);
}

/* Image-space state (HR/rasterizer_impl.h:47-54) */
typedef struct {
    float *final_T;     /* N */
    uint32_t *n_contrib;/* N */
    uint32_t *ranges;   /* T x 2 */
    uint32_t *point_list; /* R */
    const float *pixel_colors;    /* alt: the forward's colour output (AR/rasterizer_impl.cu:459) */
    const float *pixel_invdepths; /* alt: the forward's inverse depth */
} orc_img;

/* AR/rasterizer_impl.cu:52-101 (max_contrib_power_rect_gaussian_float<15, 15>) and :147-179: does the
 * Gaussian keep its instance in tile (tx, ty)?  The power at the point of the tile's pixel box that the
 * reference takes as the closest one must not exceed log(o / (1/255)).  The float operations follow the
 * reference's order (no contraction); the logarithm is taken in double and rounded, so this restatement and
 * the HIP kernels (hlgs_math.h alt_tile_keep) make identical decisions. */
static int alt_tile_keep(float mx, float my, const float *co, int tx, int ty)
{
    const float rminx = (float)(tx * TILE), rminy = (float)(ty * TILE);
    const float rmaxx = (float)((tx + 1) * TILE - 1), rmaxy = (float)((ty + 1) * TILE - 1);
    const float x_min_diff = rminx - mx;
    const float x_left = x_min_diff > 0.0f;
    const float not_in_x = x_left + (mx > rmaxx);
    const float y_min_diff = rminy - my;
    const float y_above = y_min_diff > 0.0f;
    const float not_in_y = y_above + (my > rmaxy);
    float power = 0.0f;
    if ((not_in_y + not_in_x) > 0.0f) {
        const float px = x_left * rminx + (1.0f - x_left) * rmaxx;
        const float py = y_above * rminy + (1.0f - y_above) * rmaxy;
        const float dx = copysignf(15.0f, x_min_diff), dy = copysignf(15.0f, y_min_diff);
        const float diffx = mx - px, diffy = my - py;
        const float rcx = 1.0f / (225.0f * co[0]), rcz = 1.0f / (225.0f * co[2]);
        float sx = (dx * co[0] * diffx + dx * co[1] * diffy) * rcx;
        float sy = (dy * co[1] * diffx + dy * co[2] * diffy) * rcz;
        sx = sx != sx ? 0.0f : fminf(fmaxf(sx, 0.0f), 1.0f); /* __saturatef (NaN -> 0) */
        sy = sy != sy ? 0.0f : fminf(fmaxf(sy, 0.0f), 1.0f);
        const float tx_ = not_in_y * sx, ty_ = not_in_x * sy;
        const float qx = px + tx_ * dx, qy = py + ty_ * dy;
        const float ddx = mx - qx, ddy = my - qy;
        power = 0.5f * (co[0] * ddx * ddx + co[2] * ddy * ddy) + co[1] * ddx * ddy;
    }
    const float thr = (float)log((double)(co[3] / (1.0f / 255.0f)));
    return power <= thr;
}

/* Footprint quadrant masks of the first 8 tiles of a Gaussian's rect, restated operation for operation from the HIP
 * preprocess (hlgs_math.h splat_foot, splat_bands, band_extent, row_bands, row_quad_mask, rect_quad_masks): IEEE
 * square roots and divisions, no contraction (the serial and OpenMP builds; the contracted variance build never
 * drops), fmaf where the kernels write it -- so the masks, and with drop_empty the binned instances, are
 * bit-identical.  The test itself: an 8x8 block can hold a pixel with alpha >= 1/255 only if
 * the ellipse Q(u, v) = a u^2 + 2 b u v + c v^2 <= t (t = -2 ln2 thr, widened) overlaps it; per 8-row band the
 * ellipse's x-extent is compared with the block's columns, widened by a tolerance far above the float rounding. */
typedef struct { float x, y, nb, det, at, ia, vmax, vr, tol; int mode; } orc_bands;
static inline float med3f(float v, float lo, float hi) { return fmaxf(fminf(v, lo), fminf(fmaxf(v, lo), hi)); }
static orc_bands splat_bands(float x, float y, const float *co, float thr)
{
    orc_bands s;
    s.x = x; s.y = y;
    s.nb = s.det = s.at = s.ia = s.vmax = s.vr = s.tol = 0.f;
    s.mode = 0;
    const float o = co[3];
    if (o != o || co[0] != co[0] || co[1] != co[1] || co[2] != co[2] || x != x || y != y) { s.mode = 1; return s; }
    if (o < (1.0f / 255.0f) * 0.999f) { s.mode = 2; return s; }
    const float det0 = co[0] * co[2] - co[1] * co[1]; /* splat_foot's */
    if (!(det0 > 0.f) || !(co[0] > 0.f) || !(co[2] > 0.f)) { s.mode = 1; return s; }
    const float t = fmaxf(-1.3862944f * thr, 0.f) * 1.002f + 2e-3f;
    const float a = co[0], b = co[1], c = co[2];
    const float bb = b * b, e = fmaf(-b, b, bb);
    const float det = fmaf(a, c, -bb) + e;
    if (!(det > 0.f)) { s.mode = 1; return s; }
    const float idet = 1.0f / det;
    s.ia = 1.0f / a;
    const float vmax = sqrtf(a * t * idet);
    s.nb = -b;
    s.det = det;
    s.at = a * t;
    s.vmax = fmaf(vmax, 1e-4f, vmax) + 1e-3f;
    s.vr = -b * sqrtf(t * idet * (1.0f / c));
    s.tol = 2e-3f * (sqrtf(s.at) + fabsf(b) * vmax) * s.ia + 2e-3f;
    return s;
}
static void band_extent(const orc_bands *s, float v0, float *umin, float *umax)
{
    const float lo = fmaxf(v0, -s->vmax), hi = fminf(v0 + 7.f, s->vmax);
    if (!(lo <= hi)) { *umin = 3e38f; *umax = -3e38f; return; }
    const float vR = med3f(s->vr, lo, hi), vL = med3f(-s->vr, lo, hi);
    *umax = fmaf(s->nb, vR, sqrtf(fmaxf(fmaf(-s->det * vR, vR, s->at), 0.f))) * s->ia + s->tol;
    *umin = fmaf(s->nb, vL, -sqrtf(fmaxf(fmaf(-s->det * vL, vL, s->at), 0.f))) * s->ia - s->tol;
}
static uint32_t rect_quad_masks(float x, float y, const float *co, float thr, int x0, int y0, int x1, int y1)
{
    const orc_bands s = splat_bands(x, y, co, thr);
    const int w = x1 - x0, n = (x1 - x0) * (y1 - y0) < 8 ? (x1 - x0) * (y1 - y0) : 8;
    uint32_t m = 0;
    float lo0 = 3e38f, hi0 = -3e38f, lo1 = 3e38f, hi1 = -3e38f;
    for (int r = 0; r < n; r++) {
        const int ty = y0 + r / w, tx = x0 + r % w;
        if (r == 0 || tx == x0) { /* row_bands */
            lo0 = lo1 = 3e38f;
            hi0 = hi1 = -3e38f;
            if (!s.mode) {
                const float v0 = (float)(ty * TILE) - s.y;
                band_extent(&s, v0, &lo0, &hi0);
                band_extent(&s, v0 + 8.f, &lo1, &hi1);
            }
        }
        uint32_t q; /* row_quad_mask */
        if (s.mode) q = s.mode == 1 ? 0xFu : 0u;
        else {
            const float u0 = (float)(tx * TILE) - s.x, u7 = u0 + 7.f, u8 = u0 + 8.f, u15 = u0 + 15.f;
            q = (hi0 >= u0 && lo0 <= u7 ? 1u : 0u) | (hi0 >= u8 && lo0 <= u15 ? 2u : 0u) |
                (hi1 >= u0 && lo1 <= u7 ? 4u : 0u) | (hi1 >= u8 && lo1 <= u15 ? 8u : 0u);
        }
        m |= q << (4 * r);
    }
    return m;
}

/* Forward phase 2: duplicate, stable sort, ranges, blend (HR/rasterizer_impl.cu:335-399, HR/forward.cu:450-596) */

/* Splat falloff and the alpha >= 1/255 test (forward.cu:539-560, backward.cu:614-643), restated so
 * that every implementation in this repository makes the same keep/skip decisions ("alpha
 * threshold"):
 *  - power is evaluated as e2 = power * log2(e) = (qa dx + qb dy) dx + qc dy^2 with the conic pre-scaled
 *    by -log2(e) * (1/2, 1, 1/2), in one fixed IEEE order with fused multiply-adds -- bit-identical to the
 *    HIP kernels' splat_e2; G = exp2(e2) = exp(power);
 *  - "alpha >= 1/255" is e2 >= thr, thr = the smallest float at or above the exact real threshold
 *    (-log2(255 o); with lerp, log2(a_star / o) for t a_star + (1 - t)(1 - (1 - a_star)^fr) = 1/255), computed once per
 *    Gaussian in double.  A float alpha test instead would depend on the exp implementation and, for
 *    elongated splats, on the ~1e-3 relative error of the cancelling float quadratic form. */
static inline void conic_q(const float *co, float *q)
{
    const float kL2E = 1.4426950408889634f;
    q[0] = -0.5f * kL2E * co[0];
    q[1] = -kL2E * co[1];
    q[2] = -0.5f * kL2E * co[2];
}
static inline float splat_e2(const float *q, float dx, float dy)
{
    return fmaf(q[2] * dy, dy, fmaf(q[1], dy, q[0] * dx) * dx);
}
static float alpha_e2_threshold(float o, int interp, float t, float fr)
{
    if (o != o) return -INFINITY;
    if (!(o > 0.0f)) return INFINITY;
    const double target = 1.0 / 255.0;
    double a = target;
    if (interp) {
        const double td = t, fd = fr;
#define G_(x) (td * (x) + (1.0 - td) * (1.0 - pow(1.0 - (x), fd)))
        if (G_(0.99) < target) return INFINITY;
        double lo = 0.0, hi = 0.99;
        for (int i = 0; i < 64; i++) {
            const double mid = 0.5 * (lo + hi);
            if (G_(mid) >= target) hi = mid; else lo = mid;
        }
#undef G_
        a = hi;
    }
    const double thr = log2(a / (double)o);
    float f = (float)thr;
    if ((double)f < thr) f = nextafterf(f, INFINITY);
    return f;
}
/* per-Gaussian thresholds of a frame (caller frees) */
static float *alpha_thresholds(const orc_args *a, const orc_geom *g)
{
    float *thr = (float *)malloc(sizeof(float) * (size_t)(a->P > 0 ? a->P : 1));
    const int interp = a->ts != NULL && a->kids != NULL;
    for (int i = 0; i < a->P; i++)
        thr[i] = alpha_e2_threshold(g->conic_opacity[4 * i + 3], interp, interp ? a->ts[i] : 0.0f,
                                    interp ? 1.0f / (float)a->kids[i] : 0.0f);
    return thr;
}

/* One pixel-splat pair: the falloff G and the (lerped) alpha; returns 0 when the reference skips the pair
 * (power > 0 or alpha < 1/255), decided per g_ref_order.  fwd selects the forward's __powf = exp2(fr log2 x)
 * for the lerped alpha (HR/forward.cu:551), otherwise powf (HR/backward.cu:632). */
static inline int pair_alpha(const float *co, float dx, float dy, float thr, int interp, float tt, float fr, int fwd,
                             float *G, float *my_alpha, float *alpha)
{
    float g, e2 = 0.0f;
    if (g_ref_order) {
        const float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
        if (power > 0.0f) return 0;
        g = expf(power);
    } else {
        float q[3];
        conic_q(co, q);
        e2 = splat_e2(q, dx, dy); /* power * log2(e) */
        if (e2 > 0.0f) return 0;
        g = exp2f(e2);
    }
    const float ma = fminf(0.99f, co[3] * g);
    float al = ma;
    if (interp) {
        const float ka = fwd ? 1.0f - exp2f(fr * log2f(1.0f - ma)) : 1.0f - powf(1.0f - ma, fr);
        al = tt * ma + (1.0f - tt) * ka;
    }
    if (g_ref_order ? al < 1.0f / 255.0f : e2 < thr) return 0; /* alpha < 1/255 */
    *G = g;
    *my_alpha = ma;
    *alpha = al;
    return 1;
}

void orc_forward_render(const orc_args *a, const orc_geom *g, orc_img *im, int R, float *out_color,
                        float *out_invdepth, int *seen)
{
    int gx = (a->W + TILE - 1) / TILE, gy = (a->H + TILE - 1) / TILE, T = gx * gy;
    int W = a->W, H = a->H;
    memset(out_color, 0, sizeof(float) * 3 * (size_t)W * H);
    if (out_invdepth) memset(out_invdepth, 0, sizeof(float) * (size_t)W * H);
    memset(im->ranges, 0, sizeof(uint32_t) * 2 * (size_t)T);
    if (R == 0 && !a->alt) return; /* A-7: output stays 0, not bg (the alt rasterizer renders bg) */
    kv *buf = (kv *)malloc(sizeof(kv) * (size_t)(R > 0 ? R : 1));
    float *thr = alpha_thresholds(a, g);
    /* duplicateWithKeys, HR/rasterizer_impl.cu:70-115; AR/rasterizer_impl.cu:120-191 adds the per-tile
     * culling: a culled instance gets the sentinel key (tile 0xFFFFFFFF, depth FLT_MAX) and sorts last */
    const float fltmax = FLT_MAX;
    uint32_t maxbits;
    memcpy(&maxbits, &fltmax, 4);
#pragma omp parallel for schedule(dynamic, 1024)
    for (int i = 0; i < a->P; i++) {
        if (g->radii[i] <= 0) continue;
        uint32_t off = i == 0 ? 0 : g->point_offsets[i - 1];
        const uint32_t off_to = g->point_offsets[i];
        int x0, y0, x1, y1;
        get_rect(g->means2D[2 * i], g->means2D[2 * i + 1], g->rects[2 * i], g->rects[2 * i + 1], gx, gy, &x0, &y0, &x1, &y1);
        uint32_t dbits;
        memcpy(&dbits, &g->depths[i], 4);
        const uint32_t qm = a->drop_empty ? rect_quad_masks(g->means2D[2 * i], g->means2D[2 * i + 1],
                                                            g->conic_opacity + 4 * i, thr[i], x0, y0, x1, y1)
                                          : 0xFFFFFFFFu;
        uint32_t r = 0;
        for (int y = y0; y < y1; y++)
            for (int x = x0; x < x1; x++, r++) {
                if (a->alt && !alt_tile_keep(g->means2D[2 * i], g->means2D[2 * i + 1], g->conic_opacity + 4 * i, x, y))
                    continue;
                if (r < 8 && !((qm >> (4 * r)) & 0xFu)) continue; /* drop_empty: reaches none of the quadrants */
                buf[off].key = ((uint64_t)(uint32_t)(y * gx + x) << 32) | dbits;
                buf[off].pos = off;
                buf[off].val = (uint32_t)i;
                off++;
            }
        for (; off < off_to; off++) {
            buf[off].key = ((uint64_t)0xFFFFFFFFu << 32) | maxbits;
            buf[off].pos = off;
            buf[off].val = 0xFFFFFFFFu;
        }
    }
    /* stable radix sort == sort by (key, input position), App. A-4: a stable counting pass on the key's tile word
     * (the sentinel tile last), then each tile's run sorted by (depth bits, position) -- the order of one global
     * sort by (key, position), with independent runs */
    {
        uint32_t *start = (uint32_t *)calloc((size_t)T + 2, sizeof(uint32_t));
        kv *tmp = (kv *)malloc(sizeof(kv) * (size_t)(R > 0 ? R : 1));
        for (int i = 0; i < R; i++) {
            const uint32_t t = (uint32_t)(buf[i].key >> 32);
            start[(t == 0xFFFFFFFFu ? (uint32_t)T : t) + 1]++;
        }
        for (int t = 0; t <= T; t++) start[t + 1] += start[t];
        uint32_t *cur = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)T + 1));
        memcpy(cur, start, sizeof(uint32_t) * ((size_t)T + 1));
        for (int i = 0; i < R; i++) {
            const uint32_t t = (uint32_t)(buf[i].key >> 32);
            tmp[cur[t == 0xFFFFFFFFu ? (uint32_t)T : t]++] = buf[i];
        }
#pragma omp parallel for schedule(dynamic, 16)
        for (int t = 0; t <= T; t++)
            if (start[t + 1] - start[t] > 1) qsort(tmp + start[t], start[t + 1] - start[t], sizeof(kv), kv_cmp);
        free(buf);
        buf = tmp;
        free(cur);
        free(start);
    }
    for (int i = 0; i < R; i++) im->point_list[i] = buf[i].val;
    /* identifyTileRanges, HR/rasterizer_impl.cu:120-142 (AR/rasterizer_impl.cu:195-220 skips the sentinel) */
    for (int i = 0; i < R; i++) {
        uint32_t cur = (uint32_t)(buf[i].key >> 32);
        int valid = cur != 0xFFFFFFFFu;
        if (i == 0) { if (valid) im->ranges[2 * cur] = 0; }
        else {
            uint32_t prev = (uint32_t)(buf[i - 1].key >> 32);
            if (cur != prev) { im->ranges[2 * prev + 1] = i; if (valid) im->ranges[2 * cur] = i; }
        }
        if (i == R - 1 && valid) im->ranges[2 * cur + 1] = R;
    }
    free(buf);
    const float *feat = a->colors_precomp ? a->colors_precomp : g->rgb;
    int do_interp = (a->ts != NULL && a->kids != NULL);
    /* renderCUDA<3> per pixel, HR/forward.cu:450-596 (AR/forward.cu:282-430) */
#pragma omp parallel for collapse(2) schedule(dynamic, 4)
    for (int ty = 0; ty < gy; ty++)
        for (int tx = 0; tx < gx; tx++) {
            uint32_t rs = im->ranges[2 * (ty * gx + tx)], re = im->ranges[2 * (ty * gx + tx) + 1];
            for (int py = ty * TILE; py < imin((ty + 1) * TILE, H); py++)
                for (int px = tx * TILE; px < imin((tx + 1) * TILE, W); px++) {
                    float Tt = 1.0f, C[3] = {0, 0, 0}, inv = 0.0f;
                    uint32_t contributor = 0, last = 0;
                    for (uint32_t j = rs; j < re; j++) {
                        contributor++;
                        uint32_t id = im->point_list[j];
                        float dx = g->means2D[2 * id] - (float)px, dy = g->means2D[2 * id + 1] - (float)py;
                        const float *co = g->conic_opacity + 4 * id;
                        const int ip = do_interp && (int)id < a->P;
                        float G, my_alpha, alpha;
                        if (!pair_alpha(co, dx, dy, thr[id], ip, ip ? a->ts[id] : 0.0f,
                                        ip ? 1.0f / (float)a->kids[id] : 0.0f, 1, &G, &my_alpha, &alpha))
                            continue;
                        float test_T = Tt * (1 - alpha);
                        if (test_T < 0.0001f) break; /* done */
                        if (seen) {
#pragma omp atomic write
                            seen[id] = 1;
                        }
                        for (int ch = 0; ch < 3; ch++) C[ch] += feat[3 * id + ch] * alpha * Tt;
                        if (out_invdepth) inv += (1 / g->depths[id]) * alpha * Tt;
                        Tt = test_T;
                        last = contributor;
                    }
                    size_t pid = (size_t)py * W + px;
                    im->final_T[pid] = Tt;
                    im->n_contrib[pid] = last;
                    for (int ch = 0; ch < 3; ch++) out_color[ch * (size_t)H * W + pid] = C[ch] + Tt * a->bg[ch];
                    if (out_invdepth) out_invdepth[pid] = inv;
                }
        }
    free(thr);
}

/* Diagnostics (tests/test_gpu_refparity.py, tools/ref_flips.py): the threshold decisions of one pixel's pairs in both
 * alpha modes, on a frame whose point_list / ranges are set (they do not depend on the mode).  For each of the
 * pixel's tile-list entries k < cap, front to back: keep[2k + m] = 1 if mode m (0: the shared contract A-17, 1: the
 * reference's float order) keeps the pair (power <= 0 and alpha >= 1/255), alpha[2k + m] its alpha (0 if skipped).
 * last[m] = the n_contrib of the forward walk in mode m (its T < 1e-4 stop included).  Returns the list length. */
int orc_pixel_pairs(const orc_args *a, const orc_geom *g, const orc_img *im, int px, int py, int cap, int *keep,
                    float *alpha_out, int *last)
{
    const int gx = (a->W + TILE - 1) / TILE;
    const int t = (py / TILE) * gx + px / TILE;
    const uint32_t rs = im->ranges[2 * t], re = im->ranges[2 * t + 1];
    float *thr = alpha_thresholds(a, g);
    const int saved = g_ref_order;
    const int do_interp = (a->ts != NULL && a->kids != NULL);
    for (int m = 0; m < 2; m++) {
        g_ref_order = m;
        float Tt = 1.0f;
        int stopped = 0;
        last[m] = 0;
        for (uint32_t j = rs; j < re; j++) {
            const int k = (int)(j - rs);
            const uint32_t id = im->point_list[j];
            const float dx = g->means2D[2 * id] - (float)px, dy = g->means2D[2 * id + 1] - (float)py;
            const int ip = do_interp && (int)id < a->P;
            float G, my_alpha, al = 0.0f;
            const int kp = pair_alpha(g->conic_opacity + 4 * id, dx, dy, thr[id], ip, ip ? a->ts[id] : 0.0f,
                                      ip ? 1.0f / (float)a->kids[id] : 0.0f, 1, &G, &my_alpha, &al);
            if (k < cap) {
                keep[2 * k + m] = kp;
                alpha_out[2 * k + m] = kp ? al : 0.0f;
            }
            if (!kp || stopped) continue;
            const float test_T = Tt * (1 - al);
            if (test_T < 0.0001f) { stopped = 1; continue; }
            Tt = test_T;
            last[m] = k + 1;
        }
    }
    g_ref_order = saved;
    free(thr);
    return (int)(re - rs);
}

/* Backward gradient outputs; every array has P_full rows and must be zero on entry. */
typedef struct {
    float *dmean2D;  /* x3 */
    float *dconic;   /* x4 (2x2) */
    float *dopacity; /* x1 */
    float *dcolor;   /* x3 */
    float *dinvdepth;/* x1 or NULL */
    float *dmean3D;  /* x3 */
    float *dcov3D;   /* x6 */
    float *dsh;      /* x M*3 */
    float *dscale;   /* x3 */
    float *drot;     /* x4 */
    float *ddc;      /* x3 (alt variant: gradient of the degree-0 coefficient) */
} orc_grads;

/* Record layout per tile-list position j (10 floats): dcolor r g b, dinvdepth, dmean2D x y, dconic 0 1 3, dopacity. */
static void tile_records_add(const orc_img *im, int T, const int *indices, const float *rec, orc_grads *o)
{
    for (int t = 0; t < T; t++)
        for (uint32_t j = im->ranges[2 * t]; j < im->ranges[2 * t + 1]; j++) {
            const uint32_t id = im->point_list[j];
            const int gid = indices ? indices[id] : (int)id;
            const float *r = rec + 10 * (size_t)j;
            for (int ch = 0; ch < 3; ch++) o->dcolor[3 * gid + ch] += r[ch];
            if (o->dinvdepth) o->dinvdepth[gid] += r[3];
            o->dmean2D[3 * gid] += r[4];
            o->dmean2D[3 * gid + 1] += r[5];
            o->dconic[4 * gid] += r[6];
            o->dconic[4 * gid + 1] += r[7];
            o->dconic[4 * gid + 3] += r[8];
            o->dopacity[gid] += r[9];
        }
}
static float *tile_records(const orc_img *im, int T)
{
    uint32_t n = 0;
    for (int t = 0; t < T; t++) n = n > im->ranges[2 * t + 1] ? n : im->ranges[2 * t + 1];
    return (float *)calloc(10 * (size_t)(n > 0 ? n : 1), sizeof(float));
}

/* HR/backward.cu:498-721 (renderCUDA<3> backward) */
static void blend_backward(const orc_args *a, const orc_geom *g, const orc_img *im, const float *dL_dpix,
                           const float *dL_dinv, orc_grads *o)
{
    float *thr = alpha_thresholds(a, g);
    int gx = (a->W + TILE - 1) / TILE, gy = (a->H + TILE - 1) / TILE;
    int W = a->W, H = a->H;
    const float *col = a->colors_precomp ? a->colors_precomp : g->rgb;
    int interp = (a->ts != NULL && a->kids != NULL);
    const float ddelx_dx = 0.5f * W, ddely_dy = 0.5f * H;
    float *rec = tile_records(im, gx * gy);
#pragma omp parallel for collapse(2) schedule(dynamic, 4)
    for (int ty = 0; ty < gy; ty++)
        for (int tx = 0; tx < gx; tx++) {
            uint32_t rs = im->ranges[2 * (ty * gx + tx)], re = im->ranges[2 * (ty * gx + tx) + 1];
            for (int py = ty * TILE; py < imin((ty + 1) * TILE, H); py++)
                for (int px = tx * TILE; px < imin((tx + 1) * TILE, W); px++) {
                    size_t pid = (size_t)py * W + px;
                    const float T_final = im->final_T[pid];
                    float T = T_final;
                    uint32_t contributor = re - rs;
                    const uint32_t last = im->n_contrib[pid];
                    float acc[3] = {0, 0, 0}, dpix[3], last_alpha = 0, last_color[3] = {0, 0, 0};
                    float dinv = 0, acc_inv = 0, last_inv = 0;
                    for (int i = 0; i < 3; i++) dpix[i] = dL_dpix[i * (size_t)H * W + pid];
                    if (dL_dinv) dinv = dL_dinv[pid];
                    for (uint32_t k = re; k > rs; k--) {
                        uint32_t j = k - 1;
                        contributor--;
                        if (contributor >= last) continue;
                        uint32_t id = im->point_list[j];
                        float dx = g->means2D[2 * id] - (float)px, dy = g->means2D[2 * id + 1] - (float)py;
                        const float *co = g->conic_opacity + 4 * id;
                        const float tt = interp ? a->ts[id] : 0.0f, fr = interp ? 1.0f / (float)a->kids[id] : 0.0f;
                        float G, my_alpha, alpha;
                        if (!pair_alpha(co, dx, dy, thr[id], interp, tt, fr, 0, &G, &my_alpha, &alpha)) continue;
                        const int nullalpha = co[3] * G > 0.99f;
                        T = T / (1.f - alpha);
                        const float weight = alpha * T;
                        float dL_dalpha = 0.0f;
                        float *r = rec + 10 * (size_t)j;
                        for (int ch = 0; ch < 3; ch++) {
                            const float c = col[3 * id + ch];
                            acc[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * acc[ch];
                            last_color[ch] = c;
                            dL_dalpha += (c - acc[ch]) * dpix[ch];
                            r[ch] += weight * dpix[ch];
                        }
                        if (dL_dinv) {
                            const float invd = 1.f / g->depths[id];
                            acc_inv = last_alpha * last_inv + (1.f - last_alpha) * acc_inv;
                            last_inv = invd;
                            dL_dalpha += (invd - acc_inv) * dinv;
                            r[3] += weight * dinv;
                        }
                        dL_dalpha *= T;
                        last_alpha = alpha;
                        float bg_dot = 0;
                        for (int i = 0; i < 3; i++) bg_dot += a->bg[i] * dpix[i];
                        dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
                        dL_dalpha = nullalpha ? 0 : dL_dalpha;
                        const float dL_dG = co[3] * dL_dalpha;
                        const float gdx = G * dx, gdy = G * dy;
                        const float dG_ddelx = -gdx * co[0] - gdy * co[1];
                        const float dG_ddely = -gdy * co[2] - gdx * co[1];
                        r[4] += dL_dG * dG_ddelx * ddelx_dx;
                        r[5] += dL_dG * dG_ddely * ddely_dy;
                        r[6] += -0.5f * gdx * dx * dL_dG;
                        r[7] += -0.5f * gdx * dy * dL_dG;
                        r[8] += -0.5f * gdy * dy * dL_dG;
                        float mult = 1.0f;
                        if (interp) mult = tt - powf(1.0f - my_alpha, fr - 1.0f) * (tt - 1.0f) * fr;
                        r[9] += mult * G * dL_dalpha;
                    }
                }
        }
    tile_records_add(im, gx * gy, a->indices, rec, o);
    free(rec);
    free(thr);
}


/* AR/backward.cu:452-605 (PerGaussianRenderCUDA), restated per pixel.  The reference walks each 32-splat
 * bucket over the tile's pixels starting from the forward's sampled state (T, accumulated colour and inverse
 * depth at the bucket's first splat); walking every pixel's list front to back from T = 1 and zero
 * accumulators visits the same (pixel, splat) pairs with the same state.  ar = accumulated - final colour,
 * where the final colour includes T_final * bg, and the bg term is added again (AR/backward.cu:608, 619);
 * there is no o * G > 0.99 rule. */
static void blend_backward_alt(const orc_args *a, const orc_geom *g, const orc_img *im, const float *dL_dpix,
                               const float *dL_dinv, orc_grads *o)
{
    float *thr = alpha_thresholds(a, g);
    int gx = (a->W + TILE - 1) / TILE, gy = (a->H + TILE - 1) / TILE;
    int W = a->W, H = a->H;
    const size_t HW = (size_t)W * H;
    const float *col = a->colors_precomp ? a->colors_precomp : g->rgb;
    const float ddelx_dx = 0.5f * W, ddely_dy = 0.5f * H;
    float *rec = tile_records(im, gx * gy);
#pragma omp parallel for collapse(2) schedule(dynamic, 4)
    for (int ty = 0; ty < gy; ty++)
        for (int tx = 0; tx < gx; tx++) {
            uint32_t rs = im->ranges[2 * (ty * gx + tx)], re = im->ranges[2 * (ty * gx + tx) + 1];
            for (int py = ty * TILE; py < imin((ty + 1) * TILE, H); py++)
                for (int px = tx * TILE; px < imin((tx + 1) * TILE, W); px++) {
                    const size_t pid = (size_t)py * W + px;
                    const float T_final = im->final_T[pid];
                    const uint32_t last = im->n_contrib[pid];
                    float T = 1.0f, ar[3], ard, dpix[3], dinv = dL_dinv ? dL_dinv[pid] : 0.0f;
                    for (int ch = 0; ch < 3; ch++) {
                        ar[ch] = -im->pixel_colors[ch * HW + pid];
                        dpix[ch] = dL_dpix[ch * HW + pid];
                    }
                    ard = -im->pixel_invdepths[pid];
                    for (uint32_t j = rs; j < re; j++) {
                        if (j - rs >= last) break;
                        const uint32_t id = im->point_list[j];
                        const float dx = g->means2D[2 * id] - (float)px, dy = g->means2D[2 * id + 1] - (float)py;
                        const float *co = g->conic_opacity + 4 * id;
                        float G, my_alpha, alpha;
                        if (!pair_alpha(co, dx, dy, thr[id], 0, 0.0f, 0.0f, 0, &G, &my_alpha, &alpha)) continue;
                        const float weight = alpha * T;
                        float bg_dot = 0.0f, dL_dalpha = 0.0f;
                        float *r = rec + 10 * (size_t)j;
                        for (int ch = 0; ch < 3; ch++) {
                            const float c = col[3 * id + ch];
                            ar[ch] += weight * c;
                            r[ch] += weight * dpix[ch];
                            dL_dalpha += ((c * T) - (1.0f / (1.0f - alpha)) * (-ar[ch])) * dpix[ch];
                            bg_dot += a->bg[ch] * dpix[ch];
                        }
                        const float invd = 1.f / g->depths[id];
                        ard += weight * invd;
                        if (o->dinvdepth) r[3] += weight * dinv;
                        dL_dalpha += ((invd * T) - (1.0f / (1.0f - alpha)) * (-ard)) * dinv;
                        dL_dalpha += (-T_final / (1.0f - alpha)) * bg_dot;
                        T *= (1.0f - alpha);
                        const float dL_dG = co[3] * dL_dalpha;
                        const float gdx = G * dx, gdy = G * dy;
                        const float dG_ddelx = -gdx * co[0] - gdy * co[1];
                        const float dG_ddely = -gdy * co[2] - gdx * co[1];
                        r[4] += dL_dG * dG_ddelx * ddelx_dx;
                        r[5] += dL_dG * dG_ddely * ddely_dy;
                        r[6] += -0.5f * gdx * dx * dL_dG;
                        r[7] += -0.5f * gdx * dy * dL_dG;
                        r[8] += -0.5f * gdy * dy * dL_dG;
                        r[9] += G * dL_dalpha;
                    }
                }
        }
    tile_records_add(im, gx * gy, NULL, rec, o);
    free(rec);
    free(thr);
}

/* HR/auxiliary.h:132-142 */
static v3 dnormvdv(v3 v, v3 dv)
{
    float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    v3 r;
    r.x = ((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32;
    r.y = (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32;
    r.z = (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32;
    return r;
}

/* HR/backward.cu:23-142 */
static void sh_backward_rows(int idx, int t_idx, const orc_args *a, const orc_geom *g, orc_grads *o,
                             const float *sh, float *dsh)
{
    int deg = a->D;
    v3 pos = V3(a->means3D[3 * idx], a->means3D[3 * idx + 1], a->means3D[3 * idx + 2]);
    v3 campos = V3(a->campos[0], a->campos[1], a->campos[2]);
    v3 dir_orig = vsub(pos, campos);
    float len = sqrtf(vdot(dir_orig, dir_orig));
    v3 dir = V3(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len);
#define SHV(k) V3(sh[3 * (k)], sh[3 * (k) + 1], sh[3 * (k) + 2])
    v3 dRGB = V3(o->dcolor[3 * idx], o->dcolor[3 * idx + 1], o->dcolor[3 * idx + 2]);
    uint8_t cl = g->clamped[t_idx];
    dRGB.x *= (cl & 1) ? 0 : 1;
    dRGB.y *= (cl & 2) ? 0 : 1;
    dRGB.z *= (cl & 4) ? 0 : 1;
    v3 ddx = V3(0, 0, 0), ddy = V3(0, 0, 0), ddz = V3(0, 0, 0);
    float x = dir.x, y = dir.y, z = dir.z;
#define PUT(k, s) do { v3 _v = vscale((s), dRGB); dsh[3 * (k)] = _v.x; dsh[3 * (k) + 1] = _v.y; dsh[3 * (k) + 2] = _v.z; } while (0)
    PUT(0, SH_C0);
    if (deg > 0) {
        PUT(1, -SH_C1 * y);
        PUT(2, SH_C1 * z);
        PUT(3, -SH_C1 * x);
        ddx = vscale(-SH_C1, SHV(3));
        ddy = vscale(-SH_C1, SHV(1));
        ddz = vscale(SH_C1, SHV(2));
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            PUT(4, SH_C2[0] * xy);
            PUT(5, SH_C2[1] * yz);
            PUT(6, SH_C2[2] * (2.f * zz - xx - yy));
            PUT(7, SH_C2[3] * xz);
            PUT(8, SH_C2[4] * (xx - yy));
            ddx = vadd(ddx, vadd(vadd(vadd(vscale(SH_C2[0] * y, SHV(4)), vscale(SH_C2[2] * 2.f * -x, SHV(6))),
                                      vscale(SH_C2[3] * z, SHV(7))), vscale(SH_C2[4] * 2.f * x, SHV(8))));
            ddy = vadd(ddy, vadd(vadd(vadd(vscale(SH_C2[0] * x, SHV(4)), vscale(SH_C2[1] * z, SHV(5))),
                                      vscale(SH_C2[2] * 2.f * -y, SHV(6))), vscale(SH_C2[4] * 2.f * -y, SHV(8))));
            ddz = vadd(ddz, vadd(vadd(vscale(SH_C2[1] * y, SHV(5)), vscale(SH_C2[2] * 2.f * 2.f * z, SHV(6))),
                                 vscale(SH_C2[3] * x, SHV(7))));
            if (deg > 2) {
                PUT(9, SH_C3[0] * y * (3.f * xx - yy));
                PUT(10, SH_C3[1] * xy * z);
                PUT(11, SH_C3[2] * y * (4.f * zz - xx - yy));
                PUT(12, SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy));
                PUT(13, SH_C3[4] * x * (4.f * zz - xx - yy));
                PUT(14, SH_C3[5] * z * (xx - yy));
                PUT(15, SH_C3[6] * x * (xx - 3.f * yy));
                /* glm: scalar * vec3 products, coefficients multiplied left to right */
                v3 sx = vscale(SH_C3[0], SHV(9)); sx = vscale(3.f, sx); sx = vscale(2.f * xy, sx);
                v3 t;
                t = vscale(SH_C3[1], SHV(10)); t = vscale(yz, t); sx = vadd(sx, t);
                t = vscale(SH_C3[2], SHV(11)); t = vscale(-2.f, t); t = vscale(xy, t); sx = vadd(sx, t);
                t = vscale(SH_C3[3], SHV(12)); t = vscale(-3.f, t); t = vscale(2.f * xz, t); sx = vadd(sx, t);
                t = vscale(SH_C3[4], SHV(13)); t = vscale(-3.f * xx + 4.f * zz - yy, t); sx = vadd(sx, t);
                t = vscale(SH_C3[5], SHV(14)); t = vscale(2.f, t); t = vscale(xz, t); sx = vadd(sx, t);
                t = vscale(SH_C3[6], SHV(15)); t = vscale(3.f, t); t = vscale(xx - yy, t); sx = vadd(sx, t);
                ddx = vadd(ddx, sx);
                v3 sy = vscale(SH_C3[0], SHV(9)); sy = vscale(3.f, sy); sy = vscale(xx - yy, sy);
                t = vscale(SH_C3[1], SHV(10)); t = vscale(xz, t); sy = vadd(sy, t);
                t = vscale(SH_C3[2], SHV(11)); t = vscale(-3.f * yy + 4.f * zz - xx, t); sy = vadd(sy, t);
                t = vscale(SH_C3[3], SHV(12)); t = vscale(-3.f, t); t = vscale(2.f * yz, t); sy = vadd(sy, t);
                t = vscale(SH_C3[4], SHV(13)); t = vscale(-2.f, t); t = vscale(xy, t); sy = vadd(sy, t);
                t = vscale(SH_C3[5], SHV(14)); t = vscale(-2.f, t); t = vscale(yz, t); sy = vadd(sy, t);
                t = vscale(SH_C3[6], SHV(15)); t = vscale(-3.f, t); t = vscale(2.f * xy, t); sy = vadd(sy, t);
                ddy = vadd(ddy, sy);
                v3 sz = vscale(SH_C3[1], SHV(10)); sz = vscale(xy, sz);
                t = vscale(SH_C3[2], SHV(11)); t = vscale(4.f, t); t = vscale(2.f * yz, t); sz = vadd(sz, t);
                t = vscale(SH_C3[3], SHV(12)); t = vscale(3.f, t); t = vscale(2.f * zz - xx - yy, t); sz = vadd(sz, t);
                t = vscale(SH_C3[4], SHV(13)); t = vscale(4.f, t); t = vscale(2.f * xz, t); sz = vadd(sz, t);
                t = vscale(SH_C3[5], SHV(14)); t = vscale(xx - yy, t); sz = vadd(sz, t);
                ddz = vadd(ddz, sz);
            }
        }
    }
#undef PUT
#undef SHV
    v3 dL_ddir = V3(vdot(ddx, dRGB), vdot(ddy, dRGB), vdot(ddz, dRGB));
    v3 dm = dnormvdv(dir_orig, dL_ddir);
    o->dmean3D[3 * idx] += dm.x;
    o->dmean3D[3 * idx + 1] += dm.y;
    o->dmean3D[3 * idx + 2] += dm.z;
}
static void sh_backward(int idx, int t_idx, const orc_args *a, const orc_geom *g, orc_grads *o)
{
    if (!a->alt) {
        sh_backward_rows(idx, t_idx, a, g, o, a->shs + (size_t)idx * a->M * 3, o->dsh + (size_t)idx * a->M * 3);
        return;
    }
    /* AR/backward.cu:23-146: coefficient 0 (dc) gets its own gradient, coefficients k >= 1 come from shs[k-1] */
    float sh[16 * 3], dsh[16 * 3];
    memset(sh, 0, sizeof(sh));
    memset(dsh, 0, sizeof(dsh));
    int nrest = a->M < 15 ? a->M : 15;
    memcpy(sh, a->dc + 3 * (size_t)idx, 3 * sizeof(float));
    memcpy(sh + 3, a->shs + (size_t)idx * a->M * 3, sizeof(float) * 3 * nrest);
    sh_backward_rows(idx, t_idx, a, g, o, sh, dsh);
    memcpy(o->ddc + 3 * (size_t)idx, dsh, 3 * sizeof(float));
    int ncoef = (a->D + 1) * (a->D + 1) - 1;
    for (int i = 0; i < 3 * ncoef && i < 3 * nrest; i++) o->dsh[(size_t)idx * a->M * 3 + i] = dsh[3 + i];
}

/* HR/backward.cu:330-393 */
static void cov3d_backward(int idx, v3 scale, float mod, const float *q, orc_grads *o)
{
    float r = q[0], x = q[1], y = q[2], z = q[3];
    m3 R = mcols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                 2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                 2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    m3 S = mcols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    v3 s = vscale(mod, scale);
    S.m[0][0] = s.x; S.m[1][1] = s.y; S.m[2][2] = s.z;
    m3 M = mmul(S, R);
    const float *d = o->dcov3D + 6 * idx;
    m3 dS = mcols(d[0], 0.5f * d[1], 0.5f * d[2], 0.5f * d[1], d[3], 0.5f * d[4], 0.5f * d[2], 0.5f * d[4], d[5]);
    m3 M2 = M;
    for (int c = 0; c < 3; c++) for (int rr = 0; rr < 3; rr++) M2.m[c][rr] = 2.0f * M.m[c][rr];
    m3 dM = mmul(M2, dS);
    m3 Rt = mtrans(R), dMt = mtrans(dM);
    float *ds = o->dscale + 3 * idx;
    for (int i = 0; i < 3; i++)
        ds[i] = Rt.m[i][0] * dMt.m[i][0] + Rt.m[i][1] * dMt.m[i][1] + Rt.m[i][2] * dMt.m[i][2];
    for (int rr = 0; rr < 3; rr++) { dMt.m[0][rr] *= s.x; dMt.m[1][rr] *= s.y; dMt.m[2][rr] *= s.z; }
    float *dq = o->drot + 4 * idx;
    dq[0] = 2 * z * (dMt.m[0][1] - dMt.m[1][0]) + 2 * y * (dMt.m[2][0] - dMt.m[0][2]) + 2 * x * (dMt.m[1][2] - dMt.m[2][1]);
    dq[1] = 2 * y * (dMt.m[1][0] + dMt.m[0][1]) + 2 * z * (dMt.m[2][0] + dMt.m[0][2]) + 2 * r * (dMt.m[1][2] - dMt.m[2][1]) - 4 * x * (dMt.m[2][2] + dMt.m[1][1]);
    dq[2] = 2 * x * (dMt.m[1][0] + dMt.m[0][1]) + 2 * r * (dMt.m[2][0] - dMt.m[0][2]) + 2 * z * (dMt.m[1][2] + dMt.m[2][1]) - 4 * y * (dMt.m[2][2] + dMt.m[0][0]);
    dq[3] = 2 * r * (dMt.m[0][1] - dMt.m[1][0]) + 2 * x * (dMt.m[2][0] + dMt.m[0][2]) + 2 * y * (dMt.m[1][2] + dMt.m[2][1]) - 4 * z * (dMt.m[1][1] + dMt.m[0][0]);
}

/* Full backward: HR/rasterizer_impl.cu:404-517 = blend bwd, computeCov2DCUDA (HR/backward.cu:147-326),
 * preprocessCUDA bwd (HR/backward.cu:398-495). */
void orc_backward(const orc_args *a, const orc_geom *g, const orc_img *im, int R, const float *dL_dpix,
                  const float *dL_dinv, orc_grads *o)
{
    const float focal_y = a->H / (2.0f * a->tanfovy);
    const float focal_x = a->W / (2.0f * a->tanfovx);
    if (a->alt) blend_backward_alt(a, g, im, dL_dpix, dL_dinv, o);
    else if (R > 0) blend_backward(a, g, im, dL_dpix, dL_dinv, o);
    const float *cov3Ds = a->cov3D_precomp ? a->cov3D_precomp : g->cov3D;
    /* computeCov2DCUDA (rows are per Gaussian unless render indices may repeat or write a parent's row) */
    const int par = a->indices == NULL && a->parent_indices == NULL;
#pragma omp parallel for schedule(static) if (par)
    for (int t_idx = 0; t_idx < a->P; t_idx++) {
        if (!(g->radii[t_idx] > 0)) continue;
        const float *c3 = cov3Ds + 6 * t_idx;
        int idx = a->indices ? a->indices[t_idx] : t_idx;
        v3 mean = V3(a->means3D[3 * idx], a->means3D[3 * idx + 1], a->means3D[3 * idx + 2]);
        v3 dconic = V3(o->dconic[4 * idx], o->dconic[4 * idx + 1], o->dconic[4 * idx + 3]);
        cov2d_ctx k;
        cov2d_eval(mean, focal_x, focal_y, a->tanfovx, a->tanfovy, c3, a->viewmatrix, &k);
        const float xg = k.txtz < -k.limx || k.txtz > k.limx ? 0 : 1;
        const float yg = k.tytz < -k.limy || k.tytz > k.limy ? 0 : 1;
        m3 Tm = k.T, Vrk = k.Vrk, Wm = k.W;
        float c_xx = k.cov.m[0][0], c_xy = k.cov.m[0][1], c_yy = k.cov.m[1][1];
        const float h_var = 0.3f;
        const float det_cov = c_xx * c_yy - c_xy * c_xy;
        c_xx += h_var;
        c_yy += h_var;
        const float det_h = c_xx * c_yy - c_xy * c_xy;
        float dxx = 0.f, dxy = 0.f, dyy = 0.f;
        if (!a->alt || a->antialiasing) { /* AR/backward.cu:212-245: only with antialiasing */
            const float hs = sqrtf(fmaxf(0.000025f, det_cov / det_h));
            const float dop_v = o->dopacity[idx];
            const float d_hs = dop_v * a->opacities[idx];
            o->dopacity[idx] = dop_v * hs;
            const float d_inside = (det_cov / det_h) <= 0.000025f ? 0.f : d_hs / (2 * hs);
            const float x = c_xx, y = c_yy, z = c_xy, w = h_var;
            const float sqv = w * w + w * (x + y) + x * y - z * z;
            const float denom_f = d_inside / (sqv * sqv);
            dxx = w * (w * y + y * y + z * z) * denom_f;
            dyy = w * (w * x + x * x + z * z) * denom_f;
            dxy = -2.f * w * z * (w + x + y) * denom_f;
        }
        float denom = c_xx * c_yy - c_xy * c_xy;
        float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
        float *dcov = o->dcov3D + 6 * idx;
        #define TT(c, r) Tm.m[c][r]
        if (denom2inv != 0) {
            dxx += denom2inv * (-c_yy * c_yy * dconic.x + 2 * c_xy * c_yy * dconic.y + (denom - c_xx * c_yy) * dconic.z);
            dyy += denom2inv * (-c_xx * c_xx * dconic.z + 2 * c_xx * c_xy * dconic.y + (denom - c_xx * c_yy) * dconic.x);
            dxy += denom2inv * 2 * (c_xy * c_yy * dconic.x - (denom + 2 * c_xy * c_xy) * dconic.y + c_xx * c_xy * dconic.z);
            dcov[0] = (TT(0,0) * TT(0,0) * dxx + TT(0,0) * TT(1,0) * dxy + TT(1,0) * TT(1,0) * dyy);
            dcov[3] = (TT(0,1) * TT(0,1) * dxx + TT(0,1) * TT(1,1) * dxy + TT(1,1) * TT(1,1) * dyy);
            dcov[5] = (TT(0,2) * TT(0,2) * dxx + TT(0,2) * TT(1,2) * dxy + TT(1,2) * TT(1,2) * dyy);
            dcov[1] = 2 * TT(0,0) * TT(0,1) * dxx + (TT(0,0) * TT(1,1) + TT(0,1) * TT(1,0)) * dxy + 2 * TT(1,0) * TT(1,1) * dyy;
            dcov[2] = 2 * TT(0,0) * TT(0,2) * dxx + (TT(0,0) * TT(1,2) + TT(0,2) * TT(1,0)) * dxy + 2 * TT(1,0) * TT(1,2) * dyy;
            dcov[4] = 2 * TT(0,2) * TT(0,1) * dxx + (TT(0,1) * TT(1,2) + TT(0,2) * TT(1,1)) * dxy + 2 * TT(1,1) * TT(1,2) * dyy;
        } else {
            for (int i = 0; i < 6; i++) dcov[i] = 0;
        }
        #define VK(c, r) Vrk.m[c][r]
        float dT00 = 2 * (TT(0,0) * VK(0,0) + TT(0,1) * VK(0,1) + TT(0,2) * VK(0,2)) * dxx + (TT(1,0) * VK(0,0) + TT(1,1) * VK(0,1) + TT(1,2) * VK(0,2)) * dxy;
        float dT01 = 2 * (TT(0,0) * VK(1,0) + TT(0,1) * VK(1,1) + TT(0,2) * VK(1,2)) * dxx + (TT(1,0) * VK(1,0) + TT(1,1) * VK(1,1) + TT(1,2) * VK(1,2)) * dxy;
        float dT02 = 2 * (TT(0,0) * VK(2,0) + TT(0,1) * VK(2,1) + TT(0,2) * VK(2,2)) * dxx + (TT(1,0) * VK(2,0) + TT(1,1) * VK(2,1) + TT(1,2) * VK(2,2)) * dxy;
        float dT10 = 2 * (TT(1,0) * VK(0,0) + TT(1,1) * VK(0,1) + TT(1,2) * VK(0,2)) * dyy + (TT(0,0) * VK(0,0) + TT(0,1) * VK(0,1) + TT(0,2) * VK(0,2)) * dxy;
        float dT11 = 2 * (TT(1,0) * VK(1,0) + TT(1,1) * VK(1,1) + TT(1,2) * VK(1,2)) * dyy + (TT(0,0) * VK(1,0) + TT(0,1) * VK(1,1) + TT(0,2) * VK(1,2)) * dxy;
        float dT12 = 2 * (TT(1,0) * VK(2,0) + TT(1,1) * VK(2,1) + TT(1,2) * VK(2,2)) * dyy + (TT(0,0) * VK(2,0) + TT(0,1) * VK(2,1) + TT(0,2) * VK(2,2)) * dxy;
        #undef VK
        #undef TT
        #define WW(c, r) Wm.m[c][r]
        float dJ00 = WW(0,0) * dT00 + WW(0,1) * dT01 + WW(0,2) * dT02;
        float dJ02 = WW(2,0) * dT00 + WW(2,1) * dT01 + WW(2,2) * dT02;
        float dJ11 = WW(1,0) * dT10 + WW(1,1) * dT11 + WW(1,2) * dT12;
        float dJ12 = WW(2,0) * dT10 + WW(2,1) * dT11 + WW(2,2) * dT12;
        #undef WW
        v3 t = k.t;
        float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
        float dtx = xg * -focal_x * tz2 * dJ02;
        float dty = yg * -focal_y * tz2 * dJ12;
        float dtz = -focal_x * tz2 * dJ00 - focal_y * tz2 * dJ11 + (2 * focal_x * t.x) * tz3 * dJ02 + (2 * focal_y * t.y) * tz3 * dJ12;
        if (o->dinvdepth) dtz -= a->alt ? o->dinvdepth[idx] * tz2 : o->dinvdepth[idx] / (t.z * t.z); /* AR/backward.cu:312 */
        const float *vm = a->viewmatrix;
        o->dmean3D[3 * idx] = vm[0] * dtx + vm[1] * dty + vm[2] * dtz;
        o->dmean3D[3 * idx + 1] = vm[4] * dtx + vm[5] * dty + vm[6] * dtz;
        o->dmean3D[3 * idx + 2] = vm[8] * dtx + vm[9] * dty + vm[10] * dtz;
    }
    /* preprocessCUDA backward */
    const float *proj = a->projmatrix;
#pragma omp parallel for schedule(static) if (par)
    for (int t_idx = 0; t_idx < a->P; t_idx++) {
        if (!(g->radii[t_idx] > 0)) continue;
        int idx = a->indices ? a->indices[t_idx] : t_idx;
        v3 m = V3(a->means3D[3 * idx], a->means3D[3 * idx + 1], a->means3D[3 * idx + 2]);
        float mh[4];
        xform44(m, proj, mh);
        float m_w = 1.0f / (mh[3] + 0.0000001f);
        float mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
        float mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
        float g2x = o->dmean2D[3 * idx], g2y = o->dmean2D[3 * idx + 1];
        v3 dm;
        dm.x = (proj[0] * m_w - proj[3] * mul1) * g2x + (proj[1] * m_w - proj[3] * mul2) * g2y;
        dm.y = (proj[4] * m_w - proj[7] * mul1) * g2x + (proj[5] * m_w - proj[7] * mul2) * g2y;
        dm.z = (proj[8] * m_w - proj[11] * mul1) * g2x + (proj[9] * m_w - proj[11] * mul2) * g2y;
        o->dmean3D[3 * idx] += dm.x;
        o->dmean3D[3 * idx + 1] += dm.y;
        o->dmean3D[3 * idx + 2] += dm.z;
        if (a->shs) sh_backward(idx, t_idx, a, g, o);
        if (a->scales)
            cov3d_backward(idx, V3(a->scales[3 * idx], a->scales[3 * idx + 1], a->scales[3 * idx + 2]),
                           a->scale_modifier, a->rotations + 4 * idx, o);
        if (a->parent_indices) {
            int parent = a->parent_indices[t_idx];
            if (parent == -1) continue;
            float tt = a->ts[t_idx];
            o->dopacity[idx] = 0;
            for (int i = 0; i < 3; i++) o->dscale[3 * idx + i] = 0;
            for (int i = 0; i < 4; i++) o->drot[4 * idx + i] = 0;
            float dl[3] = {o->dmean3D[3 * idx], o->dmean3D[3 * idx + 1], o->dmean3D[3 * idx + 2]};
            for (int i = 0; i < 3; i++) o->dmean3D[3 * idx + i] = 0;
            for (int i = 0; i < 3; i++) o->dmean3D[3 * parent + i] += (1.0f - tt) * dl[i];
            for (int i = 0; i < 3 * a->M; i++) o->dsh[(size_t)idx * a->M * 3 + i] = 0;
        }
    }
}

/* HR/rasterizer_impl.cu:54-66 + HR/auxiliary.h:164-189 */
void orc_mark_visible(int P, const float *means3D, const float *view, const float *proj, uint8_t *present)
{
    for (int i = 0; i < P; i++) {
        v3 p = V3(means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]);
        float ph[4];
        xform44(p, proj, ph);
        v3 pv = xform43(p, view);
        present[i] = !(pv.z <= 0.2f);
    }
}

/* HR/utils.cu:6-36 (MCMC relocation, eq. 9) */
void orc_compute_relocation(int P, const float *op_old, const float *sc_old, const int *N, const float *binoms,
                            int n_max, float *op_new, float *sc_new)
{
    for (int idx = 0; idx < P; idx++) {
        int n = N[idx];
        float denom = 0.0f;
        op_new[idx] = 1.0f - powf(1.0f - op_old[idx], 1.0f / n);
        for (int i = 1; i <= n; ++i)
            for (int k = 0; k <= i - 1; ++k) {
                float b = binoms[(i - 1) * n_max + k];
                float term = (float)((pow(-1.0, k) / sqrt((double)(k + 1))) * pow((double)op_new[idx], k + 1));
                denom += b * term;
            }
        float coeff = op_old[idx] / denom;
        for (int i = 0; i < 3; ++i) sc_new[3 * idx + i] = coeff * sc_old[3 * idx + i];
    }
}

/* ---------------- LOD (gaussianhierarchy runtime switching) ---------------- */

/* GH/runtime_switching.cu:147-163 -- offsets are computed then unused; the distance is plain */
static float gauss_dist(const float *pos, const float *vp)
{
    float d0 = vp[0] - pos[0], d1 = vp[1] - pos[1], d2 = vp[2] - pos[2];
    return sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
}
/* GH/runtime_switching.cu:165-187 */
static int in_cone(const float *pos, const float *vp, const float *zdir)
{
    float d0 = vp[0] - pos[0], d1 = vp[1] - pos[1], d2 = vp[2] - pos[2];
    float n = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
    float c = d0 / n * zdir[0] + d1 / n * zdir[1] + d2 / n * zdir[2];
    return c < -0.5;
}
/* GH/runtime_switching.cu:222-233 */
static float size_dyn(const float *pos, const float *scale, const float *vp)
{
    float md = gauss_dist(pos, vp);
    if (md < 0.0) return 0;
    return fmaxf(scale[0], fmaxf(scale[1], scale[2])) / md;
}

/* expand_to_size_dynamic: GH/runtime_switching.cu:533-582, 95-108, 748-782.
 * nodes: N x 6 int {depth, parent, child_count, first_child, next_sibling, max_side_length} */
int orc_expand_to_size_dynamic(int N, float target, const int *nodes, const float *pos, const float *scales,
                               const float *viewpoint, const float *viewdir, int *render_indices,
                               int *parent_indices, int *nodes_for_render_indices)
{
    int count = 0;
    for (int i = 0; i < N; i++) {
        const int *nd = nodes + 6 * i;
        if (!in_cone(pos + 3 * i, viewpoint, viewdir)) continue;
        float size = size_dyn(pos + 3 * i, scales + 3 * i, viewpoint);
        int c = 0;
        if (nd[0] < 0) c = 0;
        else if (size >= target && nd[2] == 0) c = 1;
        else if (nd[1] >= 0) {
            float ps = size_dyn(pos + 3 * nd[1], scales + 3 * nd[1], viewpoint);
            if (ps >= target && size < target) c = 1;
        }
        if (c) {
            render_indices[count] = i;
            nodes_for_render_indices[count] = i;
            if (nd[1] != -1) parent_indices[count] = nd[1];
            count++;
        }
    }
    return count;
}

/* get_interpolation_weights_dynamic: GH/runtime_switching.cu:637-684 */
void orc_interp_weights_dynamic(int n, const int *idx, float target, const int *nodes, const float *pos,
                                const float *scales, const float *viewpoint, float *ts, int *kids)
{
    for (int i = 0; i < n; i++) {
        int id = idx[i];
        const int *nd = nodes + 6 * id;
        float t;
        if (nd[1] < 0) t = 1.0f;
        else {
            float ps = size_dyn(pos + 3 * nd[1], scales + 3 * nd[1], viewpoint);
            if (ps > 2.0f * target) t = 1.0f;
            else {
                float s = size_dyn(pos + 3 * id, scales + 3 * id, viewpoint);
                float start = fmaxf(0.5f * ps, s);
                float diff = ps - start;
                if (diff <= 0) t = 1.0f;
                else {
                    float td = fmaxf(0.0f, target - start);
                    t = fmaxf(1.0f - (td / diff), 0.0f);
                }
            }
        }
        ts[i] = t;
        kids[i] = nd[1] < 0 ? 1 : nodes[6 * nd[1] + 2];
    }
}

/* Static (.hier) variant. Node: 7 int {depth, parent, start, count_leafs, count_merged, start_children,
 * count_children}; Box: 8 float {minn xyzw, maxx xyzw}.  GH/runtime_switching.cu:136-219 */
static float size_box(const float *box, const float *vp)
{
    int inside = 1;
    for (int i = 0; i < 3; i++) inside &= vp[i] >= box[i] && vp[i] <= box[4 + i];
    if (inside) return FLT_MAX;
    float c0 = fmaxf(box[0], fminf(box[4], vp[0])), c1 = fmaxf(box[1], fminf(box[5], vp[1])),
          c2 = fmaxf(box[2], fminf(box[6], vp[2]));
    float d0 = vp[0] - c0, d1 = vp[1] - c1, d2 = vp[2] - c2;
    float md = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
    return box[3] / md;
}

/* expand_to_size: GH/runtime_switching.cu:495-529, 68-93, 997-1030 */
int orc_expand_to_size(int N, float target, const int *nodes, const float *boxes, const float *viewpoint,
                       int *render_indices, int *parent_indices, int *nodes_for_render_indices)
{
    int off = 0;
    for (int i = 0; i < N; i++) {
        const int *nd = nodes + 7 * i;
        float size = size_box(boxes + 8 * i, viewpoint);
        int c = 0;
        if (size >= target) c = nd[3];
        else if (nd[1] != -1) {
            float ps = size_box(boxes + 8 * nd[1], viewpoint);
            if (ps >= target) { c = nd[3]; if (nd[0] != 0) c += nd[4]; }
        }
        int pg = nd[1] != -1 ? nodes[7 * nd[1] + 2] : -1;
        for (int k = 0; k < c; k++) {
            render_indices[off + k] = nd[2] + k;
            if (parent_indices) parent_indices[off + k] = pg;
            if (nodes_for_render_indices) nodes_for_render_indices[off + k] = i;
        }
        off += c;
    }
    return off;
}

/* get_interpolation_weights: GH/runtime_switching.cu:588-634 */
void orc_interp_weights(int n, const int *idx, float target, const int *nodes, const float *boxes,
                        const float *viewpoint, float *ts, int *kids)
{
    for (int i = 0; i < n; i++) {
        int id = idx[i];
        const int *nd = nodes + 7 * id;
        float t;
        if (nd[1] == -1) t = 1.0f;
        else {
            float ps = size_box(boxes + 8 * nd[1], viewpoint);
            if (ps > 2.0f * target) t = 1.0f;
            else {
                float s = size_box(boxes + 8 * id, viewpoint);
                float start = fmaxf(0.5f * ps, s);
                float diff = ps - start;
                if (diff <= 0) t = 1.0f;
                else {
                    float td = fmaxf(0.0f, target - start);
                    t = fmaxf(1.0f - (td / diff), 0.0f);
                }
            }
        }
        ts[i] = t;
        kids[i] = nd[1] == -1 ? 1 : nodes[7 * nd[1] + 6];
    }
}

/* get_spt_cut_cuda: GH/runtime_switching.cu:784-994.
 * compat=1 reproduces the reference exactly (App. A-10: boundary attribution via prefix>=idx, and
 * DeviceSelect(x != 0) dropping Gaussian 0).  compat=0 is the intended semantics of
 * scene/gaussian_model.py:163-181.  cut must hold sum(interval sizes) entries.  Returns count. */
int orc_spt_cut(int s, int E, const int *gidx, const int *starts, const float *smax, const float *smin,
                const int *sidx, const float *sdist, int compat, int *cut, int *counts_prefix, int *total_candidates)
{
    int *sizes = (int *)malloc(sizeof(int) * (s > 0 ? s : 1));
    int *prefix = (int *)malloc(sizeof(int) * (s > 0 ? s : 1));
    int *counts = (int *)calloc(s > 0 ? s : 1, sizeof(int));
    for (int k = 0; k < s; k++) {
        int index = sidx[k];
        float d = sdist[k];
        int low = starts[index], high = starts[index + 1];
        int pivot = (low + high) / 2;
        while (high - low > 1) {
            if (smax[pivot] > d) low = pivot;
            else high = pivot;
            pivot = (low + high) / 2;
        }
        sizes[k] = high - starts[index];
    }
    int sum = 0;
    for (int k = 0; k < s; k++) { prefix[k] = sum; sum += sizes[k]; }
    if (total_candidates) *total_candidates = sum;
    int n = 0;
    for (int idx = 0; idx < sum; idx++) {
        int ii;
        if (compat) {
            int low = 0, high = s;
            ii = s / 2;
            while (high - low > 1) {
                if (prefix[ii] >= idx) high = ii;
                else low = ii;
                ii = (high + low) / 2;
            }
        } else {
            int low = 0, high = s; /* largest k with prefix[k] <= idx */
            while (high - low > 1) {
                int mid = (low + high) / 2;
                if (prefix[mid] <= idx) low = mid; else high = mid;
            }
            ii = low;
        }
        int off = idx - prefix[ii];
        int g = starts[sidx[ii]] + off;
        /* compat: the misattributed candidate can index one past the last stored entry; the
         * reference reads out of bounds there, we treat it as rejected. */
        if (g >= E) continue;
        if (smin[g] < sdist[ii]) {
            counts[ii]++;
            int v = gidx[g];
            if (!compat || v != 0) cut[n++] = v;
        }
    }
    int acc = 0;
    for (int k = 0; k < s; k++) { counts_prefix[k] = acc; acc += counts[k]; }
    free(sizes); free(prefix); free(counts);
    return n;
}

/* HIP replacement target for gaussian_renderer/__init__.py:304-339 (render_post interp_python=True).
 * Activated tensors in; rows [0,S) copied, then one lerped row per render index. */
void orc_lod_interp_forward(int S, int n, int M3, const int *ridx, const int *pidx, const float *w,
                            const float *means, const float *scales, const float *rots, const float *opac,
                            const float *shs, float *o_means, float *o_scales, float *o_rots, float *o_opac,
                            float *o_shs)
{
    for (int i = 0; i < S; i++) {
        memcpy(o_means + 3 * i, means + 3 * i, 12);
        memcpy(o_scales + 3 * i, scales + 3 * i, 12);
        memcpy(o_rots + 4 * i, rots + 4 * i, 16);
        o_opac[i] = opac[i];
        if (shs) memcpy(o_shs + (size_t)M3 * i, shs + (size_t)M3 * i, sizeof(float) * M3);
    }
    for (int i = 0; i < n; i++) {
        int c = ridx[i], p = pidx[i], o = S + i;
        float t = w[i], u = 1 - w[i];
        for (int k = 0; k < 3; k++) o_means[3 * o + k] = t * means[3 * c + k] + u * means[3 * p + k];
        for (int k = 0; k < 3; k++) o_scales[3 * o + k] = t * scales[3 * c + k] + u * scales[3 * p + k];
        if (shs)
            for (int k = 0; k < M3; k++) o_shs[(size_t)M3 * o + k] = t * shs[(size_t)M3 * c + k] + u * shs[(size_t)M3 * p + k];
        float dot = 0;
        for (int k = 0; k < 4; k++) dot += rots[4 * c + k] * rots[4 * p + k];
        float sg = dot < 0 ? -1.0f : 1.0f;
        for (int k = 0; k < 4; k++) o_rots[4 * o + k] = t * rots[4 * c + k] + u * (sg * rots[4 * p + k]);
        o_opac[o] = t * opac[c] + u * opac[p];
    }
}

/* Autograd of the block above: grads accumulate into zero-initialised full-size arrays. */
void orc_lod_interp_backward(int S, int n, int M3, const int *ridx, const int *pidx, const float *w,
                             const float *rots, const float *g_means, const float *g_scales, const float *g_rots,
                             const float *g_opac, const float *g_shs, float *d_means, float *d_scales,
                             float *d_rots, float *d_opac, float *d_shs)
{
    for (int i = 0; i < S; i++) {
        for (int k = 0; k < 3; k++) { d_means[3 * i + k] += g_means[3 * i + k]; d_scales[3 * i + k] += g_scales[3 * i + k]; }
        for (int k = 0; k < 4; k++) d_rots[4 * i + k] += g_rots[4 * i + k];
        d_opac[i] += g_opac[i];
        if (g_shs) for (int k = 0; k < M3; k++) d_shs[(size_t)M3 * i + k] += g_shs[(size_t)M3 * i + k];
    }
    for (int i = 0; i < n; i++) {
        int c = ridx[i], p = pidx[i], o = S + i;
        float t = w[i], u = 1 - w[i];
        for (int k = 0; k < 3; k++) {
            d_means[3 * c + k] += t * g_means[3 * o + k];
            d_means[3 * p + k] += u * g_means[3 * o + k];
            d_scales[3 * c + k] += t * g_scales[3 * o + k];
            d_scales[3 * p + k] += u * g_scales[3 * o + k];
        }
        float dot = 0;
        for (int k = 0; k < 4; k++) dot += rots[4 * c + k] * rots[4 * p + k];
        float sg = dot < 0 ? -1.0f : 1.0f;
        for (int k = 0; k < 4; k++) {
            d_rots[4 * c + k] += t * g_rots[4 * o + k];
            d_rots[4 * p + k] += sg * (u * g_rots[4 * o + k]);
        }
        d_opac[c] += t * g_opac[o];
        d_opac[p] += u * g_opac[o];
        if (g_shs)
            for (int k = 0; k < M3; k++) {
                d_shs[(size_t)M3 * c + k] += t * g_shs[(size_t)M3 * o + k];
                d_shs[(size_t)M3 * p + k] += u * g_shs[(size_t)M3 * o + k];
            }
    }
}

/* SH -> RGB for a batch (the colour step of preprocessCUDA, HR/forward.cu:25-76), for fixture checks. */
void orc_sh_colors(int P, int D, int M, const float *shs, const float *means, const float *campos, float *rgb,
                   uint8_t *clamped)
{
    v3 cp = V3(campos[0], campos[1], campos[2]);
    for (int i = 0; i < P; i++) {
        v3 c = sh_to_rgb(D, shs + (size_t)i * M * 3, V3(means[3 * i], means[3 * i + 1], means[3 * i + 2]), cp,
                         &clamped[i]);
        rgb[3 * i] = c.x;
        rgb[3 * i + 1] = c.y;
        rgb[3 * i + 2] = c.z;
    }
}
