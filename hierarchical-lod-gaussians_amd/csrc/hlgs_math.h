// hlgs_math.h -- per-Gaussian projection / covariance / SH math shared by the gfx950 kernels.
//
// Semantics follow the reference rasterizer (paths relative to
// submodules/hierarchy-rasterizer/cuda_rasterizer): forward.cu:25-215 and
// auxiliary.h:53-142.  glm's column-major mat3 and its summation order are
// reproduced (m[c][r] = column c, row r) so results agree with the reference to
// the last few ulps; FMA contraction is left to the compiler, as nvcc does.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define HLGS_TILE 16
#define HLGS_TILE_PIX 256

namespace hlgs {

constexpr float kSH_C0 = 0.28209479177387814f;
constexpr float kSH_C1 = 0.4886025119029199f;
constexpr float kSH_C2[5] = {1.0925484305920792f, -1.0925484305920792f,
                                                       0.31539156525252005f, -1.0925484305920792f,
                                                       0.5462742152960396f};
constexpr float kSH_C3[7] = {-0.5900435899266435f, 2.890611442640554f,
                                                       -0.4570457994644658f, 0.3731763325901154f,
                                                       -0.4570457994644658f, 1.445305721320277f,
                                                       -0.5900435899266435f};

struct f3 { float x, y, z; };
struct m3 { float m[3][3]; };

__device__ __forceinline__ f3 mk(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 scl(float s, f3 a) { return mk(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

__device__ __forceinline__ m3 mcols(float a0, float a1, float a2, float a3, float a4, float a5, float a6,
                                    float a7, float a8)
{
    m3 r;
    r.m[0][0] = a0; r.m[0][1] = a1; r.m[0][2] = a2;
    r.m[1][0] = a3; r.m[1][1] = a4; r.m[1][2] = a5;
    r.m[2][0] = a6; r.m[2][1] = a7; r.m[2][2] = a8;
    return r;
}
__device__ __forceinline__ m3 mmul(const m3& a, const m3& b)
{
    m3 r;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int row = 0; row < 3; row++)
            r.m[c][row] = a.m[0][row] * b.m[c][0] + a.m[1][row] * b.m[c][1] + a.m[2][row] * b.m[c][2];
    return r;
}
__device__ __forceinline__ m3 mtrans(const m3& a)
{
    m3 r;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int row = 0; row < 3; row++) r.m[c][row] = a.m[row][c];
    return r;
}

// auxiliary.h:53-56, evaluated in double exactly as the reference does
__device__ __forceinline__ float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }

__device__ __forceinline__ f3 xform43(f3 p, const float* m)
{
    return mk(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
              m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}
__device__ __forceinline__ float xform44w(f3 p, const float* m) { return m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]; }

// auxiliary.h:70-80 (the torch path always passes per-axis rect extents)
__device__ __forceinline__ void tile_rect(float px, float py, int ex, int ey, int gx, int gy, int& x0, int& y0,
                                          int& x1, int& y1)
{
    x0 = min(gx, max(0, (int)((px - ex) / HLGS_TILE)));
    y0 = min(gy, max(0, (int)((py - ey) / HLGS_TILE)));
    x1 = min(gx, max(0, (int)((px + ex + HLGS_TILE - 1) / HLGS_TILE)));
    y1 = min(gy, max(0, (int)((py + ey + HLGS_TILE - 1) / HLGS_TILE)));
}

// forward.cu:25-76; `sh` points at M*3 floats of one Gaussian (possibly a lerped copy)
template <typename SHLoad>
__device__ __forceinline__ f3 sh_to_rgb(int deg, SHLoad shv, f3 pos, f3 campos, uint32_t& clamp_bits)
{
    f3 dir = sub(pos, campos);
    float len = sqrtf(dot(dir, dir));
    dir = mk(dir.x / len, dir.y / len, dir.z / len);
    f3 res = scl(kSH_C0, shv(0));
    if (deg > 0) {
        float x = dir.x, y = dir.y, z = dir.z;
        res = sub(add(sub(res, scl(kSH_C1 * y, shv(1))), scl(kSH_C1 * z, shv(2))), scl(kSH_C1 * x, shv(3)));
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            res = add(res, scl(kSH_C2[0] * xy, shv(4)));
            res = add(res, scl(kSH_C2[1] * yz, shv(5)));
            res = add(res, scl(kSH_C2[2] * (2.0f * zz - xx - yy), shv(6)));
            res = add(res, scl(kSH_C2[3] * xz, shv(7)));
            res = add(res, scl(kSH_C2[4] * (xx - yy), shv(8)));
            if (deg > 2) {
                res = add(res, scl(kSH_C3[0] * y * (3.0f * xx - yy), shv(9)));
                res = add(res, scl(kSH_C3[1] * xy * z, shv(10)));
                res = add(res, scl(kSH_C3[2] * y * (4.0f * zz - xx - yy), shv(11)));
                res = add(res, scl(kSH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy), shv(12)));
                res = add(res, scl(kSH_C3[4] * x * (4.0f * zz - xx - yy), shv(13)));
                res = add(res, scl(kSH_C3[5] * z * (xx - yy), shv(14)));
                res = add(res, scl(kSH_C3[6] * x * (xx - 3.0f * yy), shv(15)));
            }
        }
    }
    res = mk(res.x + 0.5f, res.y + 0.5f, res.z + 0.5f);
    clamp_bits = (res.x < 0 ? 1u : 0u) | (res.y < 0 ? 2u : 0u) | (res.z < 0 ? 4u : 0u);
    return mk(fmaxf(res.x, 0.0f), fmaxf(res.y, 0.0f), fmaxf(res.z, 0.0f));
}

// d colour / d (normalised) view direction of the SH colour: the reference's dRGBdx, dRGBdy, dRGBdz
// (backward.cu:55-139), in its operation order (glm scalar * vec3 products left to right), from the coefficients the
// forward already holds; the SH backward dots them with dL/dRGB.  `shv(c)` returns coefficient c as (r, g, b).
template <typename SHLoad>
__device__ __forceinline__ void sh_dir_jacobian(int deg, SHLoad shv, float x, float y, float z, f3& ddx, f3& ddy, f3& ddz)
{
    ddx = ddy = ddz = mk(0.f, 0.f, 0.f);
    if (deg < 1) return;
    ddx = scl(-kSH_C1, shv(3));
    ddy = scl(-kSH_C1, shv(1));
    ddz = scl(kSH_C1, shv(2));
    if (deg < 2) return;
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    ddx = add(ddx, add(add(add(scl(kSH_C2[0] * y, shv(4)), scl(kSH_C2[2] * 2.f * -x, shv(6))), scl(kSH_C2[3] * z, shv(7))),
                       scl(kSH_C2[4] * 2.f * x, shv(8))));
    ddy = add(ddy, add(add(add(scl(kSH_C2[0] * x, shv(4)), scl(kSH_C2[1] * z, shv(5))), scl(kSH_C2[2] * 2.f * -y, shv(6))),
                       scl(kSH_C2[4] * 2.f * -y, shv(8))));
    ddz = add(ddz, add(add(scl(kSH_C2[1] * y, shv(5)), scl(kSH_C2[2] * 2.f * 2.f * z, shv(6))), scl(kSH_C2[3] * x, shv(7))));
    if (deg < 3) return;
    f3 sx = scl(2.f * xy, scl(3.f, scl(kSH_C3[0], shv(9))));
    sx = add(sx, scl(yz, scl(kSH_C3[1], shv(10))));
    sx = add(sx, scl(xy, scl(-2.f, scl(kSH_C3[2], shv(11)))));
    sx = add(sx, scl(2.f * xz, scl(-3.f, scl(kSH_C3[3], shv(12)))));
    sx = add(sx, scl(-3.f * xx + 4.f * zz - yy, scl(kSH_C3[4], shv(13))));
    sx = add(sx, scl(xz, scl(2.f, scl(kSH_C3[5], shv(14)))));
    sx = add(sx, scl(xx - yy, scl(3.f, scl(kSH_C3[6], shv(15)))));
    ddx = add(ddx, sx);
    f3 sy = scl(xx - yy, scl(3.f, scl(kSH_C3[0], shv(9))));
    sy = add(sy, scl(xz, scl(kSH_C3[1], shv(10))));
    sy = add(sy, scl(-3.f * yy + 4.f * zz - xx, scl(kSH_C3[2], shv(11))));
    sy = add(sy, scl(2.f * yz, scl(-3.f, scl(kSH_C3[3], shv(12)))));
    sy = add(sy, scl(xy, scl(-2.f, scl(kSH_C3[4], shv(13)))));
    sy = add(sy, scl(yz, scl(-2.f, scl(kSH_C3[5], shv(14)))));
    sy = add(sy, scl(2.f * xy, scl(-3.f, scl(kSH_C3[6], shv(15)))));
    ddy = add(ddy, sy);
    f3 sz = scl(xy, scl(kSH_C3[1], shv(10)));
    sz = add(sz, scl(2.f * yz, scl(4.f, scl(kSH_C3[2], shv(11)))));
    sz = add(sz, scl(2.f * zz - xx - yy, scl(3.f, scl(kSH_C3[3], shv(12)))));
    sz = add(sz, scl(2.f * xz, scl(4.f, scl(kSH_C3[4], shv(13)))));
    sz = add(sz, scl(xx - yy, scl(kSH_C3[5], shv(14))));
    ddz = add(ddz, sz);
}

__device__ __forceinline__ m3 quat_rot(const float q[4])
{
    float r = q[0], x = q[1], y = q[2], z = q[3];
    return mcols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                 2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                 2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
}

// forward.cu:181-215 (quaternion used as given, no normalisation)
__device__ __forceinline__ void cov3d_fwd(f3 scale, float mod, const float q[4], float out[6])
{
    m3 S = mcols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.m[0][0] = mod * scale.x;
    S.m[1][1] = mod * scale.y;
    S.m[2][2] = mod * scale.z;
    m3 M = mmul(S, quat_rot(q));
    m3 Sig = mmul(mtrans(M), M);
    out[0] = Sig.m[0][0]; out[1] = Sig.m[0][1]; out[2] = Sig.m[0][2];
    out[3] = Sig.m[1][1]; out[4] = Sig.m[1][2]; out[5] = Sig.m[2][2];
}

// forward.cu:141-176 / backward.cu:176-204: EWA Jacobian and projected covariance
struct Cov2D {
    f3 t;
    float txtz, tytz, limx, limy;
    m3 W, T, Vrk, cov;
};
__device__ __forceinline__ void cov2d_eval(f3 mean, float fx, float fy, float tanx, float tany, const float* c3,
                                           const float* view, Cov2D& k)
{
    f3 t = xform43(mean, view);
    k.limx = 1.3f * tanx;
    k.limy = 1.3f * tany;
    k.txtz = t.x / t.z;
    k.tytz = t.y / t.z;
    t.x = fminf(k.limx, fmaxf(-k.limx, k.txtz)) * t.z;
    t.y = fminf(k.limy, fmaxf(-k.limy, k.tytz)) * t.z;
    k.t = t;
    m3 J = mcols(fx / t.z, 0.0f, -(fx * t.x) / (t.z * t.z), 0.0f, fy / t.z, -(fy * t.y) / (t.z * t.z), 0, 0, 0);
    k.W = mcols(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6], view[10]);
    k.T = mmul(k.W, J);
    k.Vrk = mcols(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
    k.cov = mmul(mmul(mtrans(k.T), mtrans(k.Vrk)), k.T);
}

// auxiliary.h:132-142
__device__ __forceinline__ f3 dnormvdv(f3 v, f3 dv)
{
    float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    f3 r;
    r.x = ((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32;
    r.y = (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32;
    r.z = (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32;
    return r;
}

// Which 8x8 pixel blocks can hold a pixel where this splat reaches alpha >= 1/255?
// alpha = min(0.99, o * exp(power)) >= 1/255 needs Q(u, v) = a u^2 + 2 b u v + c v^2 <= 2 ln(255 o) for
// (u, v) = pixel - centre (Q = conic).  The minimum of the convex Q over a block's box is 0 when the
// centre is inside, else the smallest of the four edge minima (vertex of the 1-D quadratic clamped to
// the edge).  Pairs outside are exactly the ones the reference skips (forward.cu:539-561,
// backward.cu:614-643); the kids-alpha of hierarchy mode is never larger than alpha, so the test stays
// conservative there.  Margins absorb the float rounding of power/exp.
struct SplatFoot {
    float x, y, a, b, c, kv, ku, t;  // kv = -b/c, ku = -b/a, t = threshold on Q
    int mode;                        // 0: test, 1: always (non-finite / degenerate), 2: never
};
// thr = the splat's alpha threshold on e2 (alpha_e2_threshold): alpha >= 1/255 needs e2 >= thr, i.e.
// Q <= -2 ln2 thr = 2 ln(255 o) (or the lerped bound in hierarchy mode), so the log is already in hand.
__device__ __forceinline__ SplatFoot splat_foot(float x, float y, float4 co, float thr)
{
#pragma clang fp contract(off)
    SplatFoot f;
    f.x = x; f.y = y; f.a = co.x; f.b = co.y; f.c = co.z;
    f.kv = f.ku = f.t = 0.f;
    f.mode = 0;
    const float o = co.w;
    if (o != o || co.x != co.x || co.y != co.y || co.z != co.z || x != x || y != y) { f.mode = 1; return f; }
    if (o < (1.0f / 255.0f) * 0.999f) { f.mode = 2; return f; }
    const float det = co.x * co.z - co.y * co.y;
    if (!(det > 0.f) || !(co.x > 0.f) || !(co.z > 0.f)) { f.mode = 1; return f; }
    f.t = fmaxf(-1.3862944f * thr, 0.f) * 1.002f + 2e-3f;
    f.kv = -co.y / co.z;
    f.ku = -co.y / co.x;
    return f;
}
__device__ __forceinline__ float q_edge_u(const SplatFoot& f, float U, float v0, float v1)  // u = U fixed
{
    const float v = __builtin_amdgcn_fmed3f(f.kv * U, v0, v1);
    return U * fmaf(f.a, U, 2.f * f.b * v) + f.c * v * v;
}
__device__ __forceinline__ float q_edge_v(const SplatFoot& f, float V, float u0, float u1)  // v = V fixed
{
    const float u = __builtin_amdgcn_fmed3f(f.ku * V, u0, u1);
    return V * fmaf(f.c, V, 2.f * f.b * u) + f.a * u * u;
}
__device__ __forceinline__ bool foot_touches(const SplatFoot& f, float qx, float qy)
{
    if (f.mode) return f.mode == 1;
    const float u0 = qx - f.x, u1 = u0 + 7.f, v0 = qy - f.y, v1 = v0 + 7.f;
    if (u0 <= 0.f && u1 >= 0.f && v0 <= 0.f && v1 >= 0.f) return true;
    const float m = fminf(fminf(q_edge_u(f, u0, v0, v1), q_edge_u(f, u1, v0, v1)),
                          fminf(q_edge_v(f, v0, u0, u1), q_edge_v(f, v1, u0, u1)));
    return m <= f.t;
}
__device__ __forceinline__ uint32_t quad_mask_foot(const SplatFoot& f, int x0, int y0)
{
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < 4; q++)
        if (foot_touches(f, (float)(x0 + 8 * (q & 1)), (float)(y0 + 8 * (q >> 1)))) m |= 1u << q;
    return m;
}
__device__ __forceinline__ uint32_t quad_mask(float x, float y, float4 co, float thr, int x0, int y0)
{
    return quad_mask_foot(splat_foot(x, y, co, thr), x0, y0);
}
// The same footprint test in band form, for the key scatter, which classifies every (Gaussian, tile) instance: per
// 8-row band of the tile, the exact x-extent of the footprint ellipse Q <= t inside the band (the ellipse's
// rightmost / leftmost point clamped into the band, where the concave chord ends peak), widened by a tolerance far
// above the rounding of the float operations; an 8x8 block is reached iff that extent overlaps its columns.
// det = ac - b^2 is formed with Kahan's compensated product so it does not cancel for elongated splats.  The extents
// are set up once per tile row of the rect (row_bands), so a tile costs four interval tests instead of sixteen edge
// minimisations.  tools/cull_check.py checks it against brute force like foot_touches.
// Every operation is IEEE-rounded (correctly rounded square roots and divisions, no contraction; fmaf where written),
// so the oracle's restatement (oracle/hlgs_oracle.c rect_quad_masks) computes the same masks bit for bit: with
// HLGS_DROP_EMPTY the masks decide which instances are binned, and the oracle's tile lists must match.
struct SplatBands {
    float x, y, nb, det, at, ia, vmax, vr, tol;
    int mode;  // as SplatFoot
};
__device__ __forceinline__ SplatBands splat_bands(float x, float y, float4 co, float thr)
{
#pragma clang fp contract(off)
    const SplatFoot f = splat_foot(x, y, co, thr);
    SplatBands s;
    s.x = x; s.y = y;
    s.nb = s.det = s.at = s.ia = s.vmax = s.vr = s.tol = 0.f;
    s.mode = f.mode;
    if (f.mode) return s;
    const float a = co.x, b = co.y, c = co.z, t = f.t;
    const float bb = b * b, e = fmaf(-b, b, bb);  // e = bb - b^2 exactly
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
// The footprint's x-extent [umin, umax] (offsets from the centre) inside the band v in [v0, v0 + h] (h = 7: an 8-row
// band); empty: +-3e38.
__device__ __forceinline__ void band_extent(const SplatBands& s, float v0, float& umin, float& umax, float h = 7.f)
{
#pragma clang fp contract(off)
    const float lo = fmaxf(v0, -s.vmax), hi = fminf(v0 + h, s.vmax);
    if (!(lo <= hi)) { umin = 3e38f; umax = -3e38f; return; }  // empty: overlaps no column
    const float vR = __builtin_amdgcn_fmed3f(s.vr, lo, hi), vL = __builtin_amdgcn_fmed3f(-s.vr, lo, hi);
    umax = fmaf(s.nb, vR, sqrtf(fmaxf(fmaf(-s.det * vR, vR, s.at), 0.f))) * s.ia + s.tol;
    umin = fmaf(s.nb, vL, -sqrtf(fmaxf(fmaf(-s.det * vL, vL, s.at), 0.f))) * s.ia - s.tol;
}
// One tile row of a Gaussian's rect: the extents in its two 8-row bands, set up once for every tile of the row.
struct RowBands {
    float cx, lo0, hi0, lo1, hi1;
    int mode;
};
__device__ __forceinline__ RowBands row_bands(const SplatBands& s, int ty)
{
#pragma clang fp contract(off)
    RowBands r;
    r.cx = s.x;
    r.mode = s.mode;
    r.lo0 = r.lo1 = 3e38f;
    r.hi0 = r.hi1 = -3e38f;
    if (s.mode) return r;
    const float v0 = (float)(ty * HLGS_TILE) - s.y;
    band_extent(s, v0, r.lo0, r.hi0);
    band_extent(s, v0 + 8.f, r.lo1, r.hi1);
    return r;
}
// Quadrant mask of tile column tx in that row: bit q set iff band q >> 1 reaches columns of half q & 1.
__device__ __forceinline__ uint32_t row_quad_mask(const RowBands& r, int tx)
{
#pragma clang fp contract(off)
    if (r.mode) return r.mode == 1 ? 0xFu : 0u;
    const float u0 = (float)(tx * HLGS_TILE) - r.cx, u7 = u0 + 7.f, u8 = u0 + 8.f, u15 = u0 + 15.f;
    return (r.hi0 >= u0 && r.lo0 <= u7 ? 1u : 0u) | (r.hi0 >= u8 && r.lo0 <= u15 ? 2u : 0u) |
           (r.hi1 >= u0 && r.lo1 <= u7 ? 4u : 0u) | (r.hi1 >= u8 && r.lo1 <= u15 ? 8u : 0u);
}

// Quadrant masks of the first kRectMasks tiles of a splat's rect (row-major from (x0, y0), width x1 - x0), nibble r for
// rect tile r: set up by the preprocess, which holds the splat's footprint anyway, and kept in Geom::qmask.
constexpr int kRectMasks = 8;
__device__ __forceinline__ uint32_t rect_quad_masks(float x, float y, float4 co, float thr, int x0, int y0, int x1, int y1)
{
    const SplatBands s = splat_bands(x, y, co, thr);
    const int w = x1 - x0, n = min((x1 - x0) * (y1 - y0), kRectMasks);
    uint32_t m = 0;
    RowBands row;
    for (int r = 0; r < n; r++) {
        const int ty = y0 + r / w, tx = x0 + r % w;
        if (r == 0 || tx == x0) row = row_bands(s, ty);
        m |= row_quad_mask(row, tx) << (4 * r);
    }
    return m;
}
// The quadrant mask of rect tile r from the record's masks; tiles past kRectMasks take every quadrant (conservative).
__device__ __forceinline__ uint32_t rect_tile_mask(uint32_t masks, uint32_t r)
{
    return r < (uint32_t)kRectMasks ? (masks >> (4 * r)) & 0xFu : 0xFu;
}

// Splat falloff in base 2.  conic_q pre-scales the conic by -log2(e) * (1/2, 1, 1/2); splat_e2 returns
// power * log2(e) for the reference's power = -(a dx^2 + c dy^2)/2 - b dx dy (forward.cu:377-379), with
// one fixed operation order so the forward and backward blends make identical alpha decisions.
__device__ __forceinline__ float4 conic_q(float4 co)
{
    constexpr float kL2E = 1.4426950408889634f;
    return make_float4(-0.5f * kL2E * co.x, -kL2E * co.y, -0.5f * kL2E * co.z, co.w);
}
__device__ __forceinline__ float splat_e2(float4 q, float dx, float dy)
{
    return fmaf(q.z * dy, dy, fmaf(q.y, dy, q.x * dx) * dx);
}

// The reference skips a pair when alpha < 1/255 (forward.cu:560, backward.cu:643).  Float alpha depends
// on the exp implementation, and for elongated splats the float power itself carries ~1e-3 relative error
// (the quadratic form cancels), so a float test would make different implementations keep different
// splats.  Instead, with e2 = power * log2(e) evaluated in one fixed IEEE operation order (splat_e2 --
// bit-identical here and in the oracle), "alpha >= 1/255" is decided as e2 >= thr, where thr is the
// smallest float at or above the exact real threshold: -log2(255 o) (the 0.99 clamp cannot matter), or,
// with hierarchy interpolation, log2(a_star / o) for the a_star that makes t a + (1 - t)(1 - (1 - a)^fr) = 1/255.
// thr is computed once per Gaussian in double (preprocess; oracle alpha_e2_threshold), so the blend's
// keep/skip test is a single float compare with identical results everywhere.
__device__ inline float alpha_e2_threshold(float o, bool interp, float t, float fr)
{
    if (o != o) return -INFINITY;          // NaN opacity: the reference's fminf(0.99, NaN) keeps the pair
    if (!(o > 0.f)) return INFINITY;       // alpha <= 0 never reaches 1/255
    const double target = 1.0 / 255.0;
    double a = target;
    if (interp) {
        const double td = t, fd = fr;
        auto g = [&](double x) { return td * x + (1.0 - td) * (1.0 - pow(1.0 - x, fd)); };
        if (g(0.99) < target) return INFINITY;
        double lo = 0.0, hi = 0.99;        // g is increasing: bisect to double resolution
        for (int i = 0; i < 64; i++) {
            const double mid = 0.5 * (lo + hi);
            if (g(mid) >= target) hi = mid; else lo = mid;
        }
        a = hi;
    }
    const double thr = log2(a / (double)o);
    float f = (float)thr;
    if ((double)f < thr) f = nextafterf(f, INFINITY);
    return f;
}

// Alt rasterizer's exact per-tile culling (alt-rasterizer/cuda_rasterizer/rasterizer_impl.cu:52-101 with
// PATCH = 15, applied at :147-179): the instance (Gaussian, tile (tx, ty)) exists only if the power at the
// point of the tile's pixel box the reference takes as the closest one does not exceed log(o / (1/255)).
// The binning and the backward's record reduction must decide identically, so the float operations keep the
// reference's order with contraction off in every translation unit; the logarithm is taken in double and
// rounded (the oracle's alt_tile_keep does the same), co = conic a, b, c and opacity.
__device__ __forceinline__ float alt_keep_threshold(float o)
{
    return (float)log((double)(o / (1.0f / 255.0f)));
}
// The per-Gaussian constants of the test, computed once per Gaussian instead of once per tile (round 5: the two IEEE
// divisions were half of each tile's instructions): the threshold and the reciprocals 1 / (225 a), 1 / (225 c).
struct AltKeep {
    float thr, rcx, rcz;
};
__device__ __forceinline__ AltKeep alt_keep_prep(float4 co)
{
#pragma clang fp contract(off)
    AltKeep k;
    k.thr = alt_keep_threshold(co.w);
    k.rcx = 1.0f / (225.0f * co.x);  // __frcp_rn: IEEE reciprocal
    k.rcz = 1.0f / (225.0f * co.z);
    return k;
}
__device__ __forceinline__ bool alt_tile_keep(float mx, float my, float4 co, const AltKeep& kp, int tx, int ty)
{
#pragma clang fp contract(off)
    const float rminx = (float)(tx * HLGS_TILE), rminy = (float)(ty * HLGS_TILE);
    const float rmaxx = (float)((tx + 1) * HLGS_TILE - 1), rmaxy = (float)((ty + 1) * HLGS_TILE - 1);
    const float x_min_diff = rminx - mx;
    const float x_left = x_min_diff > 0.0f ? 1.0f : 0.0f;
    const float not_in_x = x_left + (mx > rmaxx ? 1.0f : 0.0f);
    const float y_min_diff = rminy - my;
    const float y_above = y_min_diff > 0.0f ? 1.0f : 0.0f;
    const float not_in_y = y_above + (my > rmaxy ? 1.0f : 0.0f);
    float power = 0.0f;
    if ((not_in_y + not_in_x) > 0.0f) {
        const float px = x_left * rminx + (1.0f - x_left) * rmaxx;
        const float py = y_above * rminy + (1.0f - y_above) * rmaxy;
        const float dx = copysignf(15.0f, x_min_diff), dy = copysignf(15.0f, y_min_diff);
        const float diffx = mx - px, diffy = my - py;
        float sx = (dx * co.x * diffx + dx * co.y * diffy) * kp.rcx;
        float sy = (dy * co.y * diffx + dy * co.z * diffy) * kp.rcz;
        sx = sx != sx ? 0.0f : fminf(fmaxf(sx, 0.0f), 1.0f);  // __saturatef (NaN -> 0)
        sy = sy != sy ? 0.0f : fminf(fmaxf(sy, 0.0f), 1.0f);
        const float qx = px + not_in_y * sx * dx, qy = py + not_in_x * sy * dy;
        const float ddx = mx - qx, ddy = my - qy;
        power = 0.5f * (co.x * ddx * ddx + co.z * ddy * ddy) + co.y * ddx * ddy;
    }
    return power <= kp.thr;
}

// Does the alpha >= 1/255 footprint of a splat (see quad_mask) reach the 8x8 pixel block at (qx, qy)?
__device__ __forceinline__ bool touches_quad(float x, float y, float4 co, float thr, float qx, float qy)
{
    return foot_touches(splat_foot(x, y, co, thr), qx, qy);
}

// Copy n rows of M3 floats between global memory (row r at base + rows[r] * M3) and LDS (row r at
// lds + r * kShStride) with all 64 lanes on consecutive floats / float4s of the block's rows.
constexpr int kShStride = 49;  // odd stride: the per-thread row walks hit 64 distinct banks
template <int M3T, bool TO_LDS>  // M3T = 0: row length m3 known only at run time
__device__ __forceinline__ void sh_rows_copy(float* gbase, float* lds, const int* rows, int n, int lane, int m3)
{
    const int M3 = M3T ? M3T : m3;
    if constexpr (M3T > 0 && M3T % 4 == 0) {
        constexpr int M3 = M3T;
        constexpr int Q = M3 / 4;
        for (int f = lane; f < n * Q; f += 64) {
            const int r = f / Q, q = f - r * Q;
            float4* gp = reinterpret_cast<float4*>(gbase + (size_t)rows[r] * M3) + q;
            float* lp = lds + r * kShStride + 4 * q;
            if (TO_LDS) {
                const float4 v = *gp;
                lp[0] = v.x; lp[1] = v.y; lp[2] = v.z; lp[3] = v.w;
            } else {
                *gp = make_float4(lp[0], lp[1], lp[2], lp[3]);
            }
        }
    } else {
        for (int f = lane; f < n * M3; f += 64) {
            const int r = f / M3, q = f - r * M3;
            float* gp = gbase + (size_t)rows[r] * M3 + q;
            if (TO_LDS) lds[r * kShStride + q] = *gp;
            else *gp = lds[r * kShStride + q];
        }
    }
}

// Global -> LDS copy of n rows like sh_rows_copy<.., true>, with every global load of the wave issued before
// its first LDS store (registers hold the rows in flight), so a wave waits for HBM once, not once per float4.
// live (optional, LDS): rows r with live[r] == 0 are not read and land in LDS as zeros.
template <int M3T>
__device__ __forceinline__ void sh_rows_load(const float* gbase, float* lds, const int* rows, int n, int lane, int m3,
                                             const int* live = nullptr)
{
    if constexpr (M3T > 0 && M3T % 4 == 0) {
        constexpr int Q = M3T / 4;
        float4 v[Q];
#pragma unroll
        for (int k = 0; k < Q; k++) {
            const int f = lane + 64 * k;
            v[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (f < n * Q) {
                const int r = f / Q, q = f - r * Q;
                if (!live || live[r]) v[k] = reinterpret_cast<const float4*>(gbase + (size_t)rows[r] * M3T)[q];
            }
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
        constexpr int B = 12;
        for (int f0 = 0; f0 < n * M3; f0 += 64 * B) {
            float v[B];
#pragma unroll
            for (int k = 0; k < B; k++) {
                const int f = f0 + lane + 64 * k;
                v[k] = 0.f;
                if (f < n * M3) {
                    const int r = f / M3, q = f - r * M3;
                    if (!live || live[r]) v[k] = gbase[(size_t)rows[r] * M3 + q];
                }
            }
#pragma unroll
            for (int k = 0; k < B; k++) {
                const int f = f0 + lane + 64 * k;
                if (f < n * M3) {
                    const int r = f / M3, q = f - r * M3;
                    lds[r * kShStride + q] = v[k];
                }
            }
        }
    }
}

// Bijective XCD-aware block remap (cdna_hip_programming.md section 5): consecutive logical blocks
// land on the same XCD so neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg)
{
    const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// Its inverse: the workgroup whose xcd_remap is i (the i-th in XCD-grouped order).
__device__ __forceinline__ int xcd_unmap(int i, int nwg)
{
    const int q = nwg / 8, r = nwg % 8;
    if (q == 0) return i;  // fewer than 8 workgroups: the identity (and no division by q for positions past nwg)
    int x, k;
    if (i < r * (q + 1)) {
        x = i / (q + 1);
        k = i - x * (q + 1);
    } else {
        const int j = i - r * (q + 1);
        x = r + j / q;
        k = j - (x - r) * q;
    }
    return x + 8 * k;
}

// One DPP lane permutation of v (ctrl: quad_perm / row_ror / row_bcast encodings).
template <int CTRL, int ROW, bool BC>
__device__ __forceinline__ float dpp(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW, 0xF, BC));
}

// Reduce-scatter of ten per-lane values over the wave, cheapest stages first (issue costs measured by
// tools/issue_probe.hip: a DPP add 4.2 cycles per wave instruction, a permlane swap 8.3).  Each fold halves the number
// of registers: within each 16-lane row, bank-masked DPP adds fold lanes l and l^8 (values 2i into lanes 0-7, 2i+1 into
// lanes 8-15), then l and l^4 (per 4-lane bank); permlane32 / permlane16 swaps fold the halves and the row pairs; a
// quad_perm full reduction finishes each bank.  18 DPP + 3 permlane swaps, where ten full-wave reductions take
// 12 DPP + 8 permlane swaps.  (row_ror:n: lane l reads lane l - n of its row.)  The result w holds, in every lane of
// row rho and bank beta (lane = 16 rho + 4 beta + i), the total of value reduce10_index(rho, beta), or nothing for
// rho = 3.
__device__ __forceinline__ int reduce10_index(int rho, int beta)
{
    const int cb = ((beta & 1) << 1) | (beta >> 1);  // 0, 2, 1, 3
    return rho == 0 ? cb : rho == 2 ? 4 + cb : rho == 1 ? ((beta & 1) ? -1 : 8 + (beta >> 1)) : -1;
}
// One instruction stream, ordered so that every DPP / permlane-swap source was written at least two instructions
// earlier where the sequence allows it (the gfx950 VALU-write -> DPP-read and -> permlane-swap-read hazards need two
// wait states): 4 s_nop where the builtin-and-asm version took 7.
__device__ __forceinline__ float wave_reduce10_rs(const float (&v)[10])
{
    float s0, s1, s2, s3, s4, t0, t1, t2, z, w;
#define HLGS_FOLD8(d, a, b)                                                                                        \
    "v_add_f32_dpp " d ", " a ", " a " row_ror:8 row_mask:0xf bank_mask:0x3\n\t"                                  \
    "v_add_f32_dpp " d ", " b ", " b " row_ror:8 row_mask:0xf bank_mask:0xc\n\t"
#define HLGS_FOLD4(d, a, b)                                                                                        \
    "v_add_f32_dpp " d ", " a ", " a " row_ror:12 row_mask:0xf bank_mask:0x5\n\t"                                 \
    "v_add_f32_dpp " d ", " b ", " b " row_ror:4 row_mask:0xf bank_mask:0xa\n\t"
    asm volatile("s_nop 0\n\t"
                 "v_mov_b32 %8, 0\n\t"
                 HLGS_FOLD8("%0", "%10", "%11") HLGS_FOLD8("%1", "%12", "%13") HLGS_FOLD8("%2", "%14", "%15")
                 HLGS_FOLD8("%3", "%16", "%17") HLGS_FOLD8("%4", "%18", "%19")
                 HLGS_FOLD4("%6", "%2", "%3") HLGS_FOLD4("%5", "%0", "%1") HLGS_FOLD4("%7", "%4", "%4")
                 "v_permlane32_swap_b32 %5, %6\n\t"   // t0 (written two instructions back), t1
                 "v_add_f32 %5, %5, %6\n\t"           // rows 0-1: t0, rows 2-3: t1
                 "v_permlane32_swap_b32 %7, %8\n\t"   // t2 (two back), 0
                 "v_add_f32 %7, %7, %8\n\t"           // rows 0-1: t2, rows 2-3: 0
                 "s_nop 1\n\t"
                 "v_permlane16_swap_b32 %5, %7\n\t"
                 "v_add_f32 %9, %5, %7\n\t"           // row 0: t0, row 1: t2, row 2: t1, row 3: 0
                 "s_nop 1\n\t"
                 "v_add_f32_dpp %9, %9, %9 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
                 "s_nop 1\n\t"
                 "v_add_f32_dpp %9, %9, %9 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf"
                 : "=&v"(s0), "=&v"(s1), "=&v"(s2), "=&v"(s3), "=&v"(s4), "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(z),
                   "=&v"(w)
                 : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]), "v"(v[8]),
                   "v"(v[9]));
#undef HLGS_FOLD8
#undef HLGS_FOLD4
    return w;
}

}  // namespace hlgs
