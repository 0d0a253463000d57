// raster_bwd.hip -- the blend backward for gfx950 (the per-Gaussian kernels are in gauss_bwd.hip).
//
// Reference semantics (submodules/hierarchy-rasterizer/cuda_rasterizer):
//   k_blend_bwd  <- renderCUDA<3> backward      backward.cu:498-721
//
// The reference issues one global float atomic per (pixel, Gaussian, gradient component)
// (backward.cu:669-718).  Here each wave owns one tile (one chunk of its list): every 16-lane row folds its pixels'
// moments with DPP adds, the rows' totals meet in LDS, and the per-(tile, Gaussian) partial is stored once -- with a
// plain store -- into a Gaussian-major record slot (the Gaussian's point_offsets range, indexed by the tile's position
// inside its rect).  k_gauss_bwd then sums each Gaussian's contiguous records in a fixed order, so the backward has
// no global float atomics and is bitwise reproducible.
//
// The measured variants of rounds 1-4 (wave-wide quadrant passes, two splats per reduction, opacity-uniform clamp
// branches, packed moments, Newton reciprocals, tile-major chunk order, non-temporal loads and stores, and the
// traffic-attribution builds) are kept outside the product source as tools/variants/raster_bwd_r04.hip, built for A/B
// by tools/build_variant.py; DESIGN.md section 5 records each result.
#include "hlgs_internal.h"
#include "hlgs_math.h"

namespace hlgs {

// The blend backward's 4x4 sub-block masks of one tile (origin tx0, ty0 in pixels): bit 4 k + g is set iff the footprint
// reaches sub-block g (x half g & 1, y half g >> 1) of 8x8 quadrant k -- per 4-row band the footprint's x-extent (the
// band form above with 4-row bands: the same tolerances, so just as conservative; tools/cull_check.py checks both
// block sizes against brute force), tested against the band's four 4-column blocks.  Only a culling superset: the
// backward decides every pair with the exact e2 >= thr test.
__device__ __forceinline__ uint32_t sub_block_mask(const SplatBands& s, int tx0, int ty0)
{
#pragma clang fp contract(off)
    if (s.mode) return s.mode == 1 ? 0xFFFFu : 0u;
    const float u0 = (float)tx0 - s.x;
    uint32_t m = 0;
#pragma unroll
    for (int band = 0; band < 4; band++) {
        float lo, hi;
        band_extent(s, (float)(ty0 + 4 * band) - s.y, lo, hi, 3.f);
#pragma unroll
        for (int col = 0; col < 4; col++) {
            const float c0 = u0 + (float)(4 * col);
            const int k = (col >> 1) + 2 * (band >> 1), g = (col & 1) + 2 * (band & 1);
            if (hi >= c0 && lo <= c0 + 3.f) m |= 1u << (4 * k + g);
        }
    }
    return m;
}
// The same for one 8x8 quadrant at (qx0, qy0): bit g = sub-block g (x half g & 1, y half g >> 1) is reached.
__device__ __forceinline__ uint32_t quad_sub_mask(const SplatBands& s, int qx0, int qy0)
{
#pragma clang fp contract(off)
    if (s.mode) return s.mode == 1 ? 0xFu : 0u;
    const float u0 = (float)qx0 - s.x;
    uint32_t m = 0;
#pragma unroll
    for (int band = 0; band < 2; band++) {
        float lo, hi;
        band_extent(s, (float)(qy0 + 4 * band) - s.y, lo, hi, 3.f);
#pragma unroll
        for (int col = 0; col < 2; col++) {
            const float c0 = u0 + (float)(4 * col);
            if (hi >= c0 && lo <= c0 + 3.f) m |= 1u << (col + 2 * band);
        }
    }
    return m;
}
// The quadrant bits of a 4-bit mask spread over their four sub-block bits (bit k -> bits 4 k .. 4 k + 3).
__device__ __forceinline__ uint32_t quad_to_sub(uint32_t qm)
{
    return ((qm & 1u) ? 0xFu : 0u) | ((qm & 2u) ? 0xF0u : 0u) | ((qm & 4u) ? 0xF00u : 0u) | ((qm & 8u) ? 0xF000u : 0u);
}

// Ten per-lane values summed over each 16-lane row of the wave (rows independently: in the blend backward each row is one
// 4x4 sub-block working on its own splat).  Bank-masked DPP adds fold lanes l and l^8 (values 2i into banks 0-1, 2i+1
// into banks 2-3), then l and l^4 (FOLD4: five values into three), and two quad_perm adds finish each bank: 22 DPP
// adds.  Every lane of bank beta then holds t0 = the row total of value {0, 2, 1, 3}[beta], t1 = of {4, 6, 5, 7}[beta]
// and t2 = of {8, 8, 9, 9}[beta] (tools/diag/reduce_layout.py simulates the lane operations).  A row whose lanes are
// inactive (exec) is left alone: DPP row operations read within the row only.
__device__ __forceinline__ void row_reduce10(const float (&v)[10], float& t0, float& t1, float& t2)
{
    float s0, s1, s2, s3, s4;
#define HLGS_FOLD8(d, a, b)                                                                                        \
    "v_add_f32_dpp " d ", " a ", " a " row_ror:8 row_mask:0xf bank_mask:0x3\n\t"                                  \
    "v_add_f32_dpp " d ", " b ", " b " row_ror:8 row_mask:0xf bank_mask:0xc\n\t"
#define HLGS_FOLD4(d, a, b)                                                                                        \
    "v_add_f32_dpp " d ", " a ", " a " row_ror:12 row_mask:0xf bank_mask:0x5\n\t"                                 \
    "v_add_f32_dpp " d ", " b ", " b " row_ror:4 row_mask:0xf bank_mask:0xa\n\t"
#define HLGS_QUAD(d, p) "v_add_f32_dpp " d ", " d ", " d " quad_perm:" p " row_mask:0xf bank_mask:0xf\n\t"
    // every DPP source was written at least two instructions earlier (the VALU-write -> DPP-read hazard), except the
    // inputs, hence the leading s_nop
    asm volatile("s_nop 1\n\t"
                 HLGS_FOLD8("%0", "%8", "%9") HLGS_FOLD8("%1", "%10", "%11") HLGS_FOLD8("%2", "%12", "%13")
                 HLGS_FOLD8("%3", "%14", "%15") HLGS_FOLD8("%4", "%16", "%17")
                 HLGS_FOLD4("%5", "%0", "%1") HLGS_FOLD4("%6", "%2", "%3") HLGS_FOLD4("%7", "%4", "%4")
                 HLGS_QUAD("%5", "[1,0,3,2]") HLGS_QUAD("%6", "[1,0,3,2]") HLGS_QUAD("%7", "[1,0,3,2]")
                 HLGS_QUAD("%5", "[2,3,0,1]") HLGS_QUAD("%6", "[2,3,0,1]") HLGS_QUAD("%7", "[2,3,0,1]")
                 : "=&v"(s0), "=&v"(s1), "=&v"(s2), "=&v"(s3), "=&v"(s4), "=&v"(t0), "=&v"(t1), "=&v"(t2)
                 : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]), "v"(v[8]),
                   "v"(v[9]));
#undef HLGS_FOLD8
#undef HLGS_FOLD4
#undef HLGS_QUAD
}
// The moment whose row total lane position (bank beta = (l >> 2) & 3, p = l & 3) stores after row_reduce10: p = 0 -> t0,
// p = 1 -> t1, p = 2 -> t2 in banks 0 and 2; -1: none.
__host__ __device__ inline int row_reduce10_index(int beta, int p)
{
    const int cb = ((beta & 1) << 1) | (beta >> 1);  // 0, 2, 1, 3
    return p == 0 ? cb : p == 1 ? 4 + cb : (p == 2 && !(beta & 1)) ? 8 + (beta >> 1) : -1;
}


// Per-pixel state of the back-to-front replay (backward.cu:549-572).  The reference keeps the
// accumulated colour/inverse-depth behind the current splat and the previous splat's alpha and colour
// (accum_rec, last_alpha, last_color) only to form dL/dalpha = <c - accum, dL/dpixel>, which is linear
// in the accumulators; so one scalar ARD = <accum, dL/dpixel> (+ depth term), updated by the current
// splat once its own step is done, carries the same information.
//
// The background term of dL/dalpha, -T_final <bg, dL/dpixel> / (1 - alpha) (backward.cu:688-691), rides along in ARD:
// with ARD' = ARD + T_final <bg, dL/dpixel> / T_behind (T_behind = transmittance behind the current splat), the
// recursion is unchanged (T_final bgd / T_i = (1 - alpha_i) T_final bgd / T_behind) and dL/dalpha = T (cd - ARD'),
// so the step needs no product with 1/(1 - alpha) beyond the transmittance update.
struct PixB {
    float T;                 // transmittance in front of the current splat
    float ARD;               // <accum_rec, dL/dpixel> + accum_invdepth * dL/dinvdepth + T_final <bg, dL/dpixel> / T_behind
    float dr, dg, db, dinv;  // dL/dpixel, dL/dinvdepth
    uint32_t last;           // n_contrib
};

// 1 if o G <= 0.99, else 0: the reference's dL/dalpha = 0 above the alpha clamp (backward.cu:619, 693) as a factor.
// fma(-2^40, ta, 2^40 next(0.99f)) is exactly 2^40 (next(0.99f) - ta) for ta near 0.99f (both operands scaled by a
// power of two), so it is >= 2^16 (one ulp of 0.99f, scaled) for ta <= 0.99f and <= 0 for ta > 0.99f; the clamp makes
// it 1 or 0 (NaN -> 0).  2^40 next(0.99f) = 1088516587520 is exact in float32 (tests/test_gpu_parity.py::
// test_alpha_clamp_threshold_exact checks prev(0.99f), 0.99f, next(0.99f) and next(next(0.99f))).
__device__ __forceinline__ float below_clamp(float test_alpha)
{
    return __builtin_amdgcn_fmed3f(fmaf(-1099511627776.0f, test_alpha, 1088516587520.0f), 0.f, 1.f);
}

// One (pixel, splat) step of renderCUDA backward (backward.cu:601-718).  The splat's gradient terms
// are linear in w = G * dL/dalpha and its moments over the pixels,
//   dL/dmean2D = -o * (conic * [Sum w dx, Sum w dy]) * (W/2, H/2),
//   dL/dconic  = -o/2 * [Sum w dx^2, Sum w dx dy, Sum w dy^2],   dL/dopacity = Sum w (x mult if lerped),
// so each pixel adds ten moments to acc and finish_record() applies the per-splat factors once.
//   acc = [Sum w dx, Sum w dy, Sum w dx^2, Sum w dx dy, Sum w dy^2, Sum w*mult, dcolor r g b, dinvdepth]
// q = (-a/2, -b, -c/2) * log2(e) so that G = exp2(q0 dx^2 + q1 dx dy + q2 dy^2) = exp(power).
// ALT: the alt rasterizer's backward (alt-rasterizer/cuda_rasterizer/backward.cu:596-624) has no
// o * G > 0.99 => dL/dalpha = 0 rule; its doubled background term is folded into ARD by the caller.
//
// The pair step in two halves.  The front (falloff, alpha, 1/(1 - alpha), the threshold tests) depends on the pair
// alone; the back (transmittance, ARD and the moments) on the pixel's replay state.
struct BwdFront {
    float G, alpha, r1m, my_alpha, dx, dy;
    uint64_t ok;  // wave mask: alpha >= 1/255 (alpha_e2_threshold)
};

template <bool INTERP, bool ALT>
__device__ __forceinline__ BwdFront bwd_front(float dx, float dy, const float4& q, float tt, float fr, float thr)
{
    BwdFront f;
    f.dx = dx;
    f.dy = dy;
    const float e2 = splat_e2(q, dx, dy);  // power * log2(e)
    float G = __builtin_amdgcn_exp2f(e2);
    const float test_alpha = q.w * G;
    f.my_alpha = fminf(0.99f, test_alpha);
    f.alpha = f.my_alpha;
    if (INTERP) f.alpha = tt * f.my_alpha + (1.0f - tt) * (1.0f - powf(1.0f - f.my_alpha, fr));
    f.r1m = __builtin_amdgcn_rcpf(1.f - f.alpha);
    if (!ALT) {
        float b = below_clamp(test_alpha);
        asm volatile("" : "+v"(b));  // not speculatable: a scalar branch around two VALU, not a select after them
        G *= b;
    }
    f.G = G;
    // as wave masks: one v_cmp per test, combined in SALU
    f.ok = ~__builtin_amdgcn_ballot_w64(e2 > 0.0f) & ~__builtin_amdgcn_ballot_w64(e2 < thr);
    return f;
}

template <bool INTERP, bool DEPTH>
__device__ __forceinline__ void bwd_back(PixB& p, uint32_t li, const BwdFront& f, const float4& col, float invz, float tt,
                                         float fr, float (&acc)[10])
{
    const uint64_t valid = __builtin_amdgcn_ballot_w64(li < p.last) & f.ok;
    if (__builtin_amdgcn_inverse_ballot_w64(valid)) {
        const float alpha = f.alpha, dx = f.dx, dy = f.dy;
        p.T = p.T * f.r1m;
        const float weight = alpha * p.T;
        // <colour, dL/dpixel> stays uncontracted: it feeds dL/dalpha and through it the ill-conditioned conic ->
        // scale / rotation chain, where contracting it moved the GPU further from the oracle than the oracle's own
        // contracted build is (tests/test_gpu_configs.py).  The colour / depth moments feed only dL/dcolour and
        // dL/ddepth and are contracted (four VALU fewer per pass).
        float cd = col.x * p.dr + col.y * p.dg + col.z * p.db;
        if (DEPTH) cd += invz * p.dinv;
        const float raw = cd - p.ARD;
        p.ARD = fmaf(alpha, raw, p.ARD);
        acc[6] = fmaf(weight, p.dr, acc[6]);
        acc[7] = fmaf(weight, p.dg, acc[7]);
        acc[8] = fmaf(weight, p.db, acc[8]);
        if (DEPTH) acc[9] = fmaf(weight, p.dinv, acc[9]);
        const float dL_dalpha = raw * p.T;
        const float w = f.G * dL_dalpha;
        const float wdx = w * dx, wdy = w * dy;
        acc[0] += wdx;
        acc[1] += wdy;
        acc[2] = fmaf(wdx, dx, acc[2]);
        acc[3] = fmaf(wdx, dy, acc[3]);
        acc[4] = fmaf(wdy, dy, acc[4]);
        if (INTERP) acc[5] += (tt - powf(1.0f - f.my_alpha, fr - 1.0f) * (tt - 1.0f) * fr) * w;
        else acc[5] += w;
    }
}

// Per-splat record from the reduced moments (see bwd_back); co = conic and opacity of the splat.
__device__ __forceinline__ void finish_record(const float* m, float4 co, float ddelx_dx, float ddely_dy, float4& ra,
                                              float4& rb, float2& rc)
{
    const float o = co.w;
    ra.x = -o * (co.x * m[0] + co.y * m[1]) * ddelx_dx;
    ra.y = -o * (co.z * m[1] + co.y * m[0]) * ddely_dy;
    ra.z = -0.5f * o * m[2];
    ra.w = -0.5f * o * m[3];
    rb.x = -0.5f * o * m[4];
    rb.y = m[5];
    rb.z = m[6];
    rb.w = m[7];
    rc.x = m[8];
    rc.y = m[9];
}

struct BwdArgs {
    const uint2* ranges;
    const uint32_t* point_list;
    int W, H, gx, gy, T;
    Geom g;
    const float* final_Ts;
    const uint32_t* n_contrib;
    const float* split_state;
    const float* bg;
    const float* dL_dpixels;
    const float* dL_dinvdepths;
    BwdScratch rec;
    const uint32_t* misc;  // Img::misc of the forward: [kMiscPack] says whether its point_list entries are packed
};

// One wave per (tile, chunk of the tile's list), back to front.  Chunk c covers list entries [c clen, min(count,
// (c + 1) clen)) (bwd_chunk_len); blocks are ordered chunk-major, so the front chunks, where most pixels are still live,
// start first.  A pixel whose last contributor lies behind the chunk's end starts from the forward's sample there
// (transmittance, and what was blended behind it), otherwise from its final state, as the reference's single
// back-to-front pass has it at that point.
//
// Lanes and sub-blocks.  Lane l owns one pixel of each 8x8 quadrant k: 16-lane row g = l >> 4 is the 4x4 sub-block g of
// the quadrant (x half g & 1, y half g >> 1) and l & 15 the pixel inside it.  Each 64-splat batch is staged in LDS with
// a 16-bit sub-block mask per splat (sub_block_mask, intersected with the list entry's quadrant mask); per quadrant and
// sub-block, the splats that reach it and lie in front of its furthest contributor are listed in LDS, back to front.
// Then, per quadrant, every row walks its own sub-block's list: one iteration is one (splat, 4x4 sub-block) pair per row,
// the ten moments are folded over the row (row_reduce10) and the totals added into the splat's moments in LDS.  Rows
// whose list is done idle until the quadrant's longest list ends.  Against 8x8 passes with one wave-wide reduction
// per splat (round 4), this keeps 61% of the pass lanes busy instead of 36% (configs[1] frame, tools/fold_stats.py),
// and one row reduction costs 22 DPP adds where the wave reduction cost 24 instructions and 4 wait states.  After
// the batch, lane j finishes splat j's record and stores it.
// Moments of one splat meet by LDS float atomics (ds_add_f32).  Each is one instruction of one wave: the order in which
// the rows' totals arrive is fixed by the lists, so the sums are the same on every run.
constexpr int kMStride = 65;  // moment rows padded to 65 floats (moment v of splat j at v kMStride + j: distinct banks)
template <bool INTERP, bool DEPTH, bool ALT>
__global__ void __launch_bounds__(64, 5) k_blend_bwd(BwdArgs A)
{
    const int part = blockIdx.x / A.T;
    const int tile = xcd_remap(blockIdx.x - part * A.T, A.T);
    const uint2* __restrict__ ranges = A.ranges;
    const uint32_t* __restrict__ point_list = A.point_list;
    const int W = A.W, H = A.H, gx = A.gx;
    const Geom& g = A.g;
    const float* __restrict__ final_Ts = A.final_Ts;
    const uint32_t* __restrict__ n_contrib = A.n_contrib;
    const float* __restrict__ bg = A.bg;
    const float* __restrict__ dL_dpixels = A.dL_dpixels;
    const float* __restrict__ dL_dinvdepths = A.dL_dinvdepths;
    const BwdScratch& rec = A.rec;
    const uint32_t pack = __builtin_amdgcn_readfirstlane(A.misc[kMiscPack]);  // as the forward packed them
    __shared__ float4 s_sp[3 * 64];   // splat j: [j] x, y, 1/depth, -; [64 + j] conic_q, opacity; [128 + j] r, g, b, thr
    __shared__ float2 s_tf[64];       // interpolation t, 1/kids (hierarchy mode)
    __shared__ float s_m[10 * kMStride];
    __shared__ uint8_t s_list[16 * 64];  // per (quadrant k, sub-block g): the batch positions j, back to front
    __shared__ float4 s_zero[3];
    if (threadIdx.x < 3) s_zero[threadIdx.x] = make_float4(0.f, 0.f, 0.f, 0.f);  // ordered by the batch barrier
    const int lane = threadIdx.x, grp = lane >> 4;
    const int tx = tile % gx, ty = tile / gx;
    const int tx0 = tx * HLGS_TILE, ty0 = ty * HLGS_TILE;
    const uint2 range = ranges[tile];
    const uint32_t count = range.y - range.x;
    const uint32_t clen = bwd_chunk_len(count);
    const uint32_t c0 = (uint32_t)part * clen;  // chunk = local list positions [c0, cnt)
    if (c0 >= count) return;
    const uint32_t cnt = min(count, c0 + clen);
    // this lane's pixel inside each quadrant, and the forward's lane for it (its split-state column)
    const int qxl = 4 * (grp & 1) + (lane & 3), qyl = 4 * (grp >> 1) + ((lane >> 2) & 3);
    const float* __restrict__ st =
        cnt < count ? A.split_state + (size_t)(tile * kBwdSplits + part) * kSplitFloats + qxl + 8 * qyl : nullptr;
    const size_t HW = (size_t)H * W;
    const float ddelx_dx = 0.5f * W, ddely_dy = 0.5f * H;
    const float lx = (float)(tx0 + qxl), ly = (float)(ty0 + qyl);
    // the row total this lane adds into s_m (row_reduce10 layout), or none
    const int wm_i = row_reduce10_index((lane >> 2) & 3, lane & 3);
    const bool has_total = wm_i >= 0;
    const int wmd = has_total ? kMStride * wm_i : 0;
    const int psel = lane & 3;  // which of t0, t1, t2 it adds

    PixB ps[4];
    uint32_t slast[4];  // per quadrant, row-uniform: the furthest-back position any pixel of the row's sub-block needs
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int px = tx0 + 8 * (k & 1) + qxl, py = ty0 + 8 * (k >> 1) + qyl;
        const bool inside = px < W && py < H;
        const size_t pid = (size_t)W * py + px;
        PixB& p = ps[k];
        const float tf = inside ? final_Ts[pid] : 0.f;
        p.T = tf;
        p.last = inside ? n_contrib[pid] : 0u;
        p.dr = inside ? dL_dpixels[pid] : 0.f;
        p.dg = inside ? dL_dpixels[HW + pid] : 0.f;
        p.db = inside ? dL_dpixels[2 * HW + pid] : 0.f;
        p.dinv = (DEPTH && inside) ? dL_dinvdepths[pid] : 0.f;
        float bgd = 0.f;
        bgd += bg[0] * p.dr;
        bgd += bg[1] * p.dg;
        bgd += bg[2] * p.db;
        // the alt rasterizer's ar includes the final colour's T_final * bg and adds the bg term once more
        // (alt-rasterizer backward.cu:608, 619): the background enters dL/dalpha twice
        if (ALT) bgd *= 2.f;
        p.ARD = bgd;  // T_final <bg, dL/dpixel> / T_final
        if (p.last > cnt) {  // still blending at the chunk's end (so the forward sampled it there)
            const float* sk = st + k * 5 * 64;
            p.T = sk[0];
            float behind = sk[64] * p.dr + sk[128] * p.dg + sk[192] * p.db;
            if (DEPTH) behind += sk[256] * p.dinv;
            p.ARD = fmaf(tf, bgd, behind) / p.T;  // <accum_rec, dL/dpixel> (+ depth, + bg term) at the chunk's end
        }
        uint32_t m = min(p.last, cnt);
        for (int off = 8; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
        slast[k] = m;
    }
    // the same per (quadrant, sub-block) as scalars: sl[4 k + g]
    uint32_t sl[16];
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int r = 0; r < 4; r++) sl[4 * k + r] = __builtin_amdgcn_readlane(slast[k], 16 * r);
    uint32_t maxlast = 0;
#pragma unroll
    for (int b = 0; b < 16; b++) maxlast = max(maxlast, sl[b]);

    for (uint32_t b0 = 0; b0 < cnt - c0; b0 += 64) {
        // batch covers local positions cnt-1-b0 down to cnt-1-b0-(n-1), loaded back to front
        const int n = (int)min(64u, cnt - c0 - b0);
        const uint32_t li_top = cnt - 1 - b0;
        const bool lane_valid = lane < n;
        uint32_t slot = 0, sbm = 0;
        float4 my_co = make_float4(0.f, 0.f, 0.f, 0.f);
        if (lane_valid) {
            const uint32_t pos = range.x + li_top - lane;
            uint32_t id = point_list[pos], qm = 0xFu;
            if (pack) {  // packed entry (pack_entries): the quadrant mask comes with it
                qm = id & ((1u << kEntryShift) - 1u);
                id >>= kEntryShift;
            }
            const float4* sr = g.splat + 4 * (size_t)id;
            const uint32_t sbase = id ? g.point_offsets[id - 1] : 0u;
            const float4 r0 = sr[0], r1 = sr[1], r2 = sr[2], r3 = sr[3];
            const float4 co = make_float4(r0.z, r0.w, r1.x, r1.y);
            s_sp[lane] = make_float4(r0.x, r0.y, DEPTH ? r2.y : 0.f, 0.f);
            s_sp[64 + lane] = conic_q(co);
            s_sp[128 + lane] = make_float4(r1.z, r1.w, r2.x, r3.w);
            if (INTERP) s_tf[lane] = make_float2(r2.z, r2.w);
            my_co = co;
            sbm = sub_block_mask(splat_bands(r0.x, r0.y, co, r3.w), tx0, ty0) & quad_to_sub(qm);
            const int x0 = __float_as_int(r3.y) & 0xffff, y0 = (int)((uint32_t)__float_as_int(r3.y) >> 16);
            const int w = __float_as_int(r3.z);
            // the Gaussian's record slots start at the exclusive scan of the rect sizes (point_offsets is inclusive)
            slot = sbase + (uint32_t)((ty - y0) * w + (tx - x0));
        }
#pragma unroll
        for (int v = 0; v < 10; v++) s_m[kMStride * v + lane] = 0.f;
        // a batch entirely behind every pixel's last contributor leaves its records zero
        const uint32_t li_bot = li_top - (uint32_t)(n - 1);
        uint32_t nl[16];  // list lengths (scalars)
        if (li_bot < maxlast) {
            // splat j (this lane) goes to the list of sub-block b if its footprint reaches b and it lies in front of
            // b's furthest contributor (li < sl[b]); lists are in ascending j, i.e. back to front
            const uint32_t li = li_top - (uint32_t)lane;
#pragma unroll
            for (int b = 0; b < 16; b++) {
                const bool in = ((sbm >> b) & 1u) && li < sl[b];
                const uint64_t M = __builtin_amdgcn_ballot_w64(in);
                nl[b] = (uint32_t)__popcll(M);
                const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u));
                if (in) s_list[64 * b + rank] = (uint8_t)lane;
            }
        }
        __syncthreads();
        if (li_bot < maxlast) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t n0 = nl[4 * k], n1 = nl[4 * k + 1], n2 = nl[4 * k + 2], n3 = nl[4 * k + 3];
                const uint32_t nmax = max(max(n0, n1), max(n2, n3));
                const uint32_t myn = grp == 0 ? n0 : grp == 1 ? n1 : grp == 2 ? n2 : n3;
                const uint8_t* lst = s_list + 64 * (4 * k + grp);
                // Software pipeline over the row's list: iteration it works on splat j(it) while the LDS reads of splat
                // j(it + 1) and of list entry it + 2 are in flight (otherwise every iteration waits for two dependent
                // LDS round trips).  Reads past the list's end fetch unused entries (masked to a staged splat).
                int jn = lst[0] & 63, jnn = lst[1] & 63;
                float4 xy = s_sp[jn], q = s_sp[64 + jn], col = s_sp[128 + jn];
                float2 tf = INTERP ? s_tf[jn] : make_float2(0.f, 0.f);
                for (uint32_t it = 0; it < nmax; it++) {
                    if (it < myn) {
                        const int j = jn;
                        const float4 cxy = xy, cq = q, ccol = col;
                        const float2 ctf = tf;
                        jn = jnn;
                        jnn = lst[min(it + 2, 63u)] & 63;
                        xy = s_sp[jn];
                        q = s_sp[64 + jn];
                        col = s_sp[128 + jn];
                        if (INTERP) tf = s_tf[jn];
                        float acc[10];
                        {  // zeroed by three LDS reads of a zero block (the LDS pipe has room; the VALU pipe is the limit)
                            typedef float v4f __attribute__((ext_vector_type(4)));
                            typedef __attribute__((address_space(3))) const volatile v4f lds_v4f;  // stays a ds_read
                            lds_v4f* vz = (lds_v4f*)(s_zero);
                            const v4f z0 = vz[0], z1 = vz[1], z2 = vz[2];
                            acc[0] = z0.x; acc[1] = z0.y; acc[2] = z0.z; acc[3] = z0.w;
                            acc[4] = z1.x; acc[5] = z1.y; acc[6] = z1.z; acc[7] = z1.w;
                            acc[8] = z2.x; acc[9] = z2.y;
                        }
                        BwdFront f = bwd_front<INTERP, ALT>(cxy.x - (lx + 8.f * (k & 1)), cxy.y - (ly + 8.f * (k >> 1)), cq,
                                                            ctf.x, ctf.y, ccol.w);
                        // the front above the validity branch: its transcendental latency overlaps the compare -> SALU
                        // -> exec chain that decides the branch instead of following it
                        asm volatile("" : "+v"(f.G), "+v"(f.r1m), "+v"(f.alpha));
                        bwd_back<INTERP, DEPTH>(ps[k], li_top - (uint32_t)j, f, ccol, cxy.z, ctf.x, ctf.y, acc);
                        float t0, t1, t2;
                        row_reduce10(acc, t0, t1, t2);
                        const float t = psel == 0 ? t0 : psel == 1 ? t1 : t2;
                        if (has_total) atomicAdd(&s_m[wmd + j], t);
                    }
                }
            }
        }
        __syncthreads();
        if (lane_valid) {
            float m[10];
#pragma unroll
            for (int v = 0; v < 10; v++) m[v] = s_m[kMStride * v + lane];
            float4 ra, rb;
            float2 rc;
            finish_record(m, my_co, ddelx_dx, ddely_dy, ra, rb, rc);
            float4* r = rec.rec + 3 * (size_t)slot;
            r[0] = ra;
            r[1] = rb;
            r[2] = make_float4(rc.x, rc.y, 0.f, 0.f);
        }
        __syncthreads();
    }
}


void launch_blend_bwd(const hlgs_raster_args& a, const Geom& g, const Img& im, const Bin& b, const BwdScratch& rs,
                      int gx, int gy, const float* dL_dpix, const float* dL_dinv, hipStream_t s)
{
    const int T = gx * gy;
    const bool interp = a.ts != nullptr && a.kids != nullptr;
    BwdArgs A{im.ranges, b.point_list, a.W, a.H, gx, gy, T, g, im.final_T, im.n_contrib, im.split_state, a.bg, dL_dpix,
              dL_dinv, rs, im.misc};
#define HLGS_BB(I, Dp, Al) hipLaunchKernelGGL((k_blend_bwd<I, Dp, Al>), dim3((kBwdSplits + 1) * T), dim3(64), 0, s, A)
    if (a.variant == HLGS_VARIANT_ALT) { if (dL_dinv) HLGS_BB(false, true, true); else HLGS_BB(false, false, true); }
    else if (interp) { if (dL_dinv) HLGS_BB(true, true, false); else HLGS_BB(true, false, false); }
    else { if (dL_dinv) HLGS_BB(false, true, false); else HLGS_BB(false, false, false); }
#undef HLGS_BB
}


}  // namespace hlgs
