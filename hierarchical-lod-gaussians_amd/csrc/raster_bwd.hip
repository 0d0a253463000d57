// raster_bwd.hip -- the blend backward for gfx950 (the per-Gaussian kernels are in gauss_bwd.hip).
//
// Reference semantics (submodules/hierarchy-rasterizer/cuda_rasterizer):
//   k_blend_bwd  <- renderCUDA<3> backward      backward.cu:498-721
//
// The reference issues one global float atomic per (pixel, Gaussian, gradient component)
// (backward.cu:669-718).  Here each wave owns one tile: every lane folds its four pixels, a
// permlane/DPP reduce-scatter folds the 64 lanes, and the per-(tile, Gaussian) partial is stored once -- with
// a plain store -- into a Gaussian-major record slot (the Gaussian's point_offsets range, indexed by
// the tile's position inside its rect).  k_gauss_bwd then sums each Gaussian's contiguous records
// in a fixed order, so the backward has no float atomics and is bitwise reproducible.
//
// The measured variants of rounds 1-5 (two splats per reduction, opacity-uniform clamp branches, packed moments,
// Newton reciprocals, tile-major chunk order, non-temporal loads and stores, the traffic-attribution builds, and round
// 5's 4x4 sub-block lists) live outside the product source, in git history (tools/variants/INDEX.md: raster_bwd_r04.hip,
// raster_bwd_sub4.hip), built for A/B by tools/build_variant.py; DESIGN.md section 5 records each result.
#include "hlgs_internal.h"
#include "hlgs_math.h"


namespace hlgs {

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
    // as wave masks: one v_cmp per test, combined in SALU (the wave is full)
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

// One quadrant pass: the front is computed for every lane ahead of the validity branch, so its transcendental latency
// overlaps the compare -> SALU -> exec chain that decides the branch instead of following it.
template <bool INTERP, bool DEPTH, bool ALT, int K>
__device__ __forceinline__ void bwd_pass(PixB (&ps)[4], uint32_t li, float lx, float ly, const float4& xy, const float4& q,
                                         const float4& col, float2 tf, float (&acc)[10])
{
    BwdFront f = bwd_front<INTERP, ALT>(xy.x - (lx + 8.f * (K & 1)), xy.y - (ly + 8.f * (K >> 1)), q, tf.x, tf.y, col.w);
    asm volatile("" : "+v"(f.G), "+v"(f.r1m), "+v"(f.alpha));  // keep them above the branch
    bwd_back<INTERP, DEPTH>(ps[K], li, f, col, xy.z, tf.x, tf.y, acc);
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

// One wave per (tile, chunk of the tile's list), back to front; lane owns pixel (lane & 7, lane >> 3) of each 8x8
// quadrant.  Chunk c covers list entries [c clen, min(count, (c + 1) clen)) (bwd_chunk_len); blocks are ordered
// chunk-major, so the front chunks, where most pixels are still live, start first.  A pixel whose last contributor
// lies behind the chunk's end starts from the forward's sample there (transmittance, and what was blended behind
// it), otherwise from its final state, as the reference's single back-to-front pass has it at that point.  Each
// 64-splat batch is staged in LDS; per splat, the quadrants its footprint reaches (and that still hold a pixel
// whose n_contrib lies behind it) run bwd_pass, the ten moments are folded over the wave, and one record per
// (tile, splat) is stored after the batch.
// Round 5 measured 4x4 sub-block lists per 16-lane row here instead of 8x8 quadrant passes (raster_bwd_sub4.hip,
// tools/variants/INDEX.md): 61% of the pass lanes busy instead of 36%, but 697 against 354 us -- the per-row splat
// indices put six LDS round trips and an LDS float atomic on every iteration, and the LDS became the limit (SQ_LDS_IDX_ACTIVE
// 5.7x, SQ_WAIT_INST_LDS 256x); DESIGN.md section 5.
constexpr int kMStride = 65;  // moment rows padded to 65 floats (see s_m below)
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
    __shared__ float4 s_xy[64];   // x, y, 1/depth, unused
    __shared__ float4 s_q[64];    // -a/2, -b, -c/2 (times log2 e), opacity
    __shared__ float4 s_col[64];  // r, g, b, alpha threshold on e2
    __shared__ float2 s_tf[64];   // interpolation t, 1/kids
    // reduced moments per splat (+ a spare row the non-storing lanes write), rows padded to kMStride = 65 floats: the
    // ten lanes holding totals store moment v of splat j at kMStride v + j, on ten different banks ((v + j) mod 32),
    // where a 64-float stride put all ten (and the spare row) on bank j mod 32
    __shared__ float s_m[kMStride * 11];
    __shared__ float4 s_zero[3];
    if (threadIdx.x < 3) s_zero[threadIdx.x] = make_float4(0.f, 0.f, 0.f, 0.f);  // ordered by the batch barrier
    const int lane = threadIdx.x;
    const int tx = tile % gx, ty = tile / gx;
    const int tx0 = tx * HLGS_TILE, ty0 = ty * HLGS_TILE;
    const uint2 range = ranges[tile];
    const uint32_t count = range.y - range.x;
    const uint32_t clen = bwd_chunk_len(count);
    const uint32_t c0 = (uint32_t)part * clen;  // chunk = local list positions [c0, cnt)
    if (c0 >= count) return;
    const uint32_t cnt = min(count, c0 + clen);
    const float* __restrict__ st =
        cnt < count ? A.split_state + (size_t)(tile * kBwdSplits + part) * kSplitFloats + lane : nullptr;
    const size_t HW = (size_t)H * W;
    const float ddelx_dx = 0.5f * W, ddely_dy = 0.5f * H;
    const float lx = (float)(tx0 + (lane & 7)), ly = (float)(ty0 + (lane >> 3));
    // the reduced moment this lane stores (wave_reduce10_rs layout) as an offset into s_m; lanes holding no total
    // store into the spare row s_m[10 kMStride ..]
    const int wm_i = (lane & 3) ? -1 : reduce10_index(lane >> 4, (lane >> 2) & 3);
    const int wmd = wm_i < 0 ? 10 * kMStride : kMStride * wm_i;
    // lane owns pixel (lane & 7, lane >> 3) of each 8x8 quadrant k
    PixB ps[4];
    uint32_t qlast[4];  // wave-uniform per quadrant: furthest-back position any of its pixels needs
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int px = tx0 + 8 * (k & 1) + (lane & 7), py = ty0 + 8 * (k >> 1) + (lane >> 3);
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
        for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
        qlast[k] = __builtin_amdgcn_readfirstlane(m);
    }
    const uint32_t maxlast = max(max(qlast[0], qlast[1]), max(qlast[2], qlast[3]));

    for (uint32_t b0 = 0; b0 < cnt - c0; b0 += 64) {
        // batch covers local positions cnt-1-b0 down to cnt-1-b0-(n-1), loaded back to front
        const int n = (int)min(64u, cnt - c0 - b0);
        const uint32_t li_top = cnt - 1 - b0;
        const bool lane_valid = lane < n;
        uint32_t slot = 0, qm = 0;
        float4 my_co = make_float4(0.f, 0.f, 0.f, 0.f);
        if (lane_valid) {
            const uint32_t pos = range.x + li_top - lane;
            uint32_t id = point_list[pos], pm = 0;
            if (pack) {  // packed entry (pack_entries): the quadrant mask comes with it
                pm = id & ((1u << kEntryShift) - 1u);
                id >>= kEntryShift;
            }
            const float4* sr = g.splat + 4 * (size_t)id;
            const uint32_t sbase = id ? g.point_offsets[id - 1] : 0u;
            const float4 r0 = sr[0], r1 = sr[1], r2 = sr[2], r3 = sr[3];
            const float4 co = make_float4(r0.z, r0.w, r1.x, r1.y);
            qm = pack ? pm : quad_mask(r0.x, r0.y, co, r3.w, tx0, ty0);
            s_xy[lane] = make_float4(r0.x, r0.y, DEPTH ? r2.y : 0.f, 0.f);
            s_q[lane] = conic_q(co);
            my_co = co;
            s_col[lane] = make_float4(r1.z, r1.w, r2.x, r3.w);
            if (INTERP) s_tf[lane] = make_float2(r2.z, r2.w);
            const int x0 = __float_as_int(r3.y) & 0xffff, y0 = (int)((uint32_t)__float_as_int(r3.y) >> 16);
            const int w = __float_as_int(r3.z);
            // the Gaussian's record slots start at the exclusive scan of the rect sizes (point_offsets is inclusive)
            slot = sbase + (uint32_t)((ty - y0) * w + (tx - x0));
        }
#pragma unroll
        for (int v = 0; v < 10; v++) s_m[kMStride * v + lane] = 0.f;
        __syncthreads();
        // a batch entirely behind every pixel's last contributor leaves its records zero
        const uint32_t li_bot = li_top - (uint32_t)(n - 1);
        if (li_bot < maxlast) {
            // per quadrant, the wave-uniform set of the batch's splats to visit: footprint reaches the quadrant
            // (quad_mask) and the splat lies in front of the quadrant's furthest contributor (li < qlast[k],
            // i.e. j > li_top - qlast[k]); the loop then visits set bits only, with no LDS read to decide
            uint64_t qv[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                uint64_t m = __ballot((qm >> k) & 1u);
                if (li_top >= qlast[k]) {
                    const uint32_t d = li_top - qlast[k];  // splats 0..d are behind every pixel of quadrant k
                    m = d >= 63 ? 0ull : m & (~0ull << (d + 1));
                }
                qv[k] = m;
            }
            uint64_t todo = qv[0] | qv[1] | qv[2] | qv[3];
            // Splat loop with the least scalar bookkeeping: the visited bit is cleared (s_bitset0), the next visited
            // splat found by s_ff1 (-1 once none is left; its LDS reads use index 0 then), and every visited splat
            // is reduced (0.15% of them have no valid pair), so no per-pass wave-mask tracking.
            if (todo) {
                int j = __builtin_ctzll(todo);
                float4 xy = s_xy[j], co = s_q[j], col = s_col[j];
                float2 tf = INTERP ? s_tf[j] : make_float2(0.f, 0.f);
                // the quadrants splat jj visits, in quadrant order (uniform branches), into acc
                auto passes = [&](int jj, const float4& pxy, const float4& pco, const float4& pcol, const float2& ptf,
                                  float(&acc)[10]) {
                    const uint32_t li = li_top - (uint32_t)jj;
                    // the ten accumulators zeroed by three LDS reads of a zero block (the LDS pipe, ~29% busy here)
                    // instead of five v_mov_b64 on the VALU pipe, which this kernel saturates
                    {
                        typedef float v4f __attribute__((ext_vector_type(4)));
                        typedef __attribute__((address_space(3))) const volatile v4f lds_v4f;  // stays a ds_read
                        lds_v4f* vz = (lds_v4f*)(s_zero);
                        const v4f z0 = vz[0], z1 = vz[1], z2 = vz[2];
                        acc[0] = z0.x; acc[1] = z0.y; acc[2] = z0.z; acc[3] = z0.w;
                        acc[4] = z1.x; acc[5] = z1.y; acc[6] = z1.z; acc[7] = z1.w;
                        acc[8] = z2.x; acc[9] = z2.y;
                    }
                    if ((qv[0] >> jj) & 1u) bwd_pass<INTERP, DEPTH, ALT, 0>(ps, li, lx, ly, pxy, pco, pcol, ptf, acc);
                    if ((qv[1] >> jj) & 1u) bwd_pass<INTERP, DEPTH, ALT, 1>(ps, li, lx, ly, pxy, pco, pcol, ptf, acc);
                    if ((qv[2] >> jj) & 1u) bwd_pass<INTERP, DEPTH, ALT, 2>(ps, li, lx, ly, pxy, pco, pcol, ptf, acc);
                    if ((qv[3] >> jj) & 1u) bwd_pass<INTERP, DEPTH, ALT, 3>(ps, li, lx, ly, pxy, pco, pcol, ptf, acc);
                };
                float acc[10];  // (reset by passes() for every splat)
                while (true) {
                    int jn;  // s_ff1: -1 once todo is empty
                    asm("s_bitset0_b64 %0, %2\n\ts_ff1_i32_b64 %1, %0" : "+s"(todo), "=s"(jn) : "s"(j));
                    passes(j, xy, co, col, tf, acc);
                    const int jl = jn < 0 ? 0 : jn;  // the next visited splat's LDS reads ahead of the reduction
                    xy = s_xy[jl];
                    co = s_q[jl];
                    col = s_col[jl];
                    if (INTERP) tf = s_tf[jl];
                    // every lane stores (the spare row takes the non-totals), so no exec-mask change
                    s_m[wmd + j] = wave_reduce10_rs(acc);
                    if (jn < 0) break;
                    j = jn;
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
