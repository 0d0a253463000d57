// gauss_bwd.hip -- per-Gaussian backward kernels for gfx950, compiled without FMA contraction.
//
// Reference semantics (submodules/hierarchy-rasterizer/cuda_rasterizer):
//   k_gauss_bwd  <- computeCov2DCUDA            backward.cu:147-326
//                 + preprocessCUDA<3> backward  backward.cu:398-495 (cov3D :330-393)
//   k_sh_bwd     <- computeColorFromSH backward backward.cu:23-142
//
// These kernels are HBM bound (one thread per Gaussian), so they are built with -ffp-contract=off like the
// preprocess and the oracle: every product and sum is rounded on its own, in the oracle's order.  The conic ->
// cov2D -> cov3D chain is ill-conditioned for wide, nearly axis-aligned splats ((denom - c_xx c_yy) cancels to
// -c_xy^2), and contracting it moved scale / rotation gradients by up to 0.4% against the oracle.
// k_gauss_bwd sums each Gaussian's contiguous per-(tile, Gaussian) records written by k_blend_bwd
// (raster_bwd.hip) in a fixed order, so the backward has no float atomics and is bitwise reproducible.
#include "hlgs_internal.h"
#include "hlgs_math.h"

namespace hlgs {
// cov3d_fwd (forward.cu:181-215) with every product and sum rounded on its own, in the preprocess's order (both
// files are compiled without FMA contraction; the explicit roundings keep it so under any flags): the recomputed
// covariance is bit-identical to the one the forward used, so the forward need not store it (24 bytes per Gaussian written there and read here).
__device__ __forceinline__ void cov3d_exact(f3 scale, float mod, float4 q, float out[6])
{
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    auto M_ = [](float u, float v) { return __fmul_rn(u, v); };
    auto A_ = [](float u, float v) { return __fadd_rn(u, v); };
    auto S_ = [](float u, float v) { return __fsub_rn(u, v); };
    const m3 R = mcols(S_(1.f, M_(2.f, A_(M_(y, y), M_(z, z)))), M_(2.f, S_(M_(x, y), M_(r, z))),
                       M_(2.f, A_(M_(x, z), M_(r, y))), M_(2.f, A_(M_(x, y), M_(r, z))),
                       S_(1.f, M_(2.f, A_(M_(x, x), M_(z, z)))), M_(2.f, S_(M_(y, z), M_(r, x))),
                       M_(2.f, S_(M_(x, z), M_(r, y))), M_(2.f, A_(M_(y, z), M_(r, x))),
                       S_(1.f, M_(2.f, A_(M_(x, x), M_(y, y)))));
    m3 Sm = mcols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    Sm.m[0][0] = M_(mod, scale.x);
    Sm.m[1][1] = M_(mod, scale.y);
    Sm.m[2][2] = M_(mod, scale.z);
    m3 Mm, Sig;
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int row = 0; row < 3; row++)  // mmul(S, R)
            Mm.m[c][row] = A_(A_(M_(Sm.m[0][row], R.m[c][0]), M_(Sm.m[1][row], R.m[c][1])), M_(Sm.m[2][row], R.m[c][2]));
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int row = 0; row < 3; row++)  // mmul(mtrans(M), M)
            Sig.m[c][row] = A_(A_(M_(Mm.m[row][0], Mm.m[c][0]), M_(Mm.m[row][1], Mm.m[c][1])), M_(Mm.m[row][2], Mm.m[c][2]));
    out[0] = Sig.m[0][0]; out[1] = Sig.m[0][1]; out[2] = Sig.m[0][2];
    out[3] = Sig.m[1][1]; out[4] = Sig.m[1][2]; out[5] = Sig.m[2][2];
}

// Store a wave's rows of NF floats (row r = lane r; rows [0, nrows) of a contiguous row-major array starting at the
// wave's first row) through an LDS stage of 64 * NF floats, as whole float4s where the destination is 16-byte aligned.
template <int NF>
__device__ __forceinline__ void wave_rows_store(float* gdst, const float (&v)[NF], float* lds, int lane, int nrows)
{
    if (reinterpret_cast<uintptr_t>(gdst) & 15) {  // (uniform) unaligned destination: per-lane stores
        if (lane < nrows)
            for (int k = 0; k < NF; k++) gdst[NF * lane + k] = v[k];
        return;
    }
#pragma unroll
    for (int k = 0; k < NF; k++) lds[NF * lane + k] = v[k];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's stage writes before its reads
    const int nf = NF * nrows;
    for (int f4 = lane; 4 * f4 < nf; f4 += 64) {
        if (4 * f4 + 3 < nf) {
            reinterpret_cast<float4*>(gdst)[f4] = reinterpret_cast<const float4*>(lds)[f4];
        } else {
            for (int e = 4 * f4; e < nf; e++) gdst[e] = lds[e];
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the reads done before the stage is written again
}

constexpr int kGbwdChunk = 128;  // records per LDS chunk of k_gauss_bwd: 6 KiB per wave

// One thread per rasterised Gaussian: sum its per-tile records, then covariance / SH / scale-rotation
// backward.  Writes every output row it owns (zeros for invisible Gaussians), so no memset is needed.
template <bool HIER, bool ALT>
__global__ void __launch_bounds__(256) k_gauss_bwd(hlgs_raster_args a, const int* __restrict__ radii, Geom g,
                                                   BwdScratch rec, hlgs_grads o, float fx, float fy, int has_depth,
                                                   const uint32_t* __restrict__ misc)
{
    // the forward packed its entries (misc[kMiscPack]), so Geom::qmask holds this frame's quadrant masks: a slot whose
    // mask is 0 holds no record (drop_empty: never binned) or a zero one, and is skipped (rect_tile_mask)
    const bool masked = misc && misc[kMiscPack];
    // per wave: the chunk of records being summed (LDS-DMA), then the stage of the output rows
    __shared__ float4 s_rec[4][3 * kGbwdChunk];
    const int t_idx = blockIdx.x * 256 + threadIdx.x;
    // the slot range and the masks are loaded with the radius, not behind it (an invisible Gaussian's tiles_touched
    // is 0, so its range is empty; its qmask word is stale and never used)
    uint32_t r_end = 0, r_start = 0, qraw = 0xFFFFFFFFu;
    bool vis = false;
    if (t_idx < a.P) {
        vis = radii[t_idx] > 0;
        r_end = g.point_offsets[t_idx];
        r_start = r_end - g.tiles_touched[t_idx];
        qraw = g.qmask[t_idx];
    }
    if (!vis) r_start = r_end;
    // Gaussians with more than kWide record slots (rects over many tiles) are summed by their whole wave, lane-
    // strided, with a fixed butterfly at the end -- deterministic, and one wide splat no longer serialises a lane
    // over thousands of slots.  Done before any lane leaves, so every lane of the wave takes part.
    constexpr bool alt = ALT;
    // (loaded ahead of the wide sums: a wide Gaussian's constants come from its own lane, not from a second load)
    float4 kco = make_float4(0.f, 0.f, 0.f, 0.f);
    float kx = 0.f, ky = 0.f;
    AltKeep kthr{0.f, 0.f, 0.f};
    int kx0 = 0, ky0 = 0, kw = 1;
    if (alt && vis) {  // slots of tiles the binning culled (alt_tile_keep) hold no record: skip them
        const float4 r0 = g.splat[4 * (size_t)t_idx], r1 = g.splat[4 * (size_t)t_idx + 1];
        const float4 r3 = g.splat[4 * (size_t)t_idx + 3];
        kx = r0.x; ky = r0.y;
        kco = make_float4(r0.z, r0.w, r1.x, r1.y);
        kthr = alt_keep_prep(kco);
        kx0 = __float_as_int(r3.y) & 0xffff;
        ky0 = (int)((uint32_t)__float_as_int(r3.y) >> 16);
        kw = __float_as_int(r3.z);
    }
    constexpr uint32_t kWide = 32;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f, s5 = 0.f, s6 = 0.f, s7 = 0.f, s8 = 0.f, s9 = 0.f;
    const uint32_t qmasks = (vis && masked) ? qraw : 0xFFFFFFFFu;
    {
        uint64_t wide = __ballot(vis && r_end - r_start > kWide);
        const int lane = threadIdx.x & 63;
        while (wide) {
            const int src = __ffsll((long long)wide) - 1;
            wide &= wide - 1;
            const uint32_t ws = (uint32_t)__shfl((int)r_start, src, 64), we = (uint32_t)__shfl((int)r_end, src, 64);
            auto rl = [&](float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src)); };
            float4 wco = make_float4(0.f, 0.f, 0.f, 0.f);
            float wx = 0.f, wy = 0.f;
            AltKeep wthr{0.f, 0.f, 0.f};
            int wx0 = 0, wy0 = 0, ww = 1;
            if (ALT) {  // the wide Gaussian's constants, from its lane
                wx = rl(kx); wy = rl(ky);
                wco = make_float4(rl(kco.x), rl(kco.y), rl(kco.z), rl(kco.w));
                wthr = AltKeep{rl(kthr.thr), rl(kthr.rcx), rl(kthr.rcz)};
                wx0 = __builtin_amdgcn_readlane(kx0, src);
                wy0 = __builtin_amdgcn_readlane(ky0, src);
                ww = __builtin_amdgcn_readlane(kw, src);
            }
            const uint32_t wq = (uint32_t)__shfl((int)qmasks, src, 64);
            float p[10] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            // the lane's tile, stepped by 64 slots at a time (divisions once per wide Gaussian, not per slot)
            const int sy = ALT ? 64 / ww : 0, sx = ALT ? 64 - sy * ww : 0;
            int ty = ALT ? lane / ww : 0, tx = ALT ? lane - ty * ww : 0;
            for (uint32_t r = ws + lane; r < we; r += 64) {
                const int cx = tx, cy = ty;
                if (ALT) {
                    tx += sx;
                    ty += sy;
                    if (tx >= ww) { tx -= ww; ty++; }
                }
                if (!rect_tile_mask(wq, r - ws)) continue;
                if (ALT && !alt_tile_keep(wx, wy, wco, wthr, wx0 + cx, wy0 + cy)) continue;
                const float4 A = rec.rec[3 * (size_t)r];
                const float4 B = rec.rec[3 * (size_t)r + 1];
                const float4 Cc = rec.rec[3 * (size_t)r + 2];
                p[0] += A.x; p[1] += A.y; p[2] += A.z; p[3] += A.w;
                p[4] += B.x; p[5] += B.y; p[6] += B.z; p[7] += B.w;
                p[8] += Cc.x; p[9] += Cc.y;
            }
#pragma unroll
            for (int v = 0; v < 10; v++)
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) p[v] += __shfl_xor(p[v], off, 64);
            if (lane == src) {
                s0 = p[0]; s1 = p[1]; s2 = p[2]; s3 = p[3]; s4 = p[4];
                s5 = p[5]; s6 = p[6]; s7 = p[7]; s8 = p[8]; s9 = p[9];
            }
        }
    }
    // ---- per-Gaussian sum of the blend records in slot order (fixed => deterministic); wide ones were summed above.
    // The wave's records are contiguous (consecutive Gaussians own consecutive slot ranges), so they are copied to
    // LDS in chunks of kChunk records by LDS-DMA -- coalesced 1 KiB wave instructions instead of every lane reading
    // its own 48-byte records at its own address -- and each lane then sums its records from LDS, in slot order as
    // before (bitwise the same sums).  Done before any lane leaves: the copy is a wave instruction.
    const uint32_t start = r_start, end = vis && r_end - r_start > kWide ? r_start : r_end;  // narrow range
    // per-Gaussian inputs of the covariance / projection backward, issued ahead of the record sums so their latency
    // overlaps them
    // (The camera matrices too, before the kernel's first global store: a load that follows a store waits for it
    // (vmcnt counts both), and uniform loads only take the scalar path when no store can precede them.)
    float view[16], proj[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
        view[i] = a.viewmatrix[i];
        proj[i] = a.projmatrix[i];
    }
    const int idx = t_idx < a.P ? (HIER ? a.indices[t_idx] : t_idx) : 0;
    f3 mean = mk(0.f, 0.f, 0.f), scl3 = mk(0.f, 0.f, 0.f);
    float4 rq = make_float4(0.f, 0.f, 0.f, 0.f);
    float c3[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float opac = 0.f;
    if (vis) {
        mean = mk(a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]);
        opac = a.opacities[idx];
        if (a.cov3D_precomp || HIER) {
            const float* cov3D = a.cov3D_precomp ? a.cov3D_precomp + 6 * t_idx : g.cov3D + 6 * (size_t)t_idx;
            for (int i = 0; i < 6; i++) c3[i] = cov3D[i];
        }
        if (a.scales) {  // the cov3D recomputation and the scale / rotation backward
            scl3 = mk(a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]);
            rq = reinterpret_cast<const float4*>(a.rotations)[idx];
        }
    }
    {
        constexpr int kChunk = kGbwdChunk;
        float4* buf = s_rec[threadIdx.x >> 6];
        const int lane = threadIdx.x & 63;
        const bool any = start < end;
        uint32_t lo = any ? start : 0xFFFFFFFFu, hi = any ? end : 0u;
        for (int off = 32; off > 0; off >>= 1) {
            lo = min(lo, (uint32_t)__shfl_xor((int)lo, off, 64));
            hi = max(hi, (uint32_t)__shfl_xor((int)hi, off, 64));
        }
        lo = __builtin_amdgcn_readfirstlane(lo);
        hi = __builtin_amdgcn_readfirstlane(hi);
        typedef __attribute__((address_space(3))) void lds_t;
        for (uint32_t c0 = lo; c0 < hi; c0 += kChunk) {
            const uint32_t c1 = min(hi, c0 + kChunk);
            if (__ballot(start < c1 && end > c0) == 0) continue;  // inside a wide Gaussian's range: nobody needs it
            const uint32_t nf = 3 * (c1 - c0);
            const float4* src = rec.rec + 3 * (size_t)c0;
#pragma unroll
            for (int k = 0; k < 3 * kChunk / 64; k++) {
                if ((uint32_t)(64 * k) >= nf) break;  // wave-uniform
                const uint32_t f = min((uint32_t)(64 * k + lane), nf - 1);
                __builtin_amdgcn_global_load_lds((const void*)(src + f), (lds_t*)(buf + 64 * k), 16, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMA has landed (this wave's own LDS region)
            const uint32_t r0 = max(start, c0), r1 = min(end, c1);
            // the slot's tile, stepped along the rect's rows (one division per chunk, not two per slot)
            int ty = 0, tx = 0;
            if (alt && r0 < r1) {
                ty = (int)(r0 - start) / kw;
                tx = (int)(r0 - start) - ty * kw;
            }
            for (uint32_t r = r0; r < r1; r++) {
                bool use = rect_tile_mask(qmasks, r - start);
                if (alt) {
                    if (use) use = alt_tile_keep(kx, ky, kco, kthr, kx0 + tx, ky0 + ty);
                    if (++tx == kw) { tx = 0; ty++; }
                }
                if (!use) continue;
                const float4 A = buf[3 * (r - c0)], B = buf[3 * (r - c0) + 1], Cc = buf[3 * (r - c0) + 2];
                s0 += A.x; s1 += A.y; s2 += A.z; s3 += A.w;
                s4 += B.x; s5 += B.y; s6 += B.z; s7 += B.w;
                s8 += Cc.x; s9 += Cc.y;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every read of the chunk done before the next DMA
        }
    }
    const int M3 = a.M * 3;
    const bool live = t_idx < a.P;
    // the outputs, zeros for an invisible Gaussian
    float dc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, dscale[3] = {0.f, 0.f, 0.f}, dq[4] = {0.f, 0.f, 0.f, 0.f};
    f3 dmean = mk(0.f, 0.f, 0.f);
    float dop_out = 0.f;
    if (live && !vis && !HIER) {
        if (o.dsh && !a.shs)
            for (int i = 0; i < M3; i++) o.dsh[(size_t)idx * M3 + i] = 0.f;
        if (o.ddc && !a.shs) { o.ddc[3 * idx] = 0.f; o.ddc[3 * idx + 1] = 0.f; o.ddc[3 * idx + 2] = 0.f; }
    }
    if (vis) {
        // cov3D is not stored by the forward: recomputed from the scale and rotation the forward used
        if (!(a.cov3D_precomp || HIER)) cov3d_exact(scl3, a.scale_modifier, rq, c3);

        // ---- computeCov2DCUDA (backward.cu:147-326)
        Cov2D k;
        cov2d_eval(mean, fx, fy, a.tanfovx, a.tanfovy, c3, view, k);
        const float xg = k.txtz < -k.limx || k.txtz > k.limx ? 0.f : 1.f;
        const float yg = k.tytz < -k.limy || k.tytz > k.limy ? 0.f : 1.f;
        float c_xx = k.cov.m[0][0], c_xy = k.cov.m[0][1], c_yy = k.cov.m[1][1];
        const float h_var = 0.3f;
        const float det_cov = c_xx * c_yy - c_xy * c_xy;
        c_xx += h_var;
        c_yy += h_var;
        const float det_h = c_xx * c_yy - c_xy * c_xy;
        float dop = s5;
        float dxx = 0.f, dxy = 0.f, dyy = 0.f;
        if (!alt || a.antialiasing) {  // the alt rasterizer applies the AA term only with antialiasing (backward.cu:212-245)
            const float hs = sqrtf(fmaxf(0.000025f, det_cov / det_h));
            const float d_hs = s5 * opac;
            dop = s5 * hs;
            const float d_inside = (det_cov / det_h) <= 0.000025f ? 0.f : d_hs / (2 * hs);
            const float x = c_xx, y = c_yy, z = c_xy, w = h_var;
            const float sqv = w * w + w * (x + y) + x * y - z * z;
            const float denom_f = d_inside / (sqv * sqv);
            dxx = w * (w * y + y * y + z * z) * denom_f;
            dyy = w * (w * x + x * x + z * z) * denom_f;
            dxy = -2.f * w * z * (w + x + y) * denom_f;
        }
        const float dcx = s2, dcy = s3, dcz = s4;
        const float denom = c_xx * c_yy - c_xy * c_xy;
        const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
        const m3& Tm = k.T;
        const m3& V = k.Vrk;
    #define TT(c, r) Tm.m[c][r]
    #define VK(c, r) V.m[c][r]
        if (denom2inv != 0) {
            dxx += denom2inv * (-c_yy * c_yy * dcx + 2 * c_xy * c_yy * dcy + (denom - c_xx * c_yy) * dcz);
            dyy += denom2inv * (-c_xx * c_xx * dcz + 2 * c_xx * c_xy * dcy + (denom - c_xx * c_yy) * dcx);
            dxy += denom2inv * 2 * (c_xy * c_yy * dcx - (denom + 2 * c_xy * c_xy) * dcy + c_xx * c_xy * dcz);
            dc[0] = (TT(0, 0) * TT(0, 0) * dxx + TT(0, 0) * TT(1, 0) * dxy + TT(1, 0) * TT(1, 0) * dyy);
            dc[3] = (TT(0, 1) * TT(0, 1) * dxx + TT(0, 1) * TT(1, 1) * dxy + TT(1, 1) * TT(1, 1) * dyy);
            dc[5] = (TT(0, 2) * TT(0, 2) * dxx + TT(0, 2) * TT(1, 2) * dxy + TT(1, 2) * TT(1, 2) * dyy);
            dc[1] = 2 * TT(0, 0) * TT(0, 1) * dxx + (TT(0, 0) * TT(1, 1) + TT(0, 1) * TT(1, 0)) * dxy + 2 * TT(1, 0) * TT(1, 1) * dyy;
            dc[2] = 2 * TT(0, 0) * TT(0, 2) * dxx + (TT(0, 0) * TT(1, 2) + TT(0, 2) * TT(1, 0)) * dxy + 2 * TT(1, 0) * TT(1, 2) * dyy;
            dc[4] = 2 * TT(0, 2) * TT(0, 1) * dxx + (TT(0, 1) * TT(1, 2) + TT(0, 2) * TT(1, 1)) * dxy + 2 * TT(1, 1) * TT(1, 2) * dyy;
        }
        const float dT00 = 2 * (TT(0, 0) * VK(0, 0) + TT(0, 1) * VK(0, 1) + TT(0, 2) * VK(0, 2)) * dxx + (TT(1, 0) * VK(0, 0) + TT(1, 1) * VK(0, 1) + TT(1, 2) * VK(0, 2)) * dxy;
        const float dT01 = 2 * (TT(0, 0) * VK(1, 0) + TT(0, 1) * VK(1, 1) + TT(0, 2) * VK(1, 2)) * dxx + (TT(1, 0) * VK(1, 0) + TT(1, 1) * VK(1, 1) + TT(1, 2) * VK(1, 2)) * dxy;
        const float dT02 = 2 * (TT(0, 0) * VK(2, 0) + TT(0, 1) * VK(2, 1) + TT(0, 2) * VK(2, 2)) * dxx + (TT(1, 0) * VK(2, 0) + TT(1, 1) * VK(2, 1) + TT(1, 2) * VK(2, 2)) * dxy;
        const float dT10 = 2 * (TT(1, 0) * VK(0, 0) + TT(1, 1) * VK(0, 1) + TT(1, 2) * VK(0, 2)) * dyy + (TT(0, 0) * VK(0, 0) + TT(0, 1) * VK(0, 1) + TT(0, 2) * VK(0, 2)) * dxy;
        const float dT11 = 2 * (TT(1, 0) * VK(1, 0) + TT(1, 1) * VK(1, 1) + TT(1, 2) * VK(1, 2)) * dyy + (TT(0, 0) * VK(1, 0) + TT(0, 1) * VK(1, 1) + TT(0, 2) * VK(1, 2)) * dxy;
        const float dT12 = 2 * (TT(1, 0) * VK(2, 0) + TT(1, 1) * VK(2, 1) + TT(1, 2) * VK(2, 2)) * dyy + (TT(0, 0) * VK(2, 0) + TT(0, 1) * VK(2, 1) + TT(0, 2) * VK(2, 2)) * dxy;
    #undef VK
    #undef TT
        const m3& Wm = k.W;
        const float dJ00 = Wm.m[0][0] * dT00 + Wm.m[0][1] * dT01 + Wm.m[0][2] * dT02;
        const float dJ02 = Wm.m[2][0] * dT00 + Wm.m[2][1] * dT01 + Wm.m[2][2] * dT02;
        const float dJ11 = Wm.m[1][0] * dT10 + Wm.m[1][1] * dT11 + Wm.m[1][2] * dT12;
        const float dJ12 = Wm.m[2][0] * dT10 + Wm.m[2][1] * dT11 + Wm.m[2][2] * dT12;
        const f3 t = k.t;
        const float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
        const float dtx = xg * -fx * tz2 * dJ02;
        const float dty = yg * -fy * tz2 * dJ12;
        float dtz = -fx * tz2 * dJ00 - fy * tz2 * dJ11 + (2 * fx * t.x) * tz3 * dJ02 + (2 * fy * t.y) * tz3 * dJ12;
        if (has_depth) dtz -= alt ? s9 * tz2 : s9 / (t.z * t.z);  // alt-rasterizer backward.cu:312
        const float* vm = view;
        dmean = mk(vm[0] * dtx + vm[1] * dty + vm[2] * dtz, vm[4] * dtx + vm[5] * dty + vm[6] * dtz,
                      vm[8] * dtx + vm[9] * dty + vm[10] * dtz);

        // ---- preprocessCUDA backward (backward.cu:398-495): screen-space mean -> world mean
        const f3 m = mean;
        const float m_w = 1.0f / (xform44w(m, proj) + 0.0000001f);
        const float mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
        const float mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
        f3 d2;
        d2.x = (proj[0] * m_w - proj[3] * mul1) * s0 + (proj[1] * m_w - proj[3] * mul2) * s1;
        d2.y = (proj[4] * m_w - proj[7] * mul1) * s0 + (proj[5] * m_w - proj[7] * mul2) * s1;
        d2.z = (proj[8] * m_w - proj[11] * mul1) * s0 + (proj[9] * m_w - proj[11] * mul2) * s1;
        dmean = add(dmean, d2);

        // ---- SH backward (backward.cu:23-142) runs in k_sh_bwd, which adds its view-direction term to
        //      dmean3D (or to the parent-deferred share) after this kernel.
        if (!a.shs && o.dsh)
            for (int i = 0; i < M3; i++) o.dsh[(size_t)idx * M3 + i] = 0.f;
        // alt without higher-order coefficients: the reference skips the whole SH backward (backward.cu:443),
        // so even dc gets no gradient
        if (!a.shs && o.ddc) { o.ddc[3 * idx] = 0.f; o.ddc[3 * idx + 1] = 0.f; o.ddc[3 * idx + 2] = 0.f; }

        // ---- cov3D backward (backward.cu:330-393)
        if (a.scales) {
            const float qq[4] = {rq.x, rq.y, rq.z, rq.w};
            const float r = qq[0], x = qq[1], y = qq[2], z = qq[3];
            const m3 R = quat_rot(qq);
            m3 S = mcols(1, 0, 0, 0, 1, 0, 0, 0, 1);
            const f3 s = scl(a.scale_modifier, scl3);
            S.m[0][0] = s.x; S.m[1][1] = s.y; S.m[2][2] = s.z;
            const m3 Mm = mmul(S, R);
            const m3 dS = mcols(dc[0], 0.5f * dc[1], 0.5f * dc[2], 0.5f * dc[1], dc[3], 0.5f * dc[4], 0.5f * dc[2],
                                0.5f * dc[4], dc[5]);
            m3 M2 = Mm;
            for (int c = 0; c < 3; c++)
                for (int rr = 0; rr < 3; rr++) M2.m[c][rr] = 2.0f * Mm.m[c][rr];
            const m3 dM = mmul(M2, dS);
            const m3 Rt = mtrans(R);
            m3 dMt = mtrans(dM);
            for (int i = 0; i < 3; i++)
                dscale[i] = Rt.m[i][0] * dMt.m[i][0] + Rt.m[i][1] * dMt.m[i][1] + Rt.m[i][2] * dMt.m[i][2];
            for (int rr = 0; rr < 3; rr++) { dMt.m[0][rr] *= s.x; dMt.m[1][rr] *= s.y; dMt.m[2][rr] *= s.z; }
            dq[0] = 2 * z * (dMt.m[0][1] - dMt.m[1][0]) + 2 * y * (dMt.m[2][0] - dMt.m[0][2]) + 2 * x * (dMt.m[1][2] - dMt.m[2][1]);
            dq[1] = 2 * y * (dMt.m[1][0] + dMt.m[0][1]) + 2 * z * (dMt.m[2][0] + dMt.m[0][2]) + 2 * r * (dMt.m[1][2] - dMt.m[2][1]) - 4 * x * (dMt.m[2][2] + dMt.m[1][1]);
            dq[2] = 2 * x * (dMt.m[1][0] + dMt.m[0][1]) + 2 * r * (dMt.m[2][0] - dMt.m[0][2]) + 2 * z * (dMt.m[1][2] + dMt.m[2][1]) - 4 * y * (dMt.m[2][2] + dMt.m[0][0]);
            dq[3] = 2 * r * (dMt.m[0][1] - dMt.m[1][0]) + 2 * x * (dMt.m[2][0] + dMt.m[0][2]) + 2 * y * (dMt.m[1][2] + dMt.m[2][1]) - 4 * z * (dMt.m[1][1] + dMt.m[0][0]);
        }
        dop_out = dop;
        if (HIER) {
            // backward.cu:458-494: the child's opacity/scale/rotation/SH gradients are dropped and
            // (1 - t) of its mean gradient moves to the parent (added by k_parent_mean_add).
            const int parent = a.parent_indices[t_idx];
            if (parent != -1) {
                const float tt = a.ts[t_idx];
                dop_out = 0.f;
                for (int i = 0; i < 3; i++) dscale[i] = 0.f;
                for (int i = 0; i < 4; i++) dq[i] = 0.f;
                rec.parent_dmean[3 * t_idx] = (1.0f - tt) * dmean.x;
                rec.parent_dmean[3 * t_idx + 1] = (1.0f - tt) * dmean.y;
                rec.parent_dmean[3 * t_idx + 2] = (1.0f - tt) * dmean.z;
                dmean = mk(0.f, 0.f, 0.f);
            }
        }
    }
    if (HIER) {  // rows at the hierarchy's indices: per lane, visible Gaussians only
        if (!vis) return;
        o.dmean2D[3 * idx] = s0;
        o.dmean2D[3 * idx + 1] = s1;
        o.dmean2D[3 * idx + 2] = 0.f;
        o.dcolor[3 * idx] = s6;
        o.dcolor[3 * idx + 1] = s7;
        o.dcolor[3 * idx + 2] = s8;
        o.dopacity[idx] = dop_out;
        if (o.dcov3D)
            for (int i = 0; i < 6; i++) o.dcov3D[6 * idx + i] = dc[i];
        o.dmean3D[3 * idx] = dmean.x;
        o.dmean3D[3 * idx + 1] = dmean.y;
        o.dmean3D[3 * idx + 2] = dmean.z;
        o.dscale[3 * idx] = dscale[0];
        o.dscale[3 * idx + 1] = dscale[1];
        o.dscale[3 * idx + 2] = dscale[2];
        reinterpret_cast<float4*>(o.drot)[idx] = make_float4(dq[0], dq[1], dq[2], dq[3]);
        return;
    }
    // Rows at t_idx: the wave's rows of each output are contiguous, so they go out through this wave's LDS stage (the
    // record-sum buffer, free now) as whole float4s -- one or two 1 KiB wave stores per array instead of three or six
    // 4-byte stores of every lane into pieces of the same lines.
    {
        float* stage = reinterpret_cast<float*>(s_rec[threadIdx.x >> 6]);
        const int lane = threadIdx.x & 63, w0 = t_idx - lane, nrows = max(0, min(64, a.P - w0));
        if (!vis) s0 = s1 = s6 = s7 = s8 = 0.f;
        const float r_dm2[3] = {s0, s1, 0.f}, r_dcol[3] = {s6, s7, s8}, r_dop[1] = {dop_out};
        const float r_dm3[3] = {dmean.x, dmean.y, dmean.z};
        wave_rows_store<3>(o.dmean2D + 3 * (size_t)w0, r_dm2, stage, lane, nrows);
        wave_rows_store<3>(o.dcolor + 3 * (size_t)w0, r_dcol, stage, lane, nrows);
        wave_rows_store<1>(o.dopacity + (size_t)w0, r_dop, stage, lane, nrows);
        // dcov3D is an output only (the cov3D backward is fused into dscale / drot): skipped when the caller has no
        // cov3D_precomp to return it for (NULL; 24 B per Gaussian of writes)
        if (o.dcov3D) wave_rows_store<6>(o.dcov3D + 6 * (size_t)w0, dc, stage, lane, nrows);
        wave_rows_store<3>(o.dmean3D + 3 * (size_t)w0, r_dm3, stage, lane, nrows);
        wave_rows_store<3>(o.dscale + 3 * (size_t)w0, dscale, stage, lane, nrows);
        if (live) reinterpret_cast<float4*>(o.drot)[idx] = make_float4(dq[0], dq[1], dq[2], dq[3]);
    }
}

// Basis function c of the reference's SH colour (forward.cu:20-67) and its gradient with respect to the
// normalised view direction (the dRGBdx/dy/dz terms of backward.cu:55-139, per coefficient).
__device__ __forceinline__ float sh_basis(int c, float x, float y, float z, float& gx, float& gy, float& gz)
{
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    gx = gy = gz = 0.f;
    switch (c) {
    case 0: return kSH_C0;
    case 1: gy = -kSH_C1; return -kSH_C1 * y;
    case 2: gz = kSH_C1; return kSH_C1 * z;
    case 3: gx = -kSH_C1; return -kSH_C1 * x;
    case 4: gx = kSH_C2[0] * y; gy = kSH_C2[0] * x; return kSH_C2[0] * xy;
    case 5: gy = kSH_C2[1] * z; gz = kSH_C2[1] * y; return kSH_C2[1] * yz;
    case 6: gx = kSH_C2[2] * 2.f * -x; gy = kSH_C2[2] * 2.f * -y; gz = kSH_C2[2] * 2.f * 2.f * z;
            return kSH_C2[2] * (2.f * zz - xx - yy);
    case 7: gx = kSH_C2[3] * z; gz = kSH_C2[3] * x; return kSH_C2[3] * xz;
    case 8: gx = kSH_C2[4] * 2.f * x; gy = kSH_C2[4] * 2.f * -y; return kSH_C2[4] * (xx - yy);
    case 9: gx = kSH_C3[0] * 3.f * 2.f * xy; gy = kSH_C3[0] * 3.f * (xx - yy); return kSH_C3[0] * y * (3.f * xx - yy);
    case 10: gx = kSH_C3[1] * yz; gy = kSH_C3[1] * xz; gz = kSH_C3[1] * xy; return kSH_C3[1] * xy * z;
    case 11: gx = kSH_C3[2] * -2.f * xy; gy = kSH_C3[2] * (-3.f * yy + 4.f * zz - xx); gz = kSH_C3[2] * 4.f * 2.f * yz;
             return kSH_C3[2] * y * (4.f * zz - xx - yy);
    case 12: gx = kSH_C3[3] * -3.f * 2.f * xz; gy = kSH_C3[3] * -3.f * 2.f * yz;
             gz = kSH_C3[3] * 3.f * (2.f * zz - xx - yy); return kSH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy);
    case 13: gx = kSH_C3[4] * (-3.f * xx + 4.f * zz - yy); gy = kSH_C3[4] * -2.f * xy; gz = kSH_C3[4] * 4.f * 2.f * xz;
             return kSH_C3[4] * x * (4.f * zz - xx - yy);
    case 14: gx = kSH_C3[5] * 2.f * xz; gy = kSH_C3[5] * -2.f * yz; gz = kSH_C3[5] * (xx - yy);
             return kSH_C3[5] * z * (xx - yy);
    default: gx = kSH_C3[6] * 3.f * (xx - yy); gy = kSH_C3[6] * -3.f * 2.f * xy; return kSH_C3[6] * x * (xx - 3.f * yy);
    }
}

// SH backward (backward.cu:23-142), one thread per Gaussian.  The wave's 64 coefficient rows are staged
// through LDS so global reads of shs and writes of dsh are contiguous float4 runs; each thread then
// walks its own LDS row (coefficient loop unrolled at compile time), writes its dsh row in place and
// the wave stores the rows back.  Runs after k_gauss_bwd, whose dcolor output is dL/dRGB, and adds
// dnormvdv(dir, dL/ddir) to dmean3D -- or, for a hierarchy child with a parent, (1 - t) of it to the
// parent-deferred share (backward.cu:458-494).
// ALT (alt-rasterizer backward.cu:23-146): coefficient 0 is the separate dc row (gradient to ddc), and the
// staged rows hold the M higher-order coefficients 1..M.
// When the forward left d colour / d view direction in Geom::sh_jac (sh_jac_written), k_sh_bwd_jac2 below runs instead
// and reads no SH row.
template <bool HIER, int MT, bool ALT>  // MT = 0: staged row count a.M known only at run time (up to 16)
__global__ void __launch_bounds__(64) k_sh_bwd(hlgs_raster_args a, const int* __restrict__ radii, Geom g,
                                               BwdScratch rec, hlgs_grads o)
{
    constexpr int OFF = ALT ? 1 : 0;  // full coefficient index of staged row 0
    constexpr int MC = MT ? MT : (16 - OFF);
    const int M = MT ? MT : a.M;
    const int M3 = 3 * M;
    __shared__ float s_rows[64 * kShStride];
    __shared__ int s_idx[64];
    __shared__ int s_vis[64];
    const int lane = threadIdx.x;
    const int t0 = blockIdx.x * 64;
    const int n = min(64, a.P - t0);
    const int t_idx = t0 + lane;
    const bool active = lane < n;
    const int idx = active ? (HIER ? a.indices[t_idx] : t_idx) : 0;
    const bool vis = active && radii[t_idx] > 0;
    s_idx[lane] = idx;
    s_vis[lane] = vis;
    // the visible Gaussian's own inputs, issued before the row copy so both latencies overlap
    f3 m = mk(0.f, 0.f, 0.f), dcol = mk(0.f, 0.f, 0.f);
    uint32_t cl = 0;
    if (vis) {
        m = mk(a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]);
        dcol = mk(o.dcolor[3 * idx], o.dcolor[3 * idx + 1], o.dcolor[3 * idx + 2]);
        cl = g.clamped[t_idx];
    }
    __syncthreads();
    // rows of invisible Gaussians are not read: they arrive as zeros, which is their dsh row
    sh_rows_load<3 * MT>(a.shs, s_rows, s_idx, n, lane, M3, s_vis);
    // colour-factored mode (o.drgb, view-data-parallel exchange): the masked dL/dRGB row replaces dsh / ddc
    const bool factored = o.drgb != nullptr;  // uniform
    __syncthreads();
    float* row = s_rows + lane * kShStride;
    if (active) {
        const bool dropped = HIER && a.parent_indices && a.parent_indices[t_idx] != -1;
        if (!vis) {
            if (factored) {
                o.drgb[3 * idx] = 0.f; o.drgb[3 * idx + 1] = 0.f; o.drgb[3 * idx + 2] = 0.f;
            } else if (ALT) {
                o.ddc[3 * idx] = 0.f; o.ddc[3 * idx + 1] = 0.f; o.ddc[3 * idx + 2] = 0.f;
            }
        } else {
            const f3 campos = mk(a.campos[0], a.campos[1], a.campos[2]);
            const f3 dir_orig = sub(m, campos);
            const float len = sqrtf(dot(dir_orig, dir_orig));
            const float x = dir_orig.x / len, y = dir_orig.y / len, z = dir_orig.z / len;
            const float dR = (cl & 1u) ? 0.f : dcol.x;
            const float dG = (cl & 2u) ? 0.f : dcol.y;
            const float dB = (cl & 4u) ? 0.f : dcol.z;
            const int ncoef = (a.D + 1) * (a.D + 1);
            float vx = 0.f, vy = 0.f, vz = 0.f;
            float basis[MC + OFF];
#pragma unroll
            for (int c = 0; c < MC + OFF; c++) {
                float gx, gy, gz;
                basis[c] = c < ncoef ? sh_basis(c, x, y, z, gx, gy, gz) : 0.f;
                if (c > 0 && c < ncoef) {
                    const float* sc = row + 3 * (c - OFF);
                    const float proj = sc[0] * dR + sc[1] * dG + sc[2] * dB;
                    vx += proj * gx;
                    vy += proj * gy;
                    vz += proj * gz;
                }
            }
            if (factored) {
                o.drgb[3 * idx] = dropped ? 0.f : dR;
                o.drgb[3 * idx + 1] = dropped ? 0.f : dG;
                o.drgb[3 * idx + 2] = dropped ? 0.f : dB;
            } else if (ALT) {
                o.ddc[3 * idx] = basis[0] * dR;
                o.ddc[3 * idx + 1] = basis[0] * dG;
                o.ddc[3 * idx + 2] = basis[0] * dB;
            }
#pragma unroll
            for (int c = OFF; c < MC + OFF; c++) {
                if (factored) break;
                if (c - OFF >= M) break;
                const float bs = dropped ? 0.f : basis[c];
                row[3 * (c - OFF)] = bs * dR;
                row[3 * (c - OFF) + 1] = bs * dG;
                row[3 * (c - OFF) + 2] = bs * dB;
            }
            const f3 d = dnormvdv(dir_orig, mk(vx, vy, vz));
            if (dropped) {
                const float w = 1.0f - a.ts[t_idx];
                rec.parent_dmean[3 * t_idx] += w * d.x;
                rec.parent_dmean[3 * t_idx + 1] += w * d.y;
                rec.parent_dmean[3 * t_idx + 2] += w * d.z;
            } else {
                o.dmean3D[3 * idx] += d.x;
                o.dmean3D[3 * idx + 1] += d.y;
                o.dmean3D[3 * idx + 2] += d.z;
            }
        }
    }
    if (factored) return;  // wave-uniform
    __syncthreads();
    sh_rows_copy<3 * MT, false>(o.dsh, s_rows, s_idx, n, lane, M3);
}

// The Jacobian SH backward: the forward left d colour / d view direction in Geom::sh_jac (sh_jac_written), so no SH row
// is read: the view direction term is dot(dRGBd{x,y,z}, dL/dRGB) in the reference's order (backward.cu:139-141) and the
// dsh rows are basis x dL/dRGB, built in LDS and stored as contiguous float4 runs.  Two waves per 64 Gaussians: wave 0
// does the per-Gaussian work and builds the dsh rows in LDS, then both waves store the block's rows.  The 12.5 KB row stage then keeps two
// waves per block instead of one (the stores, 192 B per Gaussian, are most of the kernel's traffic).  Same arithmetic.
template <int MT, bool ALT>
__global__ void __launch_bounds__(128) k_sh_bwd_jac2(hlgs_raster_args a, const int* __restrict__ radii, Geom g,
                                                    BwdScratch rec, hlgs_grads o)
{
    constexpr int OFF = ALT ? 1 : 0;  // full coefficient index of staged row 0
    constexpr int MC = MT ? MT : (16 - OFF);
    const int M = MT ? MT : a.M;
    const int M3 = 3 * M;
    __shared__ float s_rows[64 * kShStride];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t0 = blockIdx.x * 64;
    const int n = min(64, a.P - t0);
    const bool factored = o.drgb != nullptr;  // uniform
    if (wave == 0) {
        const int t_idx = t0 + lane, idx = t_idx;
        const bool active = lane < n;
        // every input in one round trip, ahead of the first store (an invisible Gaussian's loads are unused)
        const f3 campos = mk(a.campos[0], a.campos[1], a.campos[2]);
        bool vis = false;
        f3 m = mk(0.f, 0.f, 0.f), dcol = m, jx = m, jy = m, jz = m, dm = m;
        uint32_t cl = 0;
        if (active) {
            vis = radii[t_idx] > 0;
            m = mk(a.means3D[3 * idx], a.means3D[3 * idx + 1], a.means3D[3 * idx + 2]);
            dcol = mk(o.dcolor[3 * idx], o.dcolor[3 * idx + 1], o.dcolor[3 * idx + 2]);
            cl = g.clamped[t_idx];
            const float* J = g.sh_jac + 9 * (size_t)t_idx;
            jx = mk(J[0], J[1], J[2]);
            jy = mk(J[3], J[4], J[5]);
            jz = mk(J[6], J[7], J[8]);
            dm = mk(o.dmean3D[3 * idx], o.dmean3D[3 * idx + 1], o.dmean3D[3 * idx + 2]);
        }
        float* row = s_rows + lane * kShStride;
        if (!vis) {
            for (int c = 0; c < M3; c++) row[c] = 0.f;  // invisible rows are zero
            if (active && factored) {
                o.drgb[3 * idx] = 0.f; o.drgb[3 * idx + 1] = 0.f; o.drgb[3 * idx + 2] = 0.f;
            } else if (active && ALT) {
                o.ddc[3 * idx] = 0.f; o.ddc[3 * idx + 1] = 0.f; o.ddc[3 * idx + 2] = 0.f;
            }
        } else {
            const f3 dir_orig = sub(m, campos);
            const float len = sqrtf(dot(dir_orig, dir_orig));
            const float x = dir_orig.x / len, y = dir_orig.y / len, z = dir_orig.z / len;
            const float dR = (cl & 1u) ? 0.f : dcol.x;
            const float dG = (cl & 2u) ? 0.f : dcol.y;
            const float dB = (cl & 4u) ? 0.f : dcol.z;
            const int ncoef = (a.D + 1) * (a.D + 1);
            float basis[MC + OFF];
#pragma unroll
            for (int c = 0; c < MC + OFF; c++) {
                float gx, gy, gz;
                basis[c] = c < ncoef ? sh_basis(c, x, y, z, gx, gy, gz) : 0.f;
            }
            const f3 d3 = mk(dR, dG, dB);
            const float vx = dot(jx, d3), vy = dot(jy, d3), vz = dot(jz, d3);
            if (factored) {
                o.drgb[3 * idx] = dR; o.drgb[3 * idx + 1] = dG; o.drgb[3 * idx + 2] = dB;
            } else if (ALT) {
                o.ddc[3 * idx] = basis[0] * dR;
                o.ddc[3 * idx + 1] = basis[0] * dG;
                o.ddc[3 * idx + 2] = basis[0] * dB;
            }
#pragma unroll
            for (int c = OFF; c < MC + OFF; c++) {
                if (factored) break;
                if (c - OFF >= M) break;
                row[3 * (c - OFF)] = basis[c] * dR;
                row[3 * (c - OFF) + 1] = basis[c] * dG;
                row[3 * (c - OFF) + 2] = basis[c] * dB;
            }
            const f3 d = dnormvdv(dir_orig, mk(vx, vy, vz));
            o.dmean3D[3 * idx] = dm.x + d.x;
            o.dmean3D[3 * idx + 1] = dm.y + d.y;
            o.dmean3D[3 * idx + 2] = dm.z + d.z;
        }
    }
    if (factored) return;  // block-uniform
    __syncthreads();
    // the block's rows are contiguous in dsh (non-hierarchy mode): both waves store them as float4 runs
    float* gbase = o.dsh + (size_t)t0 * M3;
    if constexpr (MT > 0 && (3 * MT) % 4 == 0) {
        constexpr int Q = 3 * MT / 4;
        for (int f = threadIdx.x; f < n * Q; f += 128) {
            const int r = f / Q, q = f - r * Q;
            const float* lp = s_rows + r * kShStride + 4 * q;
            reinterpret_cast<float4*>(gbase)[f] = make_float4(lp[0], lp[1], lp[2], lp[3]);
        }
    } else {
        for (int f = threadIdx.x; f < n * M3; f += 128) {
            const int r = f / M3, q = f - r * M3;
            gbase[f] = s_rows[r * kShStride + q];
        }
    }
}

// hlgs_sh_grad_from_colour: one thread per Gaussian rebuilds its averaged SH gradient row from the V views' colour
// gradients, with the per-view products basis_c(dir_v) * dL/dRGB_v in k_sh_bwd's operation order, summed in view
// order and scaled once; rows go out through LDS as contiguous float4 runs (as k_sh_bwd's).
template <int MT, bool ALT>  // MT = 0: row count M known only at run time (up to 16)
__global__ void __launch_bounds__(64) k_sh_from_colour(int P, int V, int D, int M_rt, const float* __restrict__ means,
                                                       const float* __restrict__ campos, const float* __restrict__ drgb,
                                                       int64_t stride, float scale, float* __restrict__ dsh,
                                                       float* __restrict__ ddc)
{
    constexpr int OFF = ALT ? 1 : 0;
    constexpr int MC = MT ? MT : (16 - OFF);
    const int M = MT ? MT : M_rt;
    __shared__ float s_rows[64 * kShStride];
    __shared__ int s_idx[64];
    const int lane = threadIdx.x;
    const int t0 = blockIdx.x * 64;
    const int n = min(64, P - t0);
    const int p = t0 + lane;
    s_idx[lane] = p;
    float acc[3 * (MC + OFF)];
#pragma unroll
    for (int i = 0; i < 3 * (MC + OFF); i++) acc[i] = 0.f;
    if (lane < n) {
        const f3 m = mk(means[3 * p], means[3 * p + 1], means[3 * p + 2]);
        const int ncoef = (D + 1) * (D + 1);
        for (int v = 0; v < V; v++) {
            const float* d = drgb + v * stride + 3 * (int64_t)p;
            const float* cp = campos + v * stride;
            const float dR = d[0], dG = d[1], dB = d[2];
            const f3 dir_orig = sub(m, mk(cp[0], cp[1], cp[2]));
            const float len = sqrtf(dot(dir_orig, dir_orig));
            const float x = dir_orig.x / len, y = dir_orig.y / len, z = dir_orig.z / len;
#pragma unroll
            for (int c = 0; c < MC + OFF; c++) {
                float gx, gy, gz;
                const float bs = c < ncoef ? sh_basis(c, x, y, z, gx, gy, gz) : 0.f;
                acc[3 * c] += bs * dR;
                acc[3 * c + 1] += bs * dG;
                acc[3 * c + 2] += bs * dB;
            }
        }
        if (ALT) {
            ddc[3 * p] = scale * acc[0];
            ddc[3 * p + 1] = scale * acc[1];
            ddc[3 * p + 2] = scale * acc[2];
        }
        float* row = s_rows + lane * kShStride;
#pragma unroll
        for (int c = OFF; c < MC + OFF; c++) {
            if (c - OFF >= M) break;
            row[3 * (c - OFF)] = scale * acc[3 * c];
            row[3 * (c - OFF) + 1] = scale * acc[3 * c + 1];
            row[3 * (c - OFF) + 2] = scale * acc[3 * c + 2];
        }
    }
    __syncthreads();
    sh_rows_copy<3 * MT, false>(dsh, s_rows, s_idx, n, lane, 3 * M);
}

void launch_sh_from_colour(int P, int V, int D, int M, bool alt, const float* means, const float* campos,
                           const float* drgb, int64_t stride, float scale, float* dsh, float* ddc, hipStream_t s)
{
    const dim3 grid((P + 63) / 64);
#define HLGS_SFC(MT, AL) hipLaunchKernelGGL((k_sh_from_colour<MT, AL>), grid, dim3(64), 0, s, P, V, D, M, means, campos, \
                                           drgb, stride, scale, dsh, ddc)
    if (alt) {
        switch (M) {
        case 3: HLGS_SFC(3, true); break;
        case 8: HLGS_SFC(8, true); break;
        case 15: HLGS_SFC(15, true); break;
        default: HLGS_SFC(0, true); break;
        }
    } else {
        switch (M) {
        case 1: HLGS_SFC(1, false); break;
        case 4: HLGS_SFC(4, false); break;
        case 9: HLGS_SFC(9, false); break;
        case 16: HLGS_SFC(16, false); break;
        default: HLGS_SFC(0, false); break;
        }
    }
#undef HLGS_SFC
}

__global__ void __launch_bounds__(256) k_parent_mean_add(int P, const int* __restrict__ radii,
                                                         const int* __restrict__ parent_indices,
                                                         const float* __restrict__ pd, float* __restrict__ dmean3D)
{
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= P || !(radii[t] > 0)) return;
    const int p = parent_indices[t];
    if (p == -1) return;
    for (int i = 0; i < 3; i++) atomicAdd(&dmean3D[3 * p + i], pd[3 * t + i]);
}

// late != nullptr: the kernels after k_gauss_bwd (SH backward, which completes dmean3D / dsh / ddc, and the
// hierarchy parent add) run on `late` behind an event on `s`, and are not joined back into `s`: the opacity, scale and
// rotation gradients are final on `s` while the SH backward still runs (hlgs_rasterize_backward_split).
void launch_gauss_bwd(const hlgs_raster_args& a, const int* radii, const Geom& g, const BwdScratch& rs,
                      const hlgs_grads& o, bool has_depth, hipStream_t s, hipStream_t late, hipEvent_t ev,
                      const uint32_t* misc)
{
    const float fy = a.H / (2.0f * a.tanfovy);
    const float fx = a.W / (2.0f * a.tanfovx);
    const dim3 grid((a.P + 255) / 256), grid_sh((a.P + 63) / 64);
    const hipStream_t sl = late ? late : s;
    auto hand_over = [&]() {
        if (late) {
            hipEventRecord(ev, s);
            hipStreamWaitEvent(late, ev, 0);
        }
    };
    const bool jac = sh_jac_written(a);  // the forward's preprocess left d colour / d direction (no SH row reads)
#define HLGS_SHK(H, MT, AL)                                                                                \
    do {                                                                                                   \
        if (!(H) && jac) hipLaunchKernelGGL((k_sh_bwd_jac2<MT, AL>), grid_sh, dim3(128), 0, sl, a, radii, g, rs, o); \
        else hipLaunchKernelGGL((k_sh_bwd<H, MT, AL>), grid_sh, dim3(64), 0, sl, a, radii, g, rs, o); \
    } while (0)
#define HLGS_SHB(H)                                                                                        \
    switch (a.M) {                                                                                         \
    case 1: HLGS_SHK(H, 1, false); break;                                                                  \
    case 4: HLGS_SHK(H, 4, false); break;                                                                  \
    case 9: HLGS_SHK(H, 9, false); break;                                                                  \
    case 16: HLGS_SHK(H, 16, false); break;                                                                \
    default: HLGS_SHK(H, 0, false); break;                                                                 \
    }
    if (a.indices) {
        hipLaunchKernelGGL((k_gauss_bwd<true, false>), grid, dim3(256), 0, s, a, radii, g, rs, o, fx, fy, (int)has_depth, misc);
        hand_over();
        if (a.shs) HLGS_SHB(true)
        if (a.parent_indices)
            hipLaunchKernelGGL(k_parent_mean_add, grid, dim3(256), 0, sl, a.P, radii, a.parent_indices,
                               rs.parent_dmean, o.dmean3D);
    } else {
        if (a.variant == HLGS_VARIANT_ALT)
            hipLaunchKernelGGL((k_gauss_bwd<false, true>), grid, dim3(256), 0, s, a, radii, g, rs, o, fx, fy,
                               (int)has_depth, misc);
        else
            hipLaunchKernelGGL((k_gauss_bwd<false, false>), grid, dim3(256), 0, s, a, radii, g, rs, o, fx, fy,
                               (int)has_depth, misc);
        hand_over();
        if (a.shs && a.variant == HLGS_VARIANT_ALT) {
            switch (a.M) {  // rest coefficients of degree 1, 2, 3
            case 3: HLGS_SHK(false, 3, true); break;
            case 8: HLGS_SHK(false, 8, true); break;
            case 15: HLGS_SHK(false, 15, true); break;
            default: HLGS_SHK(false, 0, true); break;
            }
        } else if (a.shs) {
            HLGS_SHB(false)
        }
    }
#undef HLGS_SHB
#undef HLGS_SHK
}

}  // namespace hlgs
