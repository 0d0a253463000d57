// loss.hip -- fused photometric loss kernels for gfx950: SSIM (11x11 Gaussian window, sigma 1.5) with its
// gradient, L1 and the masked inverse-depth L1 of the training step.
//
// Reference semantics: utils/loss_utils.py:17-63 (l1_loss, ssim/_ssim: F.conv2d with the window of
// create_window, zero padding window_size // 2, C1 = 0.01^2, C2 = 0.03^2, map mean), the un-vendored
// fused_ssim package train_post.py:29, 559 calls (same map; padding "same" = the zero-padded map, "valid" = its
// interior [5, H-5) x [5, W-5)), and the depth term of train_single.py:111-118
// (mean |(invdepth - mono) * mask|).
//
// Design (round 5): one plane (channel) per grid.z, a 116 x 16 output tile per 256-thread workgroup, the two
// separable passes in the order that keeps the first one in registers:
//   vertical:   thread t owns input column t & 127 of the tile (its 116 output columns plus the 5-pixel halo on
//               each side) and output rows [8 q, 8 q + 8), q = t >> 7: it loads the 18 input rows of that column
//               (zero outside the image: zero padding), forms the five moments (x, y, x^2, y^2, x y) per row and
//               writes the 11-tap column sums of its 8 rows to LDS (one row of 128 columns per (moment, row));
//   horizontal: thread t owns output row j and the 8 output columns [8 s, 8 s + 8): 18 consecutive column sums
//               per moment (four 16-byte LDS reads and one 8-byte read; row stride 132 floats puts the two rows of a
//               16-lane group on opposite halves of the 64 banks) give the 8 window sums per moment.
// Round 4 staged both images with the halo in LDS and ran the horizontal pass first over all 18 rows of an 8-row
// tile (2.25 horizontal passes per output and 11 x 5 LDS reads per output in the vertical pass): 103 us forward and
// 85 us backward at 3 x 1080 x 1920 (tools/variants/loss_r04.hip).
// The forward writes the partial derivatives of the SSIM map with respect to the window means
//   A = df/dmu1 (total), B = df/d E[x^2], C = df/d E[x y]
// so that dSSIM/dx(p) = sum_q g(q) w(q - p) (A(q) + 2 x(p) B(q) + y(p) C(q)), which the backward evaluates with
// the same two passes over the three maps.  Per-workgroup sums go to a partial array that one block reduces in
// double, in a fixed order: the losses are deterministic.
#include <algorithm>

#include "hlgs_internal.h"

namespace hlgs {

constexpr int kHalo = 5;
constexpr int kQW = 128;                // input columns per tile (one per vertical-pass thread of each half)
constexpr int kQO = 116;                // output columns per tile (a multiple of 4: 16-byte map stores)
constexpr int kQR = 8;                  // output rows per vertical-pass thread
constexpr int kQH = 2 * kQR;            // output rows per tile
constexpr int kQIn = kQR + 2 * kHalo;   // input rows per vertical-pass thread
constexpr int kQS = 132;                // LDS row stride (floats)
constexpr int kQThreads = 256;
constexpr float kC1 = 0.01f * 0.01f, kC2 = 0.03f * 0.03f;
static_assert(kQO + 2 * kHalo <= kQW && kQW * 2 == kQThreads && kQH * 16 == kQThreads, "tile shape");

struct Win11 {
    float w[11];
};

// Vertical pass: NI input planes -> NM moments per input row (mom) -> 11-tap column sums of the thread's kQR rows,
// written to vs[(m kQH + row) kQS + column].
template <int NI, int NM, class Mom>
__device__ __forceinline__ void ssim_vertical(const float* const (&pl)[NI], int H, int W, int x0, int y0,
                                              const Win11& win, float* vs, Mom mom)
{
    const int c = threadIdx.x & (kQW - 1), q = threadIdx.x / kQW;
    const int gx = x0 - kHalo + c;
    const bool colin = gx >= 0 && gx < W && c < kQO + 2 * kHalo;
    const int gxc = min(max(gx, 0), W - 1);
    const int gy0 = y0 - kHalo + kQR * q;
    float in[NI][kQIn];
#pragma unroll
    for (int r = 0; r < kQIn; r++) {  // every load issued before the first use
        const int gyc = min(max(gy0 + r, 0), H - 1);
#pragma unroll
        for (int i = 0; i < NI; i++) in[i][r] = pl[i][(size_t)gyc * W + gxc];
    }
#pragma unroll
    for (int r = 0; r < kQIn; r++) {
        const bool ok = colin && gy0 + r >= 0 && gy0 + r < H;
#pragma unroll
        for (int i = 0; i < NI; i++) in[i][r] = ok ? in[i][r] : 0.f;
    }
    float mv[NM][kQIn];
#pragma unroll
    for (int r = 0; r < kQIn; r++) mom(in, r, mv);
#pragma unroll
    for (int jj = 0; jj < kQR; jj++) {
#pragma unroll
        for (int m = 0; m < NM; m++) {
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < 11; k++) acc = fmaf(win.w[k], mv[m][jj + k], acc);
            vs[(m * kQH + kQR * q + jj) * kQS + c] = acc;
        }
    }
}

// Horizontal pass: the 8 window sums per moment of output row j, tile columns [o0, o0 + 8).  Lanes 0-7 of each
// 16-lane group take eight consecutive column groups of one row, lanes 8-15 the same groups of the next row.
__device__ __forceinline__ void ssim_lane(int& j, int& o0)
{
    const int t = threadIdx.x;
    j = 2 * (t >> 5) + ((t >> 3) & 1);
    o0 = 8 * (8 * ((t >> 4) & 1) + (t & 7));
}
template <int NM>
__device__ __forceinline__ void ssim_horizontal(const float* vs, const Win11& win, int j, int o0, float (&out)[NM][8])
{
#pragma unroll
    for (int m = 0; m < NM; m++) {
        const float* row = vs + (m * kQH + j) * kQS + o0;
        float v[kQR + 2 * kHalo];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const float4 f = *reinterpret_cast<const float4*>(row + 4 * u);
            v[4 * u] = f.x; v[4 * u + 1] = f.y; v[4 * u + 2] = f.z; v[4 * u + 3] = f.w;
        }
        const float2 f = *reinterpret_cast<const float2*>(row + 16);
        v[16] = f.x;
        v[17] = f.y;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < 11; k++) acc = fmaf(win.w[k], v[i + k], acc);
            out[m][i] = acc;
        }
    }
}

// 8 consecutive floats of one row (16-byte aligned when `vec`), zero beyond n
__device__ __forceinline__ void load8(const float* p, bool vec, int n, float (&v)[8])
{
    if (vec) {
        const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = i < n ? p[i] : 0.f;
    }
}
__device__ __forceinline__ void store8(float* p, bool vec, int n, const float (&v)[8])
{
    if (vec) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
#pragma unroll
        for (int i = 0; i < 8; i++)
            if (i < n) p[i] = v[i];
    }
}

// SSIM forward.  partial[2 * block] = (sum of the SSIM map over counted pixels, sum |x - y|).
template <bool TRAIN>
__global__ void __launch_bounds__(kQThreads) k_ssim_fwd(int H, int W, const float* __restrict__ img1,
                                                        const float* __restrict__ img2, int valid, Win11 win,
                                                        float* __restrict__ abc, float* __restrict__ partial)
{
    __shared__ __attribute__((aligned(16))) float vs[5 * kQH * kQS + 8];
    __shared__ float red[2][kQThreads / 64];
    const int ch = blockIdx.z;
    const size_t HW = (size_t)H * W;
    const float* x = img1 + ch * HW;
    const float* y = img2 + ch * HW;
    const int x0 = blockIdx.x * kQO, y0 = blockIdx.y * kQH;
    const float* const pl[2] = {x, y};
    ssim_vertical<2, 5>(pl, H, W, x0, y0, win, vs, [](const float (&in)[2][kQIn], int r, float (&mv)[5][kQIn]) {
        const float u = in[0][r], v = in[1][r];
        mv[0][r] = u;
        mv[1][r] = v;
        mv[2][r] = u * u;
        mv[3][r] = v * v;
        mv[4][r] = u * v;
    });
    __syncthreads();
    int j, o0;
    ssim_lane(j, o0);
    float mo[5][8];
    ssim_horizontal<5>(vs, win, j, o0, mo);
    const int py = y0 + j, px0 = x0 + o0;
    const int n = (py < H && o0 < kQO) ? max(0, min(min(8, kQO - o0), W - px0)) : 0;
    const bool vec = n == 8 && (W & 3) == 0;
    const size_t pid = (size_t)py * W + px0;
    float xv[8], yv[8];
    if (n > 0) {
        load8(x + pid, vec, n, xv);
        load8(y + pid, vec, n, yv);
    }
    float s_map = 0.f, s_l1 = 0.f;
    float A[8], B[8], C[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const float m1 = mo[0][i], m2 = mo[1][i], e11 = mo[2][i], e22 = mo[3][i], e12 = mo[4][i];
        const int px = px0 + i;
        const bool counted = i < n && (!valid || (px >= kHalo && px < W - kHalo && py >= kHalo && py < H - kHalo));
        const float mu1_sq = m1 * m1, mu2_sq = m2 * m2, mu12 = m1 * m2;
        const float s11 = e11 - mu1_sq, s22 = e22 - mu2_sq, s12 = e12 - mu12;
        const float a = 2.f * mu12 + kC1, b = 2.f * s12 + kC2;
        const float c = mu1_sq + mu2_sq + kC1, d = s11 + s22 + kC2;
        const float f = (a * b) / (c * d);
        if (counted) s_map += f;
        if (i < n) s_l1 += fabsf(xv[i] - yv[i]);
        A[i] = B[i] = C[i] = 0.f;
        if (TRAIN && counted) {
            const float cd = c * d;
            const float dmu1 = (2.f * m2 * b) / cd - f * (2.f * m1) / c;  // df/dmu1 at fixed sigmas
            B[i] = -f / d;                                                // df/dsigma1^2
            C[i] = (2.f * a) / cd;                                        // df/dsigma12
            A[i] = dmu1 - 2.f * m1 * B[i] - m2 * C[i];                    // through sigma = E[.] - mu mu
        }
    }
    if (TRAIN && n > 0) {
        float* o = abc + (size_t)ch * 3 * HW + pid;
        store8(o, vec, n, A);
        store8(o + HW, vec, n, B);
        store8(o + 2 * HW, vec, n, C);
    }
    // workgroup sums (fixed order: shuffles, then one lane per wave)
    for (int off = 32; off > 0; off >>= 1) {
        s_map += __shfl_xor(s_map, off, 64);
        s_l1 += __shfl_xor(s_l1, off, 64);
    }
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][wave] = s_map; red[1][wave] = s_l1; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float a = 0.f, b = 0.f;
        for (int i = 0; i < kQThreads / 64; i++) { a += red[0][i]; b += red[1][i]; }
        const size_t blk = ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        partial[2 * blk] = a;
        partial[2 * blk + 1] = b;
    }
}

// grad1 = coef[0] * dSSIM-map-sum/dx + coef[1] * sign(x - y)  (coefficients on the device: no host sync).
__global__ void __launch_bounds__(kQThreads) k_ssim_bwd(int H, int W, const float* __restrict__ img1,
                                                        const float* __restrict__ img2, const float* __restrict__ abc,
                                                        Win11 win, const float* __restrict__ coef,
                                                        float* __restrict__ grad1)
{
    __shared__ __attribute__((aligned(16))) float vs[3 * kQH * kQS + 8];
    const int ch = blockIdx.z;
    const size_t HW = (size_t)H * W;
    const int x0 = blockIdx.x * kQO, y0 = blockIdx.y * kQH;
    const float* maps = abc + (size_t)ch * 3 * HW;
    const float* const pl[3] = {maps, maps + HW, maps + 2 * HW};
    ssim_vertical<3, 3>(pl, H, W, x0, y0, win, vs, [](const float (&in)[3][kQIn], int r, float (&mv)[3][kQIn]) {
        mv[0][r] = in[0][r];
        mv[1][r] = in[1][r];
        mv[2][r] = in[2][r];
    });
    __syncthreads();
    int j, o0;
    ssim_lane(j, o0);
    float g[3][8];
    ssim_horizontal<3>(vs, win, j, o0, g);
    const int py = y0 + j, px0 = x0 + o0;
    const int n = (py < H && o0 < kQO) ? max(0, min(min(8, kQO - o0), W - px0)) : 0;
    if (n == 0) return;
    const bool vec = n == 8 && (W & 3) == 0;
    const size_t pid = (size_t)ch * HW + (size_t)py * W + px0;
    float xv[8], yv[8], out[8];
    load8(img1 + pid, vec, n, xv);
    load8(img2 + pid, vec, n, yv);
    const float c0 = coef[0], c1 = coef[1];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const float dssim = g[0][i] + 2.f * xv[i] * g[1][i] + yv[i] * g[2][i];
        const float diff = xv[i] - yv[i];
        const float sgn = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);  // torch.abs backward: sign, 0 at 0
        out[i] = c0 * dssim + c1 * sgn;
    }
    store8(grad1 + pid, vec, n, out);
}

// mean |(inv - mono) * mask| partial sums; mask may be NULL (= 1).
__global__ void __launch_bounds__(256) k_depth_l1_fwd(long n, const float* __restrict__ inv,
                                                      const float* __restrict__ mono, const float* __restrict__ mask,
                                                      float* __restrict__ partial)
{
    __shared__ float red[4];
    float s = 0.f;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const float m = mask ? mask[i] : 1.f;
        s += fabsf((inv[i] - mono[i]) * m);
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void __launch_bounds__(256) k_depth_l1_bwd(long n, const float* __restrict__ inv,
                                                      const float* __restrict__ mono, const float* __restrict__ mask,
                                                      const float* __restrict__ coef, float* __restrict__ grad)
{
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float m = mask ? mask[i] : 1.f;
    const float v = (inv[i] - mono[i]) * m;
    const float sgn = v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f);
    grad[i] = coef[0] * sgn * m;
}

// One block: out[k] = scale[k] * sum_i partial[i * stride + k] for k < stride, summed in double in index order.
__global__ void __launch_bounds__(1024) k_reduce_partials(int n, int stride, const float* __restrict__ partial,
                                                          double s0, double s1, float* __restrict__ out)
{
    __shared__ double red[2][16];
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < n; i += 1024) {
        a += (double)partial[(size_t)i * stride];
        if (stride > 1) b += (double)partial[(size_t)i * stride + 1];
    }
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_xor(a, off, 64);
        b += __shfl_xor(b, off, 64);
    }
    if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = a; red[1][threadIdx.x >> 6] = b; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double ta = 0.0, tb = 0.0;
        for (int i = 0; i < 16; i++) { ta += red[0][i]; tb += red[1][i]; }
        out[0] = (float)(ta * s0);
        if (stride > 1) out[1] = (float)(tb * s1);
    }
}

static Win11 gauss_window()
{
    // utils/loss_utils.py:23-25: exp(-(x - 5)^2 / (2 sigma^2)) in double, stored as float32, normalised in float32
    Win11 w;
    float g[11], s = 0.f;
    for (int i = 0; i < 11; i++) {
        g[i] = (float)exp(-(double)((i - 5) * (i - 5)) / (2.0 * 1.5 * 1.5));
    }
    for (int i = 0; i < 11; i++) s += g[i];
    for (int i = 0; i < 11; i++) w.w[i] = g[i] / s;
    return w;
}

static dim3 ssim_grid(int C, int H, int W) { return dim3((W + kQO - 1) / kQO, (H + kQH - 1) / kQH, C); }

size_t ssim_partials(int C, int H, int W)
{
    const dim3 g = ssim_grid(C, H, W);
    return (size_t)g.x * g.y * g.z;
}

void launch_ssim_forward(int C, int H, int W, const float* img1, const float* img2, int valid, float* abc,
                         float* partial, float* out, hipStream_t s)
{
    const dim3 g = ssim_grid(C, H, W);
    const Win11 w = gauss_window();
    if (abc)
        hipLaunchKernelGGL(k_ssim_fwd<true>, g, dim3(kQThreads), 0, s, H, W, img1, img2, valid, w, abc, partial);
    else
        hipLaunchKernelGGL(k_ssim_fwd<false>, g, dim3(kQThreads), 0, s, H, W, img1, img2, valid, w, abc, partial);
    const double n_map = valid ? (double)C * (H - 2 * kHalo) * (W - 2 * kHalo) : (double)C * H * W;
    const double n_all = (double)C * H * W;
    hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(1024), 0, s, (int)(g.x * g.y * g.z), 2, partial, 1.0 / n_map,
                       1.0 / n_all, out);
}

void launch_ssim_backward(int C, int H, int W, const float* img1, const float* img2, const float* abc,
                          const float* coef, float* grad1, hipStream_t s)
{
    hipLaunchKernelGGL(k_ssim_bwd, ssim_grid(C, H, W), dim3(kQThreads), 0, s, H, W, img1, img2, abc, gauss_window(), coef,
                       grad1);
}

int depth_l1_blocks(long n) { return (int)std::min<long>(2048, (n + 255) / 256); }

void launch_depth_l1_forward(long n, const float* inv, const float* mono, const float* mask, float* partial,
                             float* out, hipStream_t s)
{
    const int nb = depth_l1_blocks(n);
    hipLaunchKernelGGL(k_depth_l1_fwd, dim3(nb), dim3(256), 0, s, n, inv, mono, mask, partial);
    hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(1024), 0, s, nb, 1, partial, 1.0 / (double)n, 0.0, out);
}

void launch_depth_l1_backward(long n, const float* inv, const float* mono, const float* mask, const float* coef,
                              float* grad, hipStream_t s)
{
    hipLaunchKernelGGL(k_depth_l1_bwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, inv, mono, mask, coef,
                       grad);
}

}  // namespace hlgs
