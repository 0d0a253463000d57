// loss.hip -- fused photometric loss kernels for gfx950: SSIM (11x11 Gaussian window, sigma 1.5) with its
// gradient, L1 and the masked inverse-depth L1 of the training step.
//
// Reference semantics: utils/loss_utils.py:17-63 (l1_loss, ssim/_ssim: F.conv2d with the window of
// create_window, zero padding window_size // 2, C1 = 0.01^2, C2 = 0.03^2, map mean), the un-vendored
// fused_ssim package train_post.py:29, 559 calls (same map; padding "same" = the zero-padded map, "valid" = its
// interior [5, H-5) x [5, W-5)), and the depth term of train_single.py:111-118
// (mean |(invdepth - mono) * mask|).
//
// Design (round 5): one plane (channel) per grid.z, a 128 x 16 output tile per 256-thread workgroup, the two
// separable passes with the first one in registers:
//   horizontal: thread t < 208 owns input row t >> 3 of the tile's 26 (its 16 output rows and the 5-row halo above
//               and below) and the 16 output columns [16 s, 16 s + 16), s = t & 7: it loads the 26 input pixels of
//               that run (eight aligned 16-byte loads per image when W is a multiple of 4; zero outside the image:
//               zero padding), forms each moment (x, y, x^2, y^2, x y) and writes its 16 11-tap row sums to LDS;
//   vertical:   thread t owns output column t & 127 and output rows [8 q, 8 q + 8), q = t >> 7: 18 row sums per
//               moment down its column (conflict-free: a wave reads 64 consecutive columns) give the window sums,
//               and the per-pixel outputs go out as 256-byte rows.
// The sums are the round-4 kernel's fmaf chains in the same order (horizontal first, tap 0 to 10, then vertical), so
// every per-pixel value -- the SSIM map, the A, B, C maps, the gradient -- is bit-identical to it; only the
// workgroup partial sums of the loss are added in another grouping.  Round 4 staged both images with the halo in LDS
// and ran the horizontal pass over all 18 rows of each 64 x 8 tile (2.25 horizontal passes per output) and the
// vertical pass from LDS: 103 us forward and 85 us backward at 3 x 1080 x 1920 (loss_r04.hip, tools/variants/INDEX.md).
// The forward writes the partial derivatives of the SSIM map with respect to the window means
//   A = df/dmu1 (total), B = df/d E[x^2], C = df/d E[x y]
// so that dSSIM/dx(p) = sum_q g(q) w(q - p) (A(q) + 2 x(p) B(q) + y(p) C(q)), which the backward evaluates with
// the same two passes over the three maps.  Per-workgroup sums go to a partial array that one block reduces in
// double, in a fixed order: the losses are deterministic.
#include <algorithm>

#include "hlgs_internal.h"

namespace hlgs {

constexpr int kHalo = 5;
constexpr int kQW = 128;                 // output columns per tile
constexpr int kQH = 16;                  // output rows per tile
constexpr int kQRows = kQH + 2 * kHalo;  // input rows per tile (26)
constexpr int kQSeg = 16;                // output columns per horizontal-pass thread
constexpr int kQIn = kQSeg + 2 * kHalo;  // input pixels per horizontal-pass thread (26)
constexpr int kQR = 8;                   // output rows per vertical-pass thread
constexpr int kQS = 132;                 // LDS row stride (floats)
constexpr int kQThreads = 256;
constexpr float kC1 = 0.01f * 0.01f, kC2 = 0.03f * 0.03f;
static_assert(kQRows * (kQW / kQSeg) <= kQThreads && kQW * 2 == kQThreads && 2 * kQR == kQH, "tile shape");

struct Win11 {
    float w[11];
};

// The 26 input pixels of a horizontal-pass thread, columns x0 - 5 + c0 + [0, 26) of row gy (zero outside the image).
__device__ __forceinline__ void load_run26(const float* __restrict__ plane, int H, int W, int gy, int xs,
                                           float (&v)[kQIn])
{
    const bool rowin = gy >= 0 && gy < H;
    const float* rowp = plane + (size_t)min(max(gy, 0), H - 1) * W;
    if ((W & 3) == 0) {  // eight aligned float4 groups [xs - 3, xs + 29), each wholly inside or outside the image
        const int a0 = xs - 3;
        float f[32];
#pragma unroll
        for (int g4 = 0; g4 < 8; g4++) {
            const int c = a0 + 4 * g4;
            const bool in = rowin && c >= 0 && c < W;
            const float4 q = *reinterpret_cast<const float4*>(rowp + min(max(c, 0), W - 4));
            f[4 * g4] = in ? q.x : 0.f;
            f[4 * g4 + 1] = in ? q.y : 0.f;
            f[4 * g4 + 2] = in ? q.z : 0.f;
            f[4 * g4 + 3] = in ? q.w : 0.f;
        }
#pragma unroll
        for (int i = 0; i < kQIn; i++) v[i] = f[i + 3];
    } else {
#pragma unroll
        for (int i = 0; i < kQIn; i++) {
            const int c = xs + i;
            const float q = rowp[min(max(c, 0), W - 1)];
            v[i] = rowin && c >= 0 && c < W ? q : 0.f;
        }
    }
}

// 16 row sums of one moment (fmaf over taps 0..10, the round-4 order) into LDS row `dst`
__device__ __forceinline__ void row_sums16(const float (&f)[kQIn], const Win11& win, float* dst)
{
    float o[kQSeg];
#pragma unroll
    for (int i = 0; i < kQSeg; i++) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 11; k++) acc = fmaf(win.w[k], f[i + k], acc);
        o[i] = acc;
    }
#pragma unroll
    for (int u = 0; u < kQSeg / 4; u++)
        *reinterpret_cast<float4*>(dst + 4 * u) = make_float4(o[4 * u], o[4 * u + 1], o[4 * u + 2], o[4 * u + 3]);
}

// Vertical pass of one moment: the window sums of output rows [8 q, 8 q + 8) of column c
__device__ __forceinline__ void col_sums8(const float* hs_m, const Win11& win, int c, int q, float (&out)[kQR])
{
    float v[kQR + 2 * kHalo];
#pragma unroll
    for (int r = 0; r < kQR + 2 * kHalo; r++) v[r] = hs_m[(kQR * q + r) * kQS + c];
#pragma unroll
    for (int jj = 0; jj < kQR; jj++) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 11; k++) acc = fmaf(win.w[k], v[jj + k], acc);
        out[jj] = acc;
    }
}

// SSIM forward.  partial[2 * block] = (sum of the SSIM map over counted pixels, sum |x - y|).
// CLAMP: img1 enters as clamp(img1, 0, 1) -- the rendered_image.clamp(0, 1) of the reference's renderers
// (gaussian_renderer/__init__.py:142, 612) folded into the loss's own loads; NaN stays NaN, as torch.clamp keeps it.
__device__ __forceinline__ float clamp01(float v) { return v < 0.f ? 0.f : (v > 1.f ? 1.f : v); }

template <bool TRAIN, bool CLAMP>
__global__ void __launch_bounds__(kQThreads) k_ssim_fwd(int H, int W, const float* __restrict__ img1,
                                                        const float* __restrict__ img2, int valid, Win11 win,
                                                        float* __restrict__ abc, float* __restrict__ partial)
{
    __shared__ __attribute__((aligned(16))) float hs[5][kQRows * kQS];
    __shared__ float red[2][kQThreads / 64];
    const int ch = blockIdx.z;
    const size_t HW = (size_t)H * W;
    const float* x = img1 + ch * HW;
    const float* y = img2 + ch * HW;
    const int x0 = blockIdx.x * kQW, y0 = blockIdx.y * kQH;
    const int t = threadIdx.x;
    if (t < kQRows * (kQW / kQSeg)) {
        const int r = t >> 3, c0 = kQSeg * (t & 7);
        const int gy = y0 - kHalo + r, xs = x0 - kHalo + c0;
        float u[kQIn], v[kQIn], f[kQIn];
        load_run26(x, H, W, gy, xs, u);
        load_run26(y, H, W, gy, xs, v);
        if (CLAMP) {
#pragma unroll
            for (int i = 0; i < kQIn; i++) u[i] = clamp01(u[i]);
        }
        float* row = &hs[0][r * kQS + c0];
        row_sums16(u, win, row);
        row_sums16(v, win, row + kQRows * kQS);
#pragma unroll
        for (int i = 0; i < kQIn; i++) f[i] = u[i] * u[i];
        row_sums16(f, win, row + 2 * kQRows * kQS);
#pragma unroll
        for (int i = 0; i < kQIn; i++) f[i] = v[i] * v[i];
        row_sums16(f, win, row + 3 * kQRows * kQS);
#pragma unroll
        for (int i = 0; i < kQIn; i++) f[i] = u[i] * v[i];
        row_sums16(f, win, row + 4 * kQRows * kQS);
    }
    __syncthreads();
    const int c = t & (kQW - 1), q = t / kQW;
    float mo[5][kQR];
#pragma unroll
    for (int m = 0; m < 5; m++) col_sums8(hs[m], win, c, q, mo[m]);
    const int px = x0 + c;
    float s_map = 0.f, s_l1 = 0.f;
    if (px < W) {
#pragma unroll
        for (int jj = 0; jj < kQR; jj++) {
            const int py = y0 + kQR * q + jj;
            if (py >= H) break;
            const size_t pid = (size_t)py * W + px;
            const float m1 = mo[0][jj], m2 = mo[1][jj], e11 = mo[2][jj], e22 = mo[3][jj], e12 = mo[4][jj];
            const bool counted = !valid || (px >= kHalo && px < W - kHalo && py >= kHalo && py < H - kHalo);
            const float mu1_sq = m1 * m1, mu2_sq = m2 * m2, mu12 = m1 * m2;
            const float s11 = e11 - mu1_sq, s22 = e22 - mu2_sq, s12 = e12 - mu12;
            const float a = 2.f * mu12 + kC1, b = 2.f * s12 + kC2;
            const float cc = mu1_sq + mu2_sq + kC1, d = s11 + s22 + kC2;
            const float fm = (a * b) / (cc * d);
            if (counted) s_map += fm;
            s_l1 += fabsf((CLAMP ? clamp01(x[pid]) : x[pid]) - y[pid]);
            if (TRAIN) {
                float A = 0.f, B = 0.f, C = 0.f;
                if (counted) {
                    const float cd = cc * d;
                    const float dmu1 = (2.f * m2 * b) / cd - fm * (2.f * m1) / cc;  // df/dmu1 at fixed sigmas
                    B = -fm / d;                                                  // df/dsigma1^2
                    C = (2.f * a) / cd;                                           // df/dsigma12
                    A = dmu1 - 2.f * m1 * B - m2 * C;                             // through sigma = E[.] - mu mu
                }
                float* o = abc + (size_t)ch * 3 * HW + pid;
                o[0] = A;
                o[HW] = B;
                o[2 * HW] = C;
            }
        }
    }
    // workgroup sums (fixed order: shuffles, then one lane per wave)
    for (int off = 32; off > 0; off >>= 1) {
        s_map += __shfl_xor(s_map, off, 64);
        s_l1 += __shfl_xor(s_l1, off, 64);
    }
    const int wave = t >> 6;
    if ((t & 63) == 0) { red[0][wave] = s_map; red[1][wave] = s_l1; }
    __syncthreads();
    if (t == 0) {
        float sa = 0.f, sb = 0.f;
        for (int i = 0; i < kQThreads / 64; i++) { sa += red[0][i]; sb += red[1][i]; }
        const size_t blk = ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        partial[2 * blk] = sa;
        partial[2 * blk + 1] = sb;
    }
}

// grad1 = coef[0] * dSSIM-map-sum/dx + coef[1] * sign(x - y)  (coefficients on the device: no host sync).  CLAMP: x is
// clamp(img1, 0, 1) and the gradient passes only where 0 <= img1 <= 1 (torch's clamp backward; 0 elsewhere and at NaN).
template <bool CLAMP>
__global__ void __launch_bounds__(kQThreads) k_ssim_bwd(int H, int W, const float* __restrict__ img1,
                                                        const float* __restrict__ img2, const float* __restrict__ abc,
                                                        Win11 win, const float* __restrict__ coef,
                                                        float* __restrict__ grad1)
{
    __shared__ __attribute__((aligned(16))) float hs[3][kQRows * kQS];
    const int ch = blockIdx.z;
    const size_t HW = (size_t)H * W;
    const int x0 = blockIdx.x * kQW, y0 = blockIdx.y * kQH;
    const float* maps = abc + (size_t)ch * 3 * HW;
    const int t = threadIdx.x;
    if (t < kQRows * (kQW / kQSeg)) {
        const int r = t >> 3, c0 = kQSeg * (t & 7);
        const int gy = y0 - kHalo + r, xs = x0 - kHalo + c0;
        float f[kQIn];
#pragma unroll
        for (int m = 0; m < 3; m++) {
            load_run26(maps + m * HW, H, W, gy, xs, f);
            row_sums16(f, win, &hs[m][r * kQS + c0]);
        }
    }
    __syncthreads();
    const int c = t & (kQW - 1), q = t / kQW;
    const int px = x0 + c;
    if (px >= W) return;
    float g[3][kQR];
#pragma unroll
    for (int m = 0; m < 3; m++) col_sums8(hs[m], win, c, q, g[m]);
    const float c0 = coef[0], c1 = coef[1];
#pragma unroll
    for (int jj = 0; jj < kQR; jj++) {
        const int py = y0 + kQR * q + jj;
        if (py >= H) break;
        const size_t pid = (size_t)ch * HW + (size_t)py * W + px;
        const float raw = img1[pid], yv = img2[pid];
        const float xv = CLAMP ? clamp01(raw) : raw;
        const float dssim = g[0][jj] + 2.f * xv * g[1][jj] + yv * g[2][jj];
        const float diff = xv - yv;
        const float sgn = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);  // torch.abs backward: sign, 0 at 0
        const float gv = c0 * dssim + c1 * sgn;
        grad1[pid] = !CLAMP || (raw >= 0.f && raw <= 1.f) ? gv : 0.f;
    }
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

static dim3 ssim_grid(int C, int H, int W) { return dim3((W + kQW - 1) / kQW, (H + kQH - 1) / kQH, C); }

size_t ssim_partials(int C, int H, int W)
{
    const dim3 g = ssim_grid(C, H, W);
    return (size_t)g.x * g.y * g.z;
}

void launch_ssim_forward(int C, int H, int W, const float* img1, const float* img2, int valid, float* abc,
                         float* partial, float* out, hipStream_t s, bool clamp1)
{
    const dim3 g = ssim_grid(C, H, W);
    const Win11 w = gauss_window();
#define HLGS_SSIMF(TR, CL) hipLaunchKernelGGL((k_ssim_fwd<TR, CL>), g, dim3(kQThreads), 0, s, H, W, img1, img2, valid, w, \
                                              abc, partial)
    if (abc) { if (clamp1) HLGS_SSIMF(true, true); else HLGS_SSIMF(true, false); }
    else { if (clamp1) HLGS_SSIMF(false, true); else HLGS_SSIMF(false, false); }
#undef HLGS_SSIMF
    const double n_map = valid ? (double)C * (H - 2 * kHalo) * (W - 2 * kHalo) : (double)C * H * W;
    const double n_all = (double)C * H * W;
    hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(1024), 0, s, (int)(g.x * g.y * g.z), 2, partial, 1.0 / n_map,
                       1.0 / n_all, out);
}

void launch_ssim_backward(int C, int H, int W, const float* img1, const float* img2, const float* abc,
                          const float* coef, float* grad1, hipStream_t s, bool clamp1)
{
    if (clamp1)
        hipLaunchKernelGGL(k_ssim_bwd<true>, ssim_grid(C, H, W), dim3(kQThreads), 0, s, H, W, img1, img2, abc,
                           gauss_window(), coef, grad1);
    else
        hipLaunchKernelGGL(k_ssim_bwd<false>, ssim_grid(C, H, W), dim3(kQThreads), 0, s, H, W, img1, img2, abc,
                           gauss_window(), coef, grad1);
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
