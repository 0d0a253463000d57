// loss.hip -- fused photometric loss kernels for gfx950: SSIM (11x11 Gaussian window, sigma 1.5) with its
// gradient, L1 and the masked inverse-depth L1 of the training step.
//
// Reference semantics: utils/loss_utils.py:17-63 (l1_loss, ssim/_ssim: F.conv2d with the window of
// create_window, zero padding window_size // 2, C1 = 0.01^2, C2 = 0.03^2, map mean), the un-vendored
// fused_ssim package train_post.py:29, 559 calls (same map; padding "same" = the zero-padded map, "valid" = its
// interior [5, H-5) x [5, W-5)), and the depth term of train_single.py:111-118
// (mean |(invdepth - mono) * mask|).
//
// Design: one plane (channel) per grid.z, a 64 x 8 output tile per 512-thread block.  The tile plus a 5-pixel
// halo of both images is staged in LDS; a horizontal 11-tap pass produces the five window sums
// (x, y, x^2, y^2, x y) per row, a vertical pass finishes them per output pixel.  The forward writes the
// partial derivatives of the SSIM map with respect to the window means
//   A = df/dmu1 (total), B = df/d E[x^2], C = df/d E[x y]
// so that dSSIM/dx(p) = sum_q g(q) w(q - p) (A(q) + 2 x(p) B(q) + y(p) C(q)), which the backward evaluates with
// the same separable stencil over the three maps.  Per-block sums go to a partial array that one block reduces
// in double, in a fixed order: the losses are deterministic.
#include <algorithm>

#include "hlgs_internal.h"

namespace hlgs {

constexpr int kLW = 64, kLH = 8, kHalo = 5, kSW = kLW + 2 * kHalo, kSH = kLH + 2 * kHalo;
constexpr float kC1 = 0.01f * 0.01f, kC2 = 0.03f * 0.03f;

struct Win11 {
    float w[11];
};

// Load a (kSH x kSW) tile of one plane at (x0 - 5, y0 - 5) into LDS; zero outside the image (zero padding).
__device__ __forceinline__ void load_halo(float (*dst)[kSW], const float* __restrict__ plane, int H, int W, int x0,
                                          int y0)
{
    for (int i = threadIdx.x; i < kSH * kSW; i += 512) {
        const int r = i / kSW, c = i - r * kSW;
        const int gy = y0 + r - kHalo, gx = x0 + c - kHalo;
        dst[r][c] = (gy >= 0 && gy < H && gx >= 0 && gx < W) ? plane[(size_t)gy * W + gx] : 0.f;
    }
}

// SSIM forward.  partial[2 * block] = (sum of the SSIM map over counted pixels, sum |x - y|).
template <bool TRAIN>
__global__ void __launch_bounds__(512) k_ssim_fwd(int H, int W, const float* __restrict__ img1,
                                                  const float* __restrict__ img2, int valid, Win11 win,
                                                  float* __restrict__ abc, float* __restrict__ partial)
{
    __shared__ float sx[kSH][kSW], sy[kSH][kSW];
    __shared__ float hs[5][kSH][kLW];
    __shared__ float red[2][8];
    const int ch = blockIdx.z;
    const size_t HW = (size_t)H * W;
    const float* x = img1 + ch * HW;
    const float* y = img2 + ch * HW;
    const int x0 = blockIdx.x * kLW, y0 = blockIdx.y * kLH;
    load_halo(sx, x, H, W, x0, y0);
    load_halo(sy, y, H, W, x0, y0);
    __syncthreads();
    for (int i = threadIdx.x; i < kSH * kLW; i += 512) {
        const int r = i / kLW, c = i - r * kLW;
        float a = 0.f, b = 0.f, aa = 0.f, bb = 0.f, ab = 0.f;
#pragma unroll
        for (int k = 0; k < 11; k++) {
            const float u = sx[r][c + k], v = sy[r][c + k], wk = win.w[k];
            a = fmaf(wk, u, a);
            b = fmaf(wk, v, b);
            aa = fmaf(wk, u * u, aa);
            bb = fmaf(wk, v * v, bb);
            ab = fmaf(wk, u * v, ab);
        }
        hs[0][r][c] = a; hs[1][r][c] = b; hs[2][r][c] = aa; hs[3][r][c] = bb; hs[4][r][c] = ab;
    }
    __syncthreads();
    const int tx = threadIdx.x & (kLW - 1), ty = threadIdx.x / kLW;
    const int px = x0 + tx, py = y0 + ty;
    float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
    for (int k = 0; k < 11; k++) {
        const float wk = win.w[k];
        m1 = fmaf(wk, hs[0][ty + k][tx], m1);
        m2 = fmaf(wk, hs[1][ty + k][tx], m2);
        e11 = fmaf(wk, hs[2][ty + k][tx], e11);
        e22 = fmaf(wk, hs[3][ty + k][tx], e22);
        e12 = fmaf(wk, hs[4][ty + k][tx], e12);
    }
    const bool inside = px < W && py < H;
    const bool counted = inside && (!valid || (px >= kHalo && px < W - kHalo && py >= kHalo && py < H - kHalo));
    float s_map = 0.f, s_l1 = 0.f;
    if (inside) {
        const float mu1_sq = m1 * m1, mu2_sq = m2 * m2, mu12 = m1 * m2;
        const float s11 = e11 - mu1_sq, s22 = e22 - mu2_sq, s12 = e12 - mu12;
        const float a = 2.f * mu12 + kC1, b = 2.f * s12 + kC2;
        const float c = mu1_sq + mu2_sq + kC1, d = s11 + s22 + kC2;
        const float f = (a * b) / (c * d);
        if (counted) s_map = f;
        s_l1 = fabsf(sx[ty + kHalo][tx + kHalo] - sy[ty + kHalo][tx + kHalo]);
        if (TRAIN) {
            float A = 0.f, B = 0.f, C = 0.f;
            if (counted) {
                const float cd = c * d;
                const float dmu1 = (2.f * m2 * b) / cd - f * (2.f * m1) / c;  // df/dmu1 at fixed sigmas
                B = -f / d;                                                  // df/dsigma1^2
                C = (2.f * a) / cd;                                          // df/dsigma12
                A = dmu1 - 2.f * m1 * B - m2 * C;                            // through sigma = E[.] - mu mu
            }
            const size_t pid = (size_t)py * W + px;
            float* o = abc + (size_t)ch * 3 * HW;
            o[pid] = A;
            o[HW + pid] = B;
            o[2 * HW + pid] = C;
        }
    }
    // block sums (fixed order: DPP-free shuffles then one lane per wave)
    for (int off = 32; off > 0; off >>= 1) {
        s_map += __shfl_xor(s_map, off, 64);
        s_l1 += __shfl_xor(s_l1, off, 64);
    }
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][wave] = s_map; red[1][wave] = s_l1; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float a = 0.f, b = 0.f;
        for (int i = 0; i < 8; i++) { a += red[0][i]; b += red[1][i]; }
        const size_t blk = ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        partial[2 * blk] = a;
        partial[2 * blk + 1] = b;
    }
}

// grad1 = coef[0] * dSSIM-map-sum/dx + coef[1] * sign(x - y)  (coefficients on the device: no host sync).
__global__ void __launch_bounds__(512) k_ssim_bwd(int H, int W, const float* __restrict__ img1,
                                                  const float* __restrict__ img2, const float* __restrict__ abc,
                                                  Win11 win, const float* __restrict__ coef,
                                                  float* __restrict__ grad1)
{
    __shared__ float sm[3][kSH][kSW];
    __shared__ float hs[3][kSH][kLW];
    const int ch = blockIdx.z;
    const size_t HW = (size_t)H * W;
    const int x0 = blockIdx.x * kLW, y0 = blockIdx.y * kLH;
    const float* maps = abc + (size_t)ch * 3 * HW;
    load_halo(sm[0], maps, H, W, x0, y0);
    load_halo(sm[1], maps + HW, H, W, x0, y0);
    load_halo(sm[2], maps + 2 * HW, H, W, x0, y0);
    __syncthreads();
    for (int i = threadIdx.x; i < kSH * kLW; i += 512) {
        const int r = i / kLW, c = i - r * kLW;
        float a = 0.f, b = 0.f, cc = 0.f;
#pragma unroll
        for (int k = 0; k < 11; k++) {
            const float wk = win.w[k];
            a = fmaf(wk, sm[0][r][c + k], a);
            b = fmaf(wk, sm[1][r][c + k], b);
            cc = fmaf(wk, sm[2][r][c + k], cc);
        }
        hs[0][r][c] = a; hs[1][r][c] = b; hs[2][r][c] = cc;
    }
    __syncthreads();
    const int tx = threadIdx.x & (kLW - 1), ty = threadIdx.x / kLW;
    const int px = x0 + tx, py = y0 + ty;
    if (px >= W || py >= H) return;
    float ga = 0.f, gb = 0.f, gc = 0.f;
#pragma unroll
    for (int k = 0; k < 11; k++) {
        const float wk = win.w[k];
        ga = fmaf(wk, hs[0][ty + k][tx], ga);
        gb = fmaf(wk, hs[1][ty + k][tx], gb);
        gc = fmaf(wk, hs[2][ty + k][tx], gc);
    }
    const size_t pid = (size_t)ch * HW + (size_t)py * W + px;
    const float xv = img1[pid], yv = img2[pid];
    const float dssim = ga + 2.f * xv * gb + yv * gc;
    const float diff = xv - yv;
    const float sgn = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);  // torch.abs backward: sign, 0 at 0
    grad1[pid] = coef[0] * dssim + coef[1] * sgn;
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

static dim3 ssim_grid(int C, int H, int W) { return dim3((W + kLW - 1) / kLW, (H + kLH - 1) / kLH, C); }

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
        hipLaunchKernelGGL(k_ssim_fwd<true>, g, dim3(512), 0, s, H, W, img1, img2, valid, w, abc, partial);
    else
        hipLaunchKernelGGL(k_ssim_fwd<false>, g, dim3(512), 0, s, H, W, img1, img2, valid, w, abc, partial);
    const double n_map = valid ? (double)C * (H - 2 * kHalo) * (W - 2 * kHalo) : (double)C * H * W;
    const double n_all = (double)C * H * W;
    hipLaunchKernelGGL(k_reduce_partials, dim3(1), dim3(1024), 0, s, (int)(g.x * g.y * g.z), 2, partial, 1.0 / n_map,
                       1.0 / n_all, out);
}

void launch_ssim_backward(int C, int H, int W, const float* img1, const float* img2, const float* abc,
                          const float* coef, float* grad1, hipStream_t s)
{
    hipLaunchKernelGGL(k_ssim_bwd, ssim_grid(C, H, W), dim3(512), 0, s, H, W, img1, img2, abc, gauss_window(), coef,
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
