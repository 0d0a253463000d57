// optim.hip -- sparse Adam step of the alt rasterizer's SparseGaussianAdam for gfx950.
//
// Reference: submodules/alt-rasterizer/cuda_rasterizer/adam.cu:9-36 (adamUpdateCUDA), bound as
// _C.adamUpdate (rasterize_points.cu:255-281) and driven by SparseGaussianAdam.step
// (alt_gaussian_rasterization/__init__.py:244-271).  Element p of an N x M parameter belongs to Gaussian
// p / M and is updated only when that Gaussian is visible; there is no bias correction and no step count.
//
// HBM-bound streaming update: 28 bytes per visible element (param, grad, m, v in; param, m, v out) plus one
// visibility byte per Gaussian.  Each thread owns four consecutive elements and moves them as float4 when
// all four are visible; invisible elements are neither read nor written, so a sparse step only pays for
// the visible rows.
//
// k_adam_multi: the dense per-step Adam of train_post.py:793-812 (OurAdam._single_tensor_adam2,
// scene/OurAdam.py:357-448) over all six parameter tensors of the resident Gaussians in one launch, with the
// skybox gradient rows zeroed first (train_post.py:786-791).  HBM-bound: 28 bytes per element.
#include <algorithm>

#include "hlgs_internal.h"

namespace hlgs {

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, float lr, float b1, float b2, float eps)
{
    m = b1 * m + (1.0f - b1) * g;
    v = b2 * v + (1.0f - b2) * g * g;
    p += -lr * m / (sqrtf(v) + eps);
}

__global__ void __launch_bounds__(256) k_adam(float* __restrict__ param, const float* __restrict__ grad,
                                              float* __restrict__ exp_avg, float* __restrict__ exp_avg_sq,
                                              const uint8_t* __restrict__ vis, float lr, float b1, float b2,
                                              float eps, uint32_t N, uint32_t M, int vec)
{
    const uint64_t total = (uint64_t)N * M;
    const uint64_t e0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (e0 >= total) return;
    bool on[4];
    int n_on = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint64_t e = e0 + k;
        on[k] = e < total && vis[(uint32_t)(e / M)];
        n_on += on[k];
    }
    if (n_on == 0) return;
    if (vec && n_on == 4) {
        float4 p = *reinterpret_cast<const float4*>(param + e0);
        const float4 g = *reinterpret_cast<const float4*>(grad + e0);
        float4 m = *reinterpret_cast<const float4*>(exp_avg + e0);
        float4 v = *reinterpret_cast<const float4*>(exp_avg_sq + e0);
        adam_one(p.x, g.x, m.x, v.x, lr, b1, b2, eps);
        adam_one(p.y, g.y, m.y, v.y, lr, b1, b2, eps);
        adam_one(p.z, g.z, m.z, v.z, lr, b1, b2, eps);
        adam_one(p.w, g.w, m.w, v.w, lr, b1, b2, eps);
        *reinterpret_cast<float4*>(param + e0) = p;
        *reinterpret_cast<float4*>(exp_avg + e0) = m;
        *reinterpret_cast<float4*>(exp_avg_sq + e0) = v;
        return;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (!on[k]) continue;
        const uint64_t e = e0 + k;
        float p = param[e], m = exp_avg[e], v = exp_avg_sq[e];
        adam_one(p, grad[e], m, v, lr, b1, b2, eps);
        param[e] = p;
        exp_avg[e] = m;
        exp_avg_sq[e] = v;
    }
}

void launch_adam(float* param, const float* grad, float* m, float* v, const uint8_t* vis, float lr, float b1, float b2,
                 float eps, uint32_t N, uint32_t M, hipStream_t s)
{
    const uint64_t total = (uint64_t)N * M;
    const uint64_t threads = (total + 3) / 4;
    const int vec = ((((uintptr_t)param | (uintptr_t)grad | (uintptr_t)m | (uintptr_t)v) & 15u) == 0) ? 1 : 0;
    hipLaunchKernelGGL(k_adam, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, param, grad, m, v, vis, lr, b1,
                       b2, eps, N, M, vec);
}

// torch's float32 sequence: exp_avg.mul_(b1).add_(g, alpha=1-b1); exp_avg_sq.mul_(b2).addcmul_(g, g, value=1-b2);
// denom = (exp_avg_sq.sqrt() / bc2_sqrt).add_(eps); param.addcdiv_(exp_avg, denom, value=-step_size).  The two
// multiply-adds are fused as the GPU build of those torch kernels fuses them.
__device__ __forceinline__ void adam_dense(float& p, float g, float& m, float& v, float ns, float b1, float a1, float b2,
                                           float a2, float bc2s, float eps)
{
#pragma clang fp contract(off)
    m = fmaf(a1, g, m * b1);
    v = fmaf(a2 * g, g, v * b2);
    const float den = sqrtf(v) / bc2s + eps;
    p = (ns * m) / den + p;
}

struct AdamTabs {
    AdamTensor t[kMaxRowTables];
};

__global__ void __launch_bounds__(256) k_adam_multi(AdamTabs tabs, int sky, float b1, float a1, float b2, float a2,
                                                    float bc2s, float eps)
{
    const AdamTensor& t = tabs.t[blockIdx.y];
    const int64_t n = t.numel, zero_end = std::min<int64_t>((int64_t)sky * t.row_elems, n);
    const bool vec = ((((uintptr_t)t.param | (uintptr_t)t.grad | (uintptr_t)t.exp_avg | (uintptr_t)t.exp_avg_sq) & 15u) == 0);
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    for (; e < n; e += stride * 4) {
        if (vec && e + 4 <= n && e >= zero_end) {
            float4 p = *reinterpret_cast<const float4*>(t.param + e);
            const float4 g = *reinterpret_cast<const float4*>(t.grad + e);
            float4 m = *reinterpret_cast<const float4*>(t.exp_avg + e);
            float4 v = *reinterpret_cast<const float4*>(t.exp_avg_sq + e);
            adam_dense(p.x, g.x, m.x, v.x, t.neg_step_size, b1, a1, b2, a2, bc2s, eps);
            adam_dense(p.y, g.y, m.y, v.y, t.neg_step_size, b1, a1, b2, a2, bc2s, eps);
            adam_dense(p.z, g.z, m.z, v.z, t.neg_step_size, b1, a1, b2, a2, bc2s, eps);
            adam_dense(p.w, g.w, m.w, v.w, t.neg_step_size, b1, a1, b2, a2, bc2s, eps);
            *reinterpret_cast<float4*>(t.param + e) = p;
            *reinterpret_cast<float4*>(t.exp_avg + e) = m;
            *reinterpret_cast<float4*>(t.exp_avg_sq + e) = v;
            continue;
        }
        for (int64_t k = e; k < std::min<int64_t>(e + 4, n); k++) {
            float g = t.grad[k];
            if (k < zero_end) {
                g = 0.f;
                t.grad[k] = 0.f;
            }
            float p = t.param[k], m = t.exp_avg[k], v = t.exp_avg_sq[k];
            adam_dense(p, g, m, v, t.neg_step_size, b1, a1, b2, a2, bc2s, eps);
            t.param[k] = p;
            t.exp_avg[k] = m;
            t.exp_avg_sq[k] = v;
        }
    }
}

void launch_adam_multi(int T, const AdamTensor* t, int sky, float b1, float a1, float b2, float a2, float bc2_sqrt,
                       float eps, hipStream_t s)
{
    AdamTabs at{};
    int64_t most = 0;
    for (int i = 0; i < T; i++) {
        at.t[i] = t[i];
        most = std::max<int64_t>(most, t[i].numel);
    }
    const int64_t blocks = std::min<int64_t>((most + 1023) / 1024, 8192);
    if (blocks > 0)
        hipLaunchKernelGGL(k_adam_multi, dim3((unsigned)blocks, T), dim3(256), 0, s, at, sky, b1, a1, b2, a2, bc2_sqrt,
                           eps);
}

}  // namespace hlgs
