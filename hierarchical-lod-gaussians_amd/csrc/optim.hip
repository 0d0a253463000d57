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

}  // namespace hlgs
