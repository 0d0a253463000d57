// act.hip -- the parameter activations of the training step in one pass over the resident rows.
//
// Reference semantics (scene/gaussian_model.py:44-56, get_opacity / get_scaling / get_rotation, read by render() at
// gaussian_renderer/__init__.py and train_post.py's render_post): opacity = sigmoid(_opacity), scales =
// exp(_scaling), rotations = torch.nn.functional.normalize(_rotation) (eps 1e-12).  train_post.py applies them to
// every resident row each step, and torch runs each as its own elementwise kernel (sigmoid, exp, the norm reduction,
// clamp_min, the division) forward and again backward (sigmoid_backward, the exp product, and the division / norm
// chain).  Here one thread per Gaussian row reads its three raw rows once and writes the three activated rows; the
// backward reads the upstream gradients and writes the raw-parameter gradients in one pass as well.
//
// Operation order follows torch's kernels: sigmoid(x) = 1 / (1 + exp(-x)); its gradient (g (1 - y)) y; exp's gradient
// g y; normalize = x / max(||x||, eps), whose gradient through the division and the norm is
// g / d - x (sum_j g_j x_j) / d^2 / ||x|| (the second term only while ||x|| > eps, where clamp_min passes it).
#include "hlgs_internal.h"

namespace hlgs {

__global__ void __launch_bounds__(256) k_act_fwd(int64_t n, const float* __restrict__ op_raw,
                                                 const float* __restrict__ sc_raw, const float4* __restrict__ rot_raw,
                                                 float* __restrict__ op, float* __restrict__ sc,
                                                 float4* __restrict__ rot)
{
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float o = op_raw[i];
    const float s0 = sc_raw[3 * i], s1 = sc_raw[3 * i + 1], s2 = sc_raw[3 * i + 2];
    const float4 q = rot_raw[i];
    op[i] = 1.0f / (1.0f + expf(-o));
    sc[3 * i] = expf(s0);
    sc[3 * i + 1] = expf(s1);
    sc[3 * i + 2] = expf(s2);
    const float d = fmaxf(sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w), 1e-12f);
    rot[i] = make_float4(q.x / d, q.y / d, q.z / d, q.w / d);
}

__global__ void __launch_bounds__(256) k_act_bwd(int64_t n, const float* __restrict__ op, const float* __restrict__ sc,
                                                 const float4* __restrict__ rot_raw, const float* __restrict__ g_op,
                                                 const float* __restrict__ g_sc, const float4* __restrict__ g_rot,
                                                 float* __restrict__ d_op, float* __restrict__ d_sc,
                                                 float4* __restrict__ d_rot)
{
#pragma clang fp contract(off)
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    if (g_op) {
        const float y = op[i];
        d_op[i] = (g_op[i] * (1.0f - y)) * y;
    }
    if (g_sc) {
#pragma unroll
        for (int k = 0; k < 3; k++) d_sc[3 * i + k] = g_sc[3 * i + k] * sc[3 * i + k];
    }
    if (g_rot) {
        const float4 x = rot_raw[i], g = g_rot[i];
        const float nrm = sqrtf(x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w);
        const float d = fmaxf(nrm, 1e-12f);
        float4 r = make_float4(g.x / d, g.y / d, g.z / d, g.w / d);
        if (nrm > 1e-12f) {
            const float gd = -(g.x * x.x + g.y * x.y + g.z * x.z + g.w * x.w) / (d * d);  // dL/dd
            const float c = gd / nrm;                                                        // d||x||/dx = x / ||x||
            r.x += c * x.x;
            r.y += c * x.y;
            r.z += c * x.z;
            r.w += c * x.w;
        }
        d_rot[i] = r;
    }
}

void launch_act_fwd(int64_t n, const float* op_raw, const float* sc_raw, const float* rot_raw, float* op, float* sc,
                    float* rot, hipStream_t s)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(k_act_fwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, op_raw, sc_raw,
                       reinterpret_cast<const float4*>(rot_raw), op, sc, reinterpret_cast<float4*>(rot));
}

void launch_act_bwd(int64_t n, const float* op, const float* sc, const float* rot_raw, const float* g_op,
                    const float* g_sc, const float* g_rot, float* d_op, float* d_sc, float* d_rot, hipStream_t s)
{
    if (n <= 0) return;
    hipLaunchKernelGGL(k_act_bwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, op, sc,
                       reinterpret_cast<const float4*>(rot_raw), g_op, g_sc, reinterpret_cast<const float4*>(g_rot),
                       d_op, d_sc, reinterpret_cast<float4*>(d_rot));
}

}  // namespace hlgs
