// valu_probe.hip -- what VALU issue rate a SIMD reaches for dependent vs independent f32 chains, at 1..8 waves per
// SIMD (the question behind the blend kernels' ~1 VALU per SIMD quad-cycle).  Each wave runs ITERS loop
// iterations of 64 v_fma_f32 spread over C independent accumulators (C = 1: one dependent chain), optionally with
// every 16th instruction a v_exp_f32 in the chain.  Prints wave-instructions per second and the fraction of the
// 2-cycle wave64 ceiling (256 CUs x 4 SIMDs x clock / 2).
//   hipcc --offload-arch=gfx950 -O3 -o valu_probe tools/valu_probe.hip && ./valu_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048;

template <int C, bool EXP>
__global__ void __launch_bounds__(64) k_probe(float* out, float b, float c)
{
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1.f, a2 = a0 + 2.f, a3 = a0 + 3.f;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int k = 0; k < 64; k += 4) {
            if (C == 1) {
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c));
                if (EXP && k % 16 == 12) asm volatile("v_exp_f32 %0, %0" : "+v"(a0));
                else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c));
            } else if (C == 2) {
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a1) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c));
                if (EXP && k % 16 == 12) asm volatile("v_exp_f32 %0, %0" : "+v"(a1));
                else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a1) : "v"(b), "v"(c));
            } else {
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a1) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a2) : "v"(b), "v"(c));
                if (EXP && k % 16 == 12) asm volatile("v_exp_f32 %0, %0" : "+v"(a3));
                else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a3) : "v"(b), "v"(c));
            }
        }
    }
    out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3;
}

template <int C, bool EXP>
static int run(float* out, int waves_per_simd, int simds, double clock_ghz)
{
    const int blocks = simds * waves_per_simd;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_probe<C, EXP>), dim3(blocks), dim3(64), 0, 0, out, 0.999f, 1e-3f);  // warm-up
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL((k_probe<C, EXP>), dim3(blocks), dim3(64), 0, 0, out, 0.999f, 1e-3f);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 5.f;
    const double instr = (double)blocks * ITERS * 64;
    const double rate = instr / (ms * 1e-3) / 1e9;
    const double ceil2 = simds * clock_ghz / 2.0;
    printf("{\"chains\": %d, \"exp_every_16\": %s, \"waves_per_simd\": %d, \"ms\": %.4f, \"Ginstr_s\": %.1f, "
           "\"frac_of_2cyc\": %.3f, \"per_simd_quad_cycle\": %.3f}\n",
           C, EXP ? "true" : "false", waves_per_simd, ms, rate, rate / ceil2, rate / (simds * clock_ghz / 4.0));
    CHK(hipEventDestroy(e0));
    CHK(hipEventDestroy(e1));
    return 0;
}

int main()
{
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int simds = p.multiProcessorCount * 4;
    const double clock_ghz = 2.4;  // nominal; the rates are also reported per quad-cycle at this clock
    printf("# %s, %d CUs, %d SIMDs, nominal %.1f GHz\n", p.gcnArchName, p.multiProcessorCount, simds, clock_ghz);
    float* out;
    CHK(hipMalloc(&out, (size_t)simds * 8 * 64 * sizeof(float)));
    const int ws[] = {1, 2, 4, 5, 8};
    for (int w : ws) {
        if (run<1, false>(out, w, simds, clock_ghz)) return 1;
        if (run<2, false>(out, w, simds, clock_ghz)) return 1;
        if (run<4, false>(out, w, simds, clock_ghz)) return 1;
        if (run<1, true>(out, w, simds, clock_ghz)) return 1;
        if (run<4, true>(out, w, simds, clock_ghz)) return 1;
    }
    CHK(hipFree(out));
    return 0;
}
