// issue_probe.hip -- which VALU instruction kinds a SIMD issues at the 2-cycle wave64 rate when several waves share
// it, and which hold it at one per 4 cycles (the question behind k_blend_bwd's ~1 VALU per SIMD quad-cycle with
// 4-5 waves per SIMD).  Each wave runs ITERS iterations of 32 instructions spread over 8 independent
// registers, all of one kind (or a 1:1 mix of FMA and that kind); prints wave-instructions per SIMD quad-cycle at
// the nominal clock for 1, 2, 4 and 8 waves per SIMD (2.0 = the 2-cycle ceiling, 1.0 = one per 4 cycles).
//   hipcc --offload-arch=gfx950 -O3 -o tools/issue_probe tools/issue_probe.hip && tools/issue_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 1024;

enum Kind { FMA, FMAC, MUL_SGPR, CNDMASK_VCC, CMP_SGPR, DPP_ADD, EXP, PERMLANE32, MIX_SALU, MIX_EXP, MIX_DPP, MIX_CMP,
            MIX_CND, MOV, CND_E64, CND_VCC_SET, CND_E64_SET, PK_FMA, PK_MUL, DPP_BCAST31, PERMLANE16, MIX_PK,
            FMA_HALF_LO, FMA_HALF_HI, FMA_QUARTER, FMA_ODD, EXP_HALF, NKINDS };
static const char* kNames[] = {"v_fma_f32", "v_fmac_f32", "v_mul_f32 sgpr", "v_cndmask vcc", "v_cmp->sgpr",
                               "v_add_f32_dpp", "v_exp_f32", "v_permlane32_swap", "fma+s_and 1:1", "fma+exp 3:1",
                               "fma+dpp 1:1", "fma+cmp 1:1", "fma+cndmask 1:1", "v_mov_b32", "v_cndmask_e64 s[10:11]",
                               "v_cndmask vcc (vcc set)", "v_cndmask_e64 (mask set)", "v_pk_fma_f32",
                               "v_pk_mul_f32", "v_add_f32_dpp row_bcast:31", "v_permlane16_swap", "fma+pk_fma 1:1",
                               "v_fma_f32 exec=lanes 0-31", "v_fma_f32 exec=lanes 32-63", "v_fma_f32 exec=lanes 0-15",
                               "v_fma_f32 exec=odd lanes", "v_exp_f32 exec=lanes 0-31"};

#define R8(op) op(0) op(1) op(2) op(3) op(4) op(5) op(6) op(7)

template <int K>
__global__ void __launch_bounds__(64) k_issue(float* out, float b, float c)
{
    float a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x * 1e-3f + i;
    const float s = b;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 pa[4] = {{a[0], a[1]}, {a[2], a[3]}, {a[4], a[5]}, {a[6], a[7]}};
    const f2 pb = {b, b}, pc = {c, c};
    const uint64_t msk = __builtin_amdgcn_ballot_w64(threadIdx.x & 1);
    if constexpr (K == CND_VCC_SET) asm volatile("v_cmp_lt_f32 vcc, %0, %1\n\ts_nop 4" : : "v"(a[0]), "v"(b) : "vcc");
    // partial exec masks: the loop body runs under a lane predicate (does the SIMD skip an idle 32-lane half?)
    bool on = true;
    if constexpr (K == FMA_HALF_LO || K == EXP_HALF) on = threadIdx.x < 32;
    if constexpr (K == FMA_HALF_HI) on = threadIdx.x >= 32;
    if constexpr (K == FMA_QUARTER) on = threadIdx.x < 16;
    if constexpr (K == FMA_ODD) on = threadIdx.x & 1;
    if (on)
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
#define OP(i)                                                                                                     \
    if constexpr (K == FMA) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));             \
    if constexpr (K == FMAC) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));               \
    if constexpr (K == MUL_SGPR) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(a[i]) : "s"(s));                    \
    if constexpr (K == CNDMASK_VCC) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b));        \
    if constexpr (K == CMP_SGPR) asm volatile("v_cmp_lt_f32 s[10:11], %0, %1" : : "v"(a[i]), "v"(b) : "s10", "s11"); \
    if constexpr (K == DPP_ADD)                                                                                   \
        asm volatile("v_add_f32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a[i])); \
    if constexpr (K == EXP) asm volatile("v_exp_f32 %0, %0" : "+v"(a[i]));                                      \
    if constexpr (K == PERMLANE32) {                                                                              \
        if ((i) & 1) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a[((i) + 7) & 7]), "+v"(a[i]));                 \
    }                                                                                                             \
    if constexpr (K == MIX_SALU) {                                                                                \
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));                                  \
        asm volatile("s_mov_b64 s[12:13], s[14:15]" : : : "s12", "s13");                               \
    }                                                                                                             \
    if constexpr (K == MIX_EXP) {                                                                                 \
        if ((i) % 4 == 3) asm volatile("v_exp_f32 %0, %0" : "+v"(a[i]));                                        \
        else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));                             \
    }                                                                                                             \
    if constexpr (K == MIX_DPP) {                                                                                 \
        if ((i) & 1) asm volatile("v_add_f32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a[i])); \
        else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));                             \
    }                                                                                                             \
    if constexpr (K == MIX_CMP) {                                                                                 \
        if ((i) & 1) asm volatile("v_cmp_lt_f32 s[10:11], %0, %1" : : "v"(a[i]), "v"(b) : "s10", "s11");         \
        else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));                             \
    }                                                                                                             \
    if constexpr (K == MIX_CND) {                                                                                 \
        if ((i) & 1) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b));                        \
        else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));                             \
    }                                                                                                             \
    if constexpr (K == MOV) asm volatile("v_mov_b32 %0, %1" : "=v"(a[i]) : "v"(a[((i) + 1) & 7]));                 \
    if constexpr (K == CND_E64) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[10:11]" : "+v"(a[i]) : "v"(b));   \
    if constexpr (K == CND_VCC_SET) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b));        \
    if constexpr (K == PK_FMA) {                                                                                  \
        if ((i) & 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(pa[(i) >> 1]) : "v"(pb), "v"(pc));      \
    }                                                                                                             \
    if constexpr (K == PK_MUL) {                                                                                  \
        if ((i) & 1) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(pa[(i) >> 1]) : "v"(pb));                   \
    }                                                                                                             \
    if constexpr (K == MIX_PK) {                                                                                  \
        if ((i) & 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(pa[(i) >> 1]) : "v"(pb), "v"(pc));      \
        else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));                             \
    }                                                                                                             \
    if constexpr (K == DPP_BCAST31)                                                                               \
        asm volatile("v_add_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xf bank_mask:0xf" : "+v"(a[i]));          \
    if constexpr (K == PERMLANE16) {                                                                              \
        if ((i) & 1) asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(a[((i) + 7) & 7]), "+v"(a[i]));         \
    }                                                                                                             \
    if constexpr (K == CND_E64_SET) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "s"(msk));  \
    if constexpr (K == FMA_HALF_LO || K == FMA_HALF_HI || K == FMA_QUARTER || K == FMA_ODD)                       \
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));                                 \
    if constexpr (K == EXP_HALF) asm volatile("v_exp_f32 %0, %0" : "+v"(a[i]));
            R8(OP)
#undef OP
        }
    }
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; i++) t += a[i];
#pragma unroll
    for (int i = 0; i < 4; i++) t += pa[i].x + pa[i].y;
    out[blockIdx.x * 64 + threadIdx.x] = t;
}

template <int K>
static int run(float* out, int wps, int simds, double clk)
{
    const int blocks = simds * wps;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_issue<K>, dim3(blocks), dim3(64), 0, 0, out, 0.999f, 1e-3f);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k_issue<K>, dim3(blocks), dim3(64), 0, 0, out, 0.999f, 1e-3f);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 5.f;
    const int per_iter = (K == PERMLANE32 || K == PERMLANE16 || K == PK_FMA || K == PK_MUL) ? 16 : 32;  // vector instructions per iteration
    const double instr = (double)blocks * ITERS * per_iter;
    printf("{\"kind\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"valu_per_simd_quad_cycle\": %.3f}\n", kNames[K],
           wps, ms, instr / (ms * 1e-3) / (simds * clk * 1e9 / 4.0));
    fflush(stdout);
    CHK(hipEventDestroy(e0));
    CHK(hipEventDestroy(e1));
    return 0;
}

template <int K>
static int sweep(float* out, int simds, double clk)
{
    const int ws[] = {1, 2, 4, 8};
    for (int w : ws)
        if (run<K>(out, w, simds, clk)) return 1;
    return 0;
}

int main()
{
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int simds = p.multiProcessorCount * 4;
    const double clk = 2.4;
    printf("# %s, %d CUs, nominal %.1f GHz\n", p.gcnArchName, p.multiProcessorCount, clk);
    float* out;
    CHK(hipMalloc(&out, (size_t)simds * 8 * 64 * sizeof(float)));
    if (sweep<FMA_HALF_LO>(out, simds, clk) || sweep<FMA_HALF_HI>(out, simds, clk) ||
        sweep<FMA_QUARTER>(out, simds, clk) || sweep<FMA_ODD>(out, simds, clk) || sweep<EXP_HALF>(out, simds, clk) ||
        sweep<EXP>(out, simds, clk) ||
        sweep<FMA>(out, simds, clk) || sweep<FMAC>(out, simds, clk) || sweep<CMP_SGPR>(out, simds, clk) ||
        sweep<DPP_ADD>(out, simds, clk) || sweep<EXP>(out, simds, clk) || sweep<PERMLANE32>(out, simds, clk) ||
        sweep<MIX_SALU>(out, simds, clk) || sweep<MIX_EXP>(out, simds, clk) || sweep<MIX_DPP>(out, simds, clk) ||
        sweep<MIX_CMP>(out, simds, clk) || sweep<MOV>(out, simds, clk) || sweep<PK_FMA>(out, simds, clk) ||
        sweep<PK_MUL>(out, simds, clk) || sweep<MIX_PK>(out, simds, clk) || sweep<DPP_BCAST31>(out, simds, clk) ||
        sweep<PERMLANE16>(out, simds, clk))
        return 1;
    CHK(hipFree(out));
    return 0;
}
