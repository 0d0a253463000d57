// scan.hip -- device-wide inclusive prefix sum over uint32 (reduce-then-scan, recursive on block
// totals).  Replaces the reference's cub::DeviceScan::InclusiveSum calls
// (rasterizer_impl.cu:322, runtime_switching.cu:774-776) with a hand-written wave64 scan.
#include "hlgs_internal.h"

namespace hlgs {

size_t scan_scratch_elems(size_t n)
{
    size_t total = 0;
    while (n > (size_t)kScanItems) {
        n = (n + kScanItems - 1) / kScanItems;
        total += n;
    }
    return total + 1;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane)
{
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

// 256 threads x 8 items; in-place safe (each block reads its range before writing it).
__global__ void __launch_bounds__(256) k_scan_block(const uint32_t* in, uint32_t* out, uint32_t* partials, size_t n)
{
    __shared__ uint32_t wsum[4];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const size_t base = (size_t)blockIdx.x * kScanItems + (size_t)tid * 8;
    uint32_t v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = (base + i < n) ? in[base + i] : 0u;
#pragma unroll
    for (int i = 1; i < 8; i++) v[i] += v[i - 1];
    uint32_t incl = wave_incl_scan(v[7], lane);
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    uint32_t woff = 0;
    for (int w = 0; w < wid; w++) woff += wsum[w];
    const uint32_t excl = woff + incl - v[7];
#pragma unroll
    for (int i = 0; i < 8; i++)
        if (base + i < n) out[base + i] = v[i] + excl;
    if (tid == 255) partials[blockIdx.x] = woff + incl;
}

__global__ void __launch_bounds__(256) k_scan_add(uint32_t* out, const uint32_t* partials, size_t n)
{
    if (blockIdx.x == 0) return;
    const uint32_t add = partials[blockIdx.x - 1];
    const size_t base = (size_t)blockIdx.x * kScanItems + threadIdx.x;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        size_t e = base + (size_t)i * 256;
        if (e < n) out[e] += add;
    }
}

void scan_inclusive_u32(const uint32_t* in, uint32_t* out, size_t n, uint32_t* tmp, hipStream_t s)
{
    if (n == 0) return;
    const size_t nb = (n + kScanItems - 1) / kScanItems;
    hipLaunchKernelGGL(k_scan_block, dim3((unsigned)nb), dim3(256), 0, s, in, out, tmp, n);
    if (nb > 1) {
        scan_inclusive_u32(tmp, tmp, nb, tmp + nb, s);
        hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nb), dim3(256), 0, s, out, tmp, n);
    }
}

}  // namespace hlgs
