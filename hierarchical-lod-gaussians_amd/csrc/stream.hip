// stream.hip -- the SPT streaming step around the SPT cut for gfx950.
//
//   k_upper_cut     <- GaussianModel.cut_hierarchy_on_condition over the upper tree with the frustum-sphere
//                      cull and the LOD distance condition (scene/gaussian_model.py:108-140, 364-404;
//                      train_post.py:326-343), a level-synchronous walk in one workgroup
//   k_rows_gather / k_rows_scatter
//                   <- the cache's parameter and Adam-moment traffic: storage[idx].cuda() loads and
//                      storage[idx] = values.to(storage) write-backs (train_post.py:439-488).  Either side
//                      may be pinned host memory: the GPU reads and writes it directly over the host link
//                      instead of a CPU gather/scatter plus a copy.
#include "hlgs_internal.h"

namespace hlgs {

// ---------------------------------------------------------------- upper-tree cut
// Node columns: 2 child_count, 3 first_child, 4 next_sibling (HierarchyNode, types.h:60-67).
// Per level the frontier (the reference's `stack`) is filtered by the cull; leaves go to the cut, then the
// non-leaves whose condition is false, each group in frontier order; the next frontier is the first children
// of the expanded nodes in order, followed by their first children's next siblings in order.
__device__ __forceinline__ int cut_state(const CutArgs& a, int v)
{
#pragma clang fp contract(off)
    // 0 culled, 1 leaf -> cut, 2 condition false -> cut, 3 expand
    const float px = a.xyz[3 * v], py = a.xyz[3 * v + 1], pz = a.xyz[3 * v + 2];
    if (a.use_frustum) {
        const float r = a.bounds[v];
        for (int k = 0; k < 4; k++) {
            const float* pl = a.planes + 4 * k;
            const float sd = px * pl[0] + py * pl[1] + pz * pl[2] + pl[3];  // torch.sum over 3, then + distance
            if (sd + r < 0.f) return 0;
        }
    }
    if (a.nodes[6 * v + 2] == 0) return 1;
    if (a.use_lod) {
        const float dx = a.campos[0] - px, dy = a.campos[1] - py, dz = a.campos[2] - pz;
        const float d2 = dx * dx + dy * dy + dz * dz;
        if (!(a.min_dist2[v] > d2 * a.dmul)) return 2;
    }
    return 3;
}

// exclusive prefix of `flag` over the 1024-thread block; returns the block total in *total
__device__ __forceinline__ int block_excl(int flag, int* s_w, int* total)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t b = __ballot(flag);
    const int in_wave = __popcll(b & ((1ull << lane) - 1ull));
    __syncthreads();
    if (lane == 0) s_w[w] = __popcll(b);
    __syncthreads();
    int before = 0, t = 0;
    for (int i = 0; i < 16; i++) {
        const int c = s_w[i];
        if (i < w) before += c;
        t += c;
    }
    *total = t;
    return before + in_wave;
}

__global__ void __launch_bounds__(1024) k_upper_cut(CutArgs a)
{
    __shared__ int s_w[16];
    int* front = a.front_a;
    int* next = a.front_b;
    int size = a.N > 0 ? 1 : 0;
    if (threadIdx.x == 0) front[0] = 0;  // root_node = 0
    int total = 0;
    bool overflow = false;
    __syncthreads();
    while (size > 0 && !overflow) {
        // pass 1: level totals of the three outcomes
        int n1 = 0, n2 = 0, n3 = 0;
        for (int c0 = 0; c0 < size; c0 += 1024) {
            const int i = c0 + threadIdx.x;
            const int st = i < size ? cut_state(a, front[i]) : 0;
            int t1, t2, t3;
            block_excl(st == 1, s_w, &t1);
            block_excl(st == 2, s_w, &t2);
            block_excl(st == 3, s_w, &t3);
            n1 += t1; n2 += t2; n3 += t3;
        }
        if (total + n1 + n2 > a.capacity || 2 * n3 > a.capacity) { overflow = true; break; }
        // pass 2: write the cut and the next frontier in the reference's order
        int o1 = 0, o2 = 0, o3 = 0;
        for (int c0 = 0; c0 < size; c0 += 1024) {
            const int i = c0 + threadIdx.x;
            const int v = i < size ? front[i] : 0;
            const int st = i < size ? cut_state(a, v) : 0;
            int t1, t2, t3;
            const int p1 = block_excl(st == 1, s_w, &t1);
            const int p2 = block_excl(st == 2, s_w, &t2);
            const int p3 = block_excl(st == 3, s_w, &t3);
            if (st == 1) a.cut[total + o1 + p1] = v;
            if (st == 2) a.cut[total + n1 + o2 + p2] = v;
            if (st == 3) {
                const int fc = a.nodes[6 * v + 3];
                next[o3 + p3] = fc;
                next[n3 + o3 + p3] = a.nodes[6 * fc + 4];
            }
            o1 += t1; o2 += t2; o3 += t3;
        }
        total += n1 + n2;
        size = 2 * n3;
        int* t = front; front = next; next = t;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        a.count[0] = total;
        a.count[1] = overflow ? 1 : 0;
    }
}

void launch_upper_cut(const CutArgs& a, hipStream_t s)
{
    hipLaunchKernelGGL(k_upper_cut, dim3(1), dim3(1024), 0, s, a);
}

// ---------------------------------------------------------------- row gather / scatter
// 16 lanes per row (four rows per wave); each lane moves 16-byte words when the row size and both bases allow,
// 4-byte words otherwise.
template <typename W>
__global__ void __launch_bounds__(256) k_rows_gather(long n, int words, const int64_t* __restrict__ idx,
                                                     const W* __restrict__ src, W* __restrict__ dst)
{
    const long r = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
    if (r >= n) return;
    const int l = threadIdx.x & 15;
    const W* s = src + idx[r] * words;
    W* d = dst + r * words;
    for (int k = l; k < words; k += 16) d[k] = s[k];
}

template <typename W>
__global__ void __launch_bounds__(256) k_rows_scatter(long n, int words, const int64_t* __restrict__ idx,
                                                      const W* __restrict__ src, W* __restrict__ dst)
{
    const long r = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
    if (r >= n) return;
    const int l = threadIdx.x & 15;
    const W* s = src + r * words;
    W* d = dst + idx[r] * words;
    for (int k = l; k < words; k += 16) d[k] = s[k];
}

void launch_rows(bool gather, long n, int row_bytes, const int64_t* idx, const void* src, void* dst, hipStream_t s)
{
    const dim3 grid((unsigned)((n + 15) / 16));
    const bool wide = row_bytes % 16 == 0 && (((uintptr_t)src | (uintptr_t)dst) & 15u) == 0;
    if (wide) {
        if (gather)
            hipLaunchKernelGGL(k_rows_gather<float4>, grid, dim3(256), 0, s, n, row_bytes / 16, idx,
                               (const float4*)src, (float4*)dst);
        else
            hipLaunchKernelGGL(k_rows_scatter<float4>, grid, dim3(256), 0, s, n, row_bytes / 16, idx,
                               (const float4*)src, (float4*)dst);
    } else {
        if (gather)
            hipLaunchKernelGGL(k_rows_gather<uint32_t>, grid, dim3(256), 0, s, n, row_bytes / 4, idx,
                               (const uint32_t*)src, (uint32_t*)dst);
        else
            hipLaunchKernelGGL(k_rows_scatter<uint32_t>, grid, dim3(256), 0, s, n, row_bytes / 4, idx,
                               (const uint32_t*)src, (uint32_t*)dst);
    }
}

}  // namespace hlgs
