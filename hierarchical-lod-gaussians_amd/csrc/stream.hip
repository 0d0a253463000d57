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
//   k_rows_multi    <- the same traffic for all of a step's tensors (parameters and Adam moments) in one launch
//   k_rows_packed   <- the host legs of that traffic when the host storage is one packed row per Gaussian (all
//                      six parameters and twelve Adam moments back to back, padded to whole 64-byte lines): every
//                      wave moves whole host lines instead of one 12-180-byte fragment per tensor
//   k_cache_lists / k_cache_keep / k_cache_split
//                   <- the SPT cache's bookkeeping (train_post.py:346-430): which of the previous view's SPTs
//                      are reused, which are loaded, the new SPT_counts prefix, and which cached Gaussians stay
//                      resident or are written back.  The reference does this with per-SPT Python loops and a
//                      host read per kept SPT; here it is one single-workgroup pass over the SPT lists plus two
//                      scans over the resident Gaussians, with one host read for all the sizes.
#include <algorithm>

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

// Pass 1 classifies the level once (the states go to LDS when the level fits, so pass 2 does not reload the nodes)
// and counts with wave ballots and LDS atomics, without block barriers, so the waves' node loads overlap.
constexpr int kCutLds = 48 * 1024;

__global__ void __launch_bounds__(1024) k_upper_cut(CutArgs a)
{
    __shared__ int s_w[16];
    __shared__ int s_n[3];
    __shared__ uint8_t s_st[kCutLds];
    int* front = a.front_a;
    int* next = a.front_b;
    int size = a.N > 0 ? 1 : 0;
    if (threadIdx.x == 0) front[0] = 0;  // root_node = 0
    int total = 0;
    bool overflow = false;
    const int lane = threadIdx.x & 63;
    __syncthreads();
    while (size > 0 && !overflow) {
        // pass 1: classify, level totals of the three outcomes
        if (threadIdx.x < 3) s_n[threadIdx.x] = 0;
        __syncthreads();
        const bool cached = size <= kCutLds;
        for (int c0 = 0; c0 < size; c0 += 1024) {
            const int i = c0 + threadIdx.x;
            const int st = i < size ? cut_state(a, front[i]) : 0;
            if (cached && i < size) s_st[i] = (uint8_t)st;
            const uint64_t b1 = __ballot(st == 1), b2 = __ballot(st == 2), b3 = __ballot(st == 3);
            if (lane == 0) {
                if (b1) atomicAdd(&s_n[0], __popcll(b1));
                if (b2) atomicAdd(&s_n[1], __popcll(b2));
                if (b3) atomicAdd(&s_n[2], __popcll(b3));
            }
        }
        __syncthreads();
        const int n1 = s_n[0], n2 = s_n[1], n3 = s_n[2];
        if (total + n1 + n2 > a.capacity || 2 * n3 > a.capacity) { overflow = true; break; }
        // pass 2: write the cut and the next frontier in the reference's order
        int o1 = 0, o2 = 0, o3 = 0;
        for (int c0 = 0; c0 < size; c0 += 1024) {
            const int i = c0 + threadIdx.x;
            const int v = i < size ? front[i] : 0;
            const int st = i < size ? (cached ? (int)s_st[i] : cut_state(a, v)) : 0;
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

// ---------------------------------------------------------------- multi-tensor row copy
// dst_t[dst_rows[i]] = src_t[src_rows[i]] for every table t (blockIdx.y); a NULL row list is the identity.  One
// lane per 4-byte word, words numbered row after row, so every wave touches one contiguous span of the identity
// side with all lanes busy; a lane's (row, word) advances by the grid stride without dividing in the loop.
struct RowTabs {
    RowCopy t[kMaxRowTables];
};

typedef uint4 __attribute__((aligned(4))) uint4_a4;  // 16-byte access at 4-byte alignment (global_load_dwordx4)

__global__ void __launch_bounds__(256) k_rows_multi(RowTabs tabs, int64_t n, const int* __restrict__ src_rows,
                                                    const int* __restrict__ dst_rows)
{
    const RowCopy& tb = tabs.t[blockIdx.y];
    const int64_t words = tb.row_bytes >> 2;
    if (words == 0) return;
    const uint32_t* __restrict__ src = static_cast<const uint32_t*>(tb.src);
    uint32_t* __restrict__ dst = static_cast<uint32_t*>(tb.dst);
    // lanes own U consecutive words (U = 4 for device-only tables, whose interior row chunks move as one 16-byte
    // access; 1 otherwise, since a 16-byte access to host memory may straddle a page)
#ifndef HLGS_ROWS_WIDE
#define HLGS_ROWS_WIDE 1  // 0: 4-byte lanes everywhere; 1: 16-byte lanes for device-only tables; 2: only if rows are whole 16-byte chunks
#endif
    const int U = (HLGS_ROWS_WIDE == 1 && tb.device_only) || (HLGS_ROWS_WIDE == 2 && tb.device_only && (words & 3) == 0) ? 4 : 1;
    const int64_t w0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * U, S = (int64_t)gridDim.x * 256 * U;
    int64_t r = w0 / words, k = w0 - r * words;
    const int64_t dr = S / words, dk = S - dr * words;
    while (r < n) {
        int64_t rr = r, kk = k;
        if (U == 4 && k + 4 <= words) {
            const int64_t sr = src_rows ? src_rows[r] : r;
            const int64_t drow = dst_rows ? dst_rows[r] : r;
            *reinterpret_cast<uint4_a4*>(dst + drow * words + k) = *reinterpret_cast<const uint4_a4*>(src + sr * words + k);
        } else {
            for (int u = 0; u < U && rr < n; u++) {
                const int64_t sr = src_rows ? src_rows[rr] : rr;
                const int64_t drow = dst_rows ? dst_rows[rr] : rr;
                dst[drow * words + kk] = src[sr * words + kk];
                if (++kk == words) {
                    kk = 0;
                    rr++;
                }
            }
        }
        r += dr;
        k += dk;
        while (k >= words) {
            k -= words;
            r++;
        }
    }
}

// ---------------------------------------------------------------- packed host rows
// Host row h = words [h * hw, (h + 1) * hw) of `host`: table 0's row, table 1's row, ..., then zero padding to hw
// (a multiple of 16 words, so a row is whole 64-byte lines).  One wave per row at a time; lane l owns host words
// l, l + 64, l + 128, l + 192 of every row, so each store (to host) or load (from host) instruction of the wave
// covers 256 contiguous bytes of the host row, and the device side of the same instruction is one contiguous run
// per table row.  A lane's (table, word) for each of its slots is found once, before the row loop.
struct PackTabs {
    float* t[kMaxRowTables];
    int words[kMaxRowTables];
};

template <bool TO_HOST>
__global__ void __launch_bounds__(256) k_rows_packed(PackTabs tabs, int T, int64_t n, const int* __restrict__ dev_rows,
                                                     const int* __restrict__ host_rows, float* __restrict__ host,
                                                     int hw)
{
    const int lane = threadIdx.x & 63;
    float* base[kPackSlots];
    int width[kPackSlots], off[kPackSlots];
    bool live[kPackSlots];
#pragma unroll
    for (int m = 0; m < kPackSlots; m++) {
        const int w = lane + 64 * m;
        int start = 0, t = 0;
        while (t < T && w >= start + tabs.words[t]) start += tabs.words[t++];
        live[m] = t < T;  // a data word (else padding, or beyond the row when m * 64 >= hw)
        base[m] = live[m] ? tabs.t[t] : nullptr;
        width[m] = live[m] ? tabs.words[t] : 0;
        off[m] = w - start;
    }
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t r = wave; r < n; r += nwaves) {
        const int64_t dr = dev_rows ? dev_rows[r] : r;
        const int64_t hr = host_rows ? host_rows[r] : r;
        float* hrow = host + hr * hw;
        if (TO_HOST) {
            float v[kPackSlots];
#pragma unroll
            for (int m = 0; m < kPackSlots; m++) v[m] = live[m] ? base[m][dr * width[m] + off[m]] : 0.f;
#pragma unroll
            for (int m = 0; m < kPackSlots; m++)
                if (lane + 64 * m < hw) hrow[lane + 64 * m] = v[m];  // padding words too: whole lines
        } else {
            float v[kPackSlots];
#pragma unroll
            for (int m = 0; m < kPackSlots; m++) v[m] = live[m] ? hrow[lane + 64 * m] : 0.f;
#pragma unroll
            for (int m = 0; m < kPackSlots; m++)
                if (live[m]) base[m][dr * width[m] + off[m]] = v[m];
        }
    }
}

void launch_rows_packed(int T, float* const* tabs, const int* words, int64_t n, const int* dev_rows,
                        const int* host_rows, float* host, int hw, bool to_host, hipStream_t s)
{
    PackTabs pt{};
    for (int t = 0; t < T; t++) {
        pt.t[t] = tabs[t];
        pt.words[t] = words[t];
    }
    const int64_t blocks = std::min<int64_t>((n + 3) / 4, 2048);  // 4 waves (rows) per block, grid-stride above
    if (blocks <= 0) return;
    if (to_host) hipLaunchKernelGGL(k_rows_packed<true>, dim3((unsigned)blocks), dim3(256), 0, s, pt, T, n, dev_rows, host_rows, host, hw);
    else hipLaunchKernelGGL(k_rows_packed<false>, dim3((unsigned)blocks), dim3(256), 0, s, pt, T, n, dev_rows, host_rows, host, hw);
}

void launch_rows_multi(int T, const RowCopy* tabs, int64_t n, const int* src_rows, const int* dst_rows, hipStream_t s)
{
    RowTabs rt{};
    int64_t most = 0;
    for (int t = 0; t < T; t++) {
        rt.t[t] = tabs[t];
        most = std::max<int64_t>(most, (n * (tabs[t].row_bytes >> 2) + 3) / (tabs[t].device_only ? 4 : 1));
    }
    const int64_t blocks = std::min<int64_t>((most + 255) / 256, 4096);
    if (blocks > 0) hipLaunchKernelGGL(k_rows_multi, dim3((unsigned)blocks, T), dim3(256), 0, s, rt, n, src_rows, dst_rows);
}

// ---------------------------------------------------------------- SPT cache bookkeeping
// exclusive prefix of an int over the 1024-thread block
__device__ __forceinline__ int block_excl_sum(int v, int* s_w, int* total)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    __syncthreads();
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    int before = 0, t = 0;
    for (int i = 0; i < 16; i++) {
        const int c = s_w[i];
        if (i < w) before += c;
        t += c;
    }
    *total = t;
    return before + x - v;
}

// a Python slice bound against a sequence of length R (step 1)
__device__ __forceinline__ int py_bound(int x, int R)
{
    if (x < 0) {
        x += R;
        return x < 0 ? 0 : x;
    }
    return x > R ? R : x;
}

// torch.isclose on float32 (allowed = atol + |rtol * b|; finite |a - b| <= allowed, or a == b)
__device__ __forceinline__ bool is_close(float a, float b, float rtol, float atol)
{
#pragma clang fp contract(off)
    if (a == b) return true;
    const float err = fabsf(a - b);
    const float allowed = atol + fabsf(rtol * b);
    return isfinite(err) && err <= allowed;
}

__global__ void __launch_bounds__(1024) k_cache_lists(CacheArgs a)
{
#pragma clang fp contract(off)
    __shared__ int s_w[16];
    // 1. leaves of the cut, in cut order: SPT leaves (first_child >= 0, with their camera distance) and
    //    upper-tree Gaussians to render (first_child <= 0; a leaf holding SPT 0 is in both lists, as in the
    //    reference's two masks)
    int ns = 0, nu = 0;
    for (int c0 = 0; c0 < a.n_cut; c0 += 1024) {
        const int i = c0 + threadIdx.x;
        int v = 0, fc = -1;
        bool leaf = false;
        if (i < a.n_cut) {
            v = a.cut[i];
            leaf = a.nodes[6 * v + 2] == 0;
            fc = a.nodes[6 * v + 3];
        }
        const bool is_s = leaf && fc >= 0, is_u = leaf && fc <= 0;
        int ts, tu;
        const int ps = block_excl(is_s, s_w, &ts);
        const int pu = block_excl(is_u, s_w, &tu);
        if (is_s) {
            const float dx = a.xyz[3 * v] - a.campos[0], dy = a.xyz[3 * v + 1] - a.campos[1],
                        dz = a.xyz[3 * v + 2] - a.campos[2];
            a.spt_idx[ns + ps] = fc;
            a.spt_dist[ns + ps] = sqrtf(dx * dx + dy * dy + dz * dz) * a.dmul;
        }
        if (is_u) a.upper[nu + pu] = a.nodes[6 * v + 5];
        ns += ts;
        nu += tu;
    }
    __syncthreads();
    // 2. previous SPTs: torch.searchsorted (lower bound; the list is in cut order, not sorted, and the search
    //    runs on it as it is), equal id and isclose distance -> kept, with the reference's segment bounds
    int nk = 0, prefix = 0;
    for (int c0 = 0; c0 < a.m; c0 += 1024) {
        const int j = c0 + threadIdx.x;
        bool keep = false;
        int pv = 0, d = 0, start = 0, to = 0;
        if (j < a.m) {
            pv = a.prev_idx[j];
            int lo = 0, hi = ns;
            while (lo < hi) {
                const int mid = lo + ((hi - lo) >> 1);
                if (!(a.spt_idx[mid] >= pv)) lo = mid + 1;
                else hi = mid;
            }
            keep = lo < ns && a.spt_idx[lo] == pv && is_close(a.spt_dist[lo], a.prev_dist[j], a.rtol, a.atol);
            if (keep) {
                start = a.prev_counts[j];
                to = j == a.m - 1 ? a.tail_end : a.prev_counts[j + 1];
                d = to - start;
            }
        }
        int tk, td;
        const int pk = block_excl(keep, s_w, &tk);
        const int pd = block_excl_sum(d, s_w, &td);
        if (keep) {
            a.keep_idx[nk + pk] = pv;
            a.keep_dist[nk + pk] = a.prev_dist[j];
            a.keep_counts[nk + pk] = prefix + pd;
            if (pv >= 0 && pv < a.num_spts) a.flag[pv] = 1;
            const int lo = py_bound(start, a.R), hi = py_bound(to, a.R);
            if (hi > lo) {
                atomicAdd(a.diff + lo, 1);
                atomicAdd(a.diff + hi, -1);
            }
        }
        nk += tk;
        prefix += td;
    }
    __syncthreads();
    // 3. the cut's SPTs whose id was not kept (torch.isin) are loaded, in cut order
    int nl = 0;
    for (int c0 = 0; c0 < ns; c0 += 1024) {
        const int k = c0 + threadIdx.x;
        bool load = false;
        int v = 0;
        if (k < ns) {
            v = a.spt_idx[k];
            load = !(v >= 0 && v < a.num_spts && a.flag[v]);
        }
        int tl;
        const int pl = block_excl(load, s_w, &tl);
        if (load) {
            a.load_idx[nl + pl] = v;
            a.load_dist[nl + pl] = a.spt_dist[k];
        }
        nl += tl;
    }
    if (threadIdx.x == 0) {
        a.sizes[0] = nk;
        a.sizes[1] = nl;
        a.sizes[2] = nu;
        a.sizes[3] = prefix;
    }
}

void launch_cache_lists(const CacheArgs& a, hipStream_t s)
{
    hipLaunchKernelGGL(k_cache_lists, dim3(1), dim3(1024), 0, s, a);
}

// keep_gaussians_mask: the skybox prefix, or covered by a kept SPT's segment (running sum of the +1/-1 marks)
__global__ void __launch_bounds__(256) k_cache_keep(int R, int sky, const uint32_t* __restrict__ diff_incl,
                                                    uint32_t* __restrict__ keep)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < R) keep[i] = (i < sky || (int)diff_incl[i] > 0) ? 1u : 0u;
}

void launch_cache_keep(int R, int sky, const uint32_t* diff_incl, uint32_t* keep, hipStream_t s)
{
    hipLaunchKernelGGL(k_cache_keep, dim3((R + 255) / 256), dim3(256), 0, s, R, sky, diff_incl, keep);
}

// render_indices[keep] / nonzero(keep) and render_indices[~keep] / nonzero(~keep), both in order
__global__ void __launch_bounds__(256) k_cache_split(int R, const int* __restrict__ render,
                                                     const uint32_t* __restrict__ keep_incl, int* __restrict__ keep_rows,
                                                     int* __restrict__ render_kept, int* __restrict__ wb_rows,
                                                     int* __restrict__ wb_indices)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= R) return;
    const int incl = (int)keep_incl[i];
    const int prev = i ? (int)keep_incl[i - 1] : 0;
    if (incl != prev) {
        keep_rows[incl - 1] = i;
        render_kept[incl - 1] = render[i];
    } else {
        const int w = i - incl;
        wb_rows[w] = i;
        wb_indices[w] = render[i];
    }
}

void launch_cache_split(int R, const int* render, const uint32_t* keep_incl, int* keep_rows, int* render_kept,
                        int* wb_rows, int* wb_indices, hipStream_t s)
{
    hipLaunchKernelGGL(k_cache_split, dim3((R + 255) / 256), dim3(256), 0, s, R, render, keep_incl, keep_rows,
                       render_kept, wb_rows, wb_indices);
}

}  // namespace hlgs
