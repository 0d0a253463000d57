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
// A node's cut state (0 culled, 1 leaf -> cut, 2 condition false -> cut, 3 expand), with its first child and that
// child's next sibling when it expands.  Every load that depends only on v is issued before any test, so a level
// costs two dependent global round trips (v's row, then the first child's sibling).
struct CutNode {
    int st, fc, ns;
};
template <bool SIB = true>
__device__ __forceinline__ CutNode cut_node(const CutArgs& a, int v)
{
#pragma clang fp contract(off)
    const float px = a.xyz[3 * v], py = a.xyz[3 * v + 1], pz = a.xyz[3 * v + 2];
    const float r = a.use_frustum ? a.bounds[v] : 0.f;
    const int kids = a.nodes[6 * v + 2], fc = a.nodes[6 * v + 3];
    const float md = a.use_lod ? a.min_dist2[v] : 0.f;
    CutNode c{3, 0, 0};
    if (a.use_frustum) {  // culled unless the sphere reaches into some view's frustum
        bool any = false;
        for (int g = 0; g < a.nviews; g++) {
            bool in = true;
            for (int k = 0; k < 4; k++) {
                const float* pl = a.planes + 16 * g + 4 * k;
                const float sd = px * pl[0] + py * pl[1] + pz * pl[2] + pl[3];  // torch.sum over 3, then + distance
                if (sd + r < 0.f) in = false;
            }
            any = any || in;
        }
        if (!any) c.st = 0;
    }
    if (c.st == 3 && kids == 0) c.st = 1;
    if (c.st == 3 && a.use_lod) {  // the nearest camera decides (min over views of the squared distance)
        float d2 = INFINITY;
        for (int g = 0; g < a.nviews; g++) {
            const float dx = a.campos[3 * g] - px, dy = a.campos[3 * g + 1] - py, dz = a.campos[3 * g + 2] - pz;
            d2 = fminf(d2, dx * dx + dy * dy + dz * dz);
        }
        if (!(md > d2 * a.dmul)) c.st = 2;
    }
    if (SIB && c.st == 3) {
        c.fc = fc;
        c.ns = a.nodes[6 * fc + 4];
    }
    return c;
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

// Narrow levels (the top of the tree) are walked by one workgroup, k_upper_cut: thread t owns a contiguous run of
// ceil(size / 1024) frontier entries, visited in batches of eight whose loads are all issued together.  Pass 1
// counts the three outcomes per thread, one three-way block scan turns the counts into output offsets, and pass 2
// re-classifies the same entries and writes the cut (leaves, then condition-false nodes) and the next frontier
// (first children, then their siblings) in frontier order.  A level costs ~3 us that way, but one CU streams only
// ~160 nodes per us, and the last levels of a 1M-leaf upper tree hold 4k-22k nodes.  So once a level exceeds
// kCutNarrow entries the workgroup hands off (CutState), and each following level runs as one launch of
// k_cut_level over many workgroups: the same two passes, with the per-workgroup outcome counts combined through
// an arrival counter (every workgroup of a level is resident: a level uses at most kCutMaxBlocks = 64).  A fixed number
// of such launches is queued; a final k_upper_cut in resume mode finishes any deeper levels and writes the count.
constexpr int kCutBatch = 8;
constexpr int kCutNarrow = 1024;

// exclusive prefix of (x, y, z) over the 1024-thread block, and the block totals
__device__ __forceinline__ int3 block_excl3(int3 v, int* s_w, int3* tot)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int3 inc = v;
    for (int d = 1; d < 64; d <<= 1) {
        const int x = __shfl_up(inc.x, d, 64), y = __shfl_up(inc.y, d, 64), z = __shfl_up(inc.z, d, 64);
        if (lane >= d) { inc.x += x; inc.y += y; inc.z += z; }
    }
    __syncthreads();  // s_w is free
    if (lane == 63) { s_w[3 * w] = inc.x; s_w[3 * w + 1] = inc.y; s_w[3 * w + 2] = inc.z; }
    __syncthreads();
    int3 before = make_int3(0, 0, 0), t = make_int3(0, 0, 0);
    for (int k = 0; k < 16; k++) {
        const int cx = s_w[3 * k], cy = s_w[3 * k + 1], cz = s_w[3 * k + 2];
        if (k < w) { before.x += cx; before.y += cy; before.z += cz; }
        t.x += cx; t.y += cy; t.z += cz;
    }
    *tot = t;
    return make_int3(before.x + inc.x - v.x, before.y + inc.y - v.y, before.z + inc.z - v.z);
}

// Outcome counts of frontier entries [i0, i1)
__device__ __forceinline__ int3 cut_count(const CutArgs& a, const int* front, int i0, int i1)
{
    int3 n = make_int3(0, 0, 0);
    for (int b = i0; b < i1; b += kCutBatch) {
        int v[kCutBatch];
#pragma unroll
        for (int j = 0; j < kCutBatch; j++) v[j] = b + j < i1 ? front[b + j] : -1;
#pragma unroll
        for (int j = 0; j < kCutBatch; j++) {
            if (v[j] < 0) continue;
            const int st = cut_node<false>(a, v[j]).st;
            n.x += st == 1;
            n.y += st == 2;
            n.z += st == 3;
        }
    }
    return n;
}

// Writes of frontier entries [i0, i1): leaves at cut[o1...], condition-false nodes at cut[o2...], first children at
// next[o3...] and their siblings at next[n3 + o3...]
__device__ __forceinline__ void cut_write(const CutArgs& a, const int* front, int* next, int i0, int i1, int o1,
                                          int o2, int o3, int n3)
{
    for (int b = i0; b < i1; b += kCutBatch) {
        int v[kCutBatch];
#pragma unroll
        for (int j = 0; j < kCutBatch; j++) v[j] = b + j < i1 ? front[b + j] : -1;
#pragma unroll
        for (int j = 0; j < kCutBatch; j++) {
            if (v[j] < 0) continue;
            const CutNode c = cut_node(a, v[j]);
            if (c.st == 1) a.cut[o1++] = v[j];
            else if (c.st == 2) a.cut[o2++] = v[j];
            else if (c.st == 3) {
                next[o3] = c.fc;
                next[n3 + o3] = c.ns;
                o3++;
            }
        }
    }
}

// A thread's run of at most kCutRun frontier entries, classified once (with the expanding nodes' siblings): pass 1
// counts from it and pass 2 writes from it, so pass 2 makes no global round trip (it re-read the entries, their rows
// and the siblings: three of a level's five dependent round trips).
constexpr int kCutRun = 2;  // entries per thread of a cached run (a level of up to 2,048 entries per workgroup)
struct CutRun {
    int v[kCutRun];
    CutNode c[kCutRun];
};
__device__ __forceinline__ int3 cut_eval(const CutArgs& a, const int* front, int i0, int i1, CutRun& run)
{
    int3 n = make_int3(0, 0, 0);
#pragma unroll
    for (int j = 0; j < kCutRun; j++) run.v[j] = i0 + j < i1 ? front[i0 + j] : -1;
#pragma unroll
    for (int j = 0; j < kCutRun; j++) {
        run.c[j] = CutNode{0, 0, 0};
        if (run.v[j] < 0) continue;
        run.c[j] = cut_node(a, run.v[j]);
        n.x += run.c[j].st == 1;
        n.y += run.c[j].st == 2;
        n.z += run.c[j].st == 3;
    }
    return n;
}
__device__ __forceinline__ void cut_write_run(const CutArgs& a, const CutRun& run, int* next, int o1, int o2, int o3,
                                              int n3)
{
#pragma unroll
    for (int j = 0; j < kCutRun; j++) {
        if (run.v[j] < 0) continue;
        const CutNode& c = run.c[j];
        if (c.st == 1) a.cut[o1++] = run.v[j];
        else if (c.st == 2) a.cut[o2++] = run.v[j];
        else if (c.st == 3) {
            next[o3] = c.fc;
            next[n3 + o3] = c.ns;
            o3++;
        }
    }
}

// resume = 0: start at the root and hand off at the first level wider than kCutNarrow;  resume = 1: continue from
// the state the level launches left, to the end, and write the count.
__global__ void __launch_bounds__(1024) k_upper_cut(CutArgs a, int resume)
{
    __shared__ int s_w[16 * 3];
    CutState* cs = a.state;
    int size, total, parity, overflow;
    if (!resume) {
        size = a.N > 0 ? 1 : 0;
        total = 0;
        parity = 0;
        overflow = 0;
        if (threadIdx.x == 0) a.front_a[0] = 0;  // root_node = 0
        if (threadIdx.x < kCutLevelLaunches) a.arrive[threadIdx.x] = 0;
    } else {
        size = cs->size;
        total = cs->total;
        parity = cs->parity;
        overflow = cs->overflow;
    }
    __syncthreads();
    while (size > 0 && !overflow) {
        if (!resume && size > kCutNarrow) break;  // hand off to k_cut_level
        const int* front = parity ? a.front_b : a.front_a;
        int* next = parity ? a.front_a : a.front_b;
        const int K = (size + 1023) / 1024;
        const int i0 = min(size, (int)threadIdx.x * K), i1 = min(size, i0 + K);
        int3 tot;
        if (K <= kCutRun) {  // (uniform) one classification for both passes
            CutRun run;
            const int3 o = block_excl3(cut_eval(a, front, i0, i1, run), s_w, &tot);
            if (total + tot.x + tot.y > a.capacity || 2 * tot.z > a.capacity) { overflow = 1; break; }
            cut_write_run(a, run, next, total + o.x, total + tot.x + o.y, o.z, tot.z);
        } else {
            const int3 o = block_excl3(cut_count(a, front, i0, i1), s_w, &tot);
            if (total + tot.x + tot.y > a.capacity || 2 * tot.z > a.capacity) { overflow = 1; break; }
            cut_write(a, front, next, i0, i1, total + o.x, total + tot.x + o.y, o.z, tot.z);
        }
        total += tot.x + tot.y;
        size = 2 * tot.z;
        parity ^= 1;
        __syncthreads();  // the next frontier is visible to the whole workgroup
    }
    if (threadIdx.x == 0) {
        cs->size = overflow ? 0 : size;
        cs->total = total;
        cs->parity = parity;
        cs->overflow = overflow;
        if (resume || size == 0 || overflow) {
            a.count[0] = total;
            a.count[1] = overflow;
        }
    }
}

// One wide level over many workgroups (launch number `launch` of kCutLevelLaunches).  Workgroup b owns the contiguous
// entries [b E, (b + 1) E) with E = 1024 * ceil(size / (1024 * kCutMaxBlocks)); the workgroups of the level publish
// their outcome counts, then wait until all of them have (they are all resident), so each can form its offsets.
__global__ void __launch_bounds__(1024) k_cut_level(CutArgs a, int launch)
{
    __shared__ int s_w[16 * 3];
    __shared__ int3 s_pre, s_tot;
    CutState* cs = a.state;
    const int size = cs->size;
    if (size == 0 || cs->overflow) return;
    const int per = 1024 * ((size + 1024 * kCutMaxBlocks - 1) / (1024 * kCutMaxBlocks));
    const int nb = (size + per - 1) / per;
    const int b = blockIdx.x;
    if (b >= nb) return;
    const int total = cs->total, parity = cs->parity;
    const int* front = parity ? a.front_b : a.front_a;
    int* next = parity ? a.front_a : a.front_b;
    const int K = per / 1024;
    const int e0 = b * per, e1 = min(size, e0 + per);
    const int i0 = min(e1, e0 + (int)threadIdx.x * K), i1 = min(e1, i0 + K);
    int3 bt, o;
    CutRun run;
    const bool cached = K <= kCutRun;  // uniform: one classification for both passes
    if (cached) o = block_excl3(cut_eval(a, front, i0, i1, run), s_w, &bt);
    else o = block_excl3(cut_count(a, front, i0, i1), s_w, &bt);
    if (threadIdx.x == 0) {
        int* pb = a.level_counts + 3 * b;
        __hip_atomic_store(pb, bt.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pb + 1, bt.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pb + 2, bt.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(a.arrive + launch, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        while (__hip_atomic_load(a.arrive + launch, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)nb)
            __builtin_amdgcn_s_sleep(2);
    }
    __syncthreads();
    // workgroup prefix and level totals over the published counts (thread t < nb holds workgroup t's)
    int3 mine = make_int3(0, 0, 0);
    if ((int)threadIdx.x < nb) {
        const int* pt = a.level_counts + 3 * threadIdx.x;
        mine = make_int3(__hip_atomic_load(pt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                         __hip_atomic_load(pt + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                         __hip_atomic_load(pt + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    int3 tot;
    const int3 pre = block_excl3(mine, s_w, &tot);
    if ((int)threadIdx.x == b) s_pre = pre;
    __syncthreads();
    const int3 bp = s_pre;
    if (total + tot.x + tot.y > a.capacity || 2 * tot.z > a.capacity) {
        if (b == 0 && threadIdx.x == 0) cs->overflow = 1;
        return;
    }
    if (cached) cut_write_run(a, run, next, total + bp.x + o.x, total + tot.x + bp.y + o.y, bp.z + o.z, tot.z);
    else cut_write(a, front, next, i0, i1, total + bp.x + o.x, total + tot.x + bp.y + o.y, bp.z + o.z, tot.z);
    if (b == 0 && threadIdx.x == 0) {  // every workgroup read the state before it arrived
        cs->size = 2 * tot.z;
        cs->total = total + tot.x + tot.y;
        cs->parity = parity ^ 1;
    }
}

void launch_upper_cut(const CutArgs& a, hipStream_t s)
{
    hipLaunchKernelGGL(k_upper_cut, dim3(1), dim3(1024), 0, s, a, 0);
    const int blocks = std::min(kCutMaxBlocks, (2 * a.N + 2 + 1023) / 1024);
    for (int l = 0; l < kCutLevelLaunches; l++) hipLaunchKernelGGL(k_cut_level, dim3(blocks), dim3(1024), 0, s, a, l);
    hipLaunchKernelGGL(k_upper_cut, dim3(1), dim3(1024), 0, s, a, 1);
}
// ---------------------------------------------------------------- flat coarse cut (round 5)
// The same cut from the walk order hlgs_upper_tree_order precomputes (see there for why the order is static): the
// level walk above costs a dependent chain per level (~3 us a narrow level, ~13 us a wide one, 180 us for the 21
// levels of config #5's upper tree); here every node's state is one parallel pass and a single workgroup places the
// survivors.
//   k_cut_flat_eval:  per F* entry i: its state (cut_node) and, in preorder, the end of its subtree interval if it
//                     does not expand (culled, leaf, condition false), else 0.
//   k_cut_flat_place: covered(p) = (max of those ends over preorder positions < p) > p -- a max scan over preorder
//                     into an LDS bit mask; then per F* entry alive = !covered(its position); the leaves and
//                     condition-false nodes that are alive are counted per thread run and scanned (one workgroup);
//   k_cut_flat_write: places them, one thread per entry: a leaf at (stops before its level) + (leaves before it), a
//                     condition-false node at (leaves up to the end of its level) + (stops before it).
constexpr int kFlatRun = 64;  // entries per thread of k_cut_flat_place (1024 x 64 > HLGS_CUT_FLAT_MAX_ENTRIES)
static_assert(1024 * kFlatRun > HLGS_CUT_FLAT_MAX_ENTRIES, "one 64-bit mask per thread run");

// A blob the flat cut can use for these nodes: usable (word 2), built for this node count (word 3; a blob of another
// tree would read nodes past N and leave holes in the cut), entries and levels within the kernels' limits.  The same
// test in all three kernels (uniform); k_cut_flat_place reports a failure through count[1].
__device__ __forceinline__ bool flat_blob_ok(const CutArgs& a, const int* order)
{
    const int M = order[0], nlev = order[1];
    return order[2] == 1 && order[3] == a.N && M > 0 && M <= a.N && M <= HLGS_CUT_FLAT_MAX_ENTRIES && nlev >= 1 &&
           nlev <= HLGS_CUT_FLAT_MAX_LEVELS;
}

__global__ void __launch_bounds__(256) k_cut_flat_eval(CutArgs a, const int* __restrict__ order,
                                                       uint8_t* __restrict__ st8, uint16_t* __restrict__ endv)
{
    const int M = order[0];
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (!flat_blob_ok(a, order) || i >= M) return;  // an unusable blob: k_cut_flat_place reports it
    const int* fn = order + HLGS_CUT_ORDER_HEADER;
    const int v = fn[i], pe = fn[M + i];
    const int st = cut_node<false>(a, v).st;
    st8[i] = (uint8_t)st;
    endv[pe & 0xffff] = (uint16_t)(st == 3 ? 0 : (unsigned)pe >> 16);
}

// exclusive max over the 1024-thread block (values >= 0)
__device__ __forceinline__ int block_excl_max(int v, int* s_w)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int inc = v;
    for (int d = 1; d < 64; d <<= 1) {
        const int x = __shfl_up(inc, d, 64);
        if (lane >= d) inc = max(inc, x);
    }
    int ex = __shfl_up(inc, 1, 64);
    if (lane == 0) ex = 0;
    __syncthreads();
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    for (int k = 0; k < w; k++) ex = max(ex, s_w[k]);
    return ex;
}

// A thread's run of 64 16-bit (or 8-bit) entries from p0 as 32-bit words, in 16-byte loads.  Entries at or beyond M
// are read (the scratch regions and the order blob leave room for a whole run past M) but never used.
template <int BYTES, int W>
__device__ __forceinline__ void load_run(const void* base, int p0, uint32_t (&wd)[W])
{
    const uint4* q = reinterpret_cast<const uint4*>(static_cast<const char*>(base) + (size_t)p0 * BYTES);
#pragma unroll
    for (int u = 0; u < W / 4; u++) {
        const uint4 x = q[u];
        wd[4 * u] = x.x; wd[4 * u + 1] = x.y; wd[4 * u + 2] = x.z; wd[4 * u + 3] = x.w;
    }
}
template <int BYTES>
__device__ __forceinline__ uint32_t run_at(const uint32_t (&wd)[kFlatRun * BYTES / 4], int k)
{
    constexpr int kPer = 4 / BYTES;
    return (wd[k / kPer] >> (8 * BYTES * (k % kPer))) & (BYTES == 2 ? 0xffffu : 0xffu);
}
static_assert(HLGS_CUT_ORDER_HEADER % 4 == 0, "16-byte aligned runs in the order blob");

__global__ void __launch_bounds__(1024) k_cut_flat_place(CutArgs a, const int* __restrict__ order,
                                                         const uint8_t* __restrict__ st8,
                                                         const uint16_t* __restrict__ endv)
{
    __shared__ uint32_t s_bits[1024 * kFlatRun / 32];
    __shared__ int s_w[16 * 3];
    __shared__ int s_ls[HLGS_CUT_FLAT_MAX_LEVELS + 1];
    __shared__ int2 s_lev[HLGS_CUT_FLAT_MAX_LEVELS + 1];
    const int M = order[0], nlev = order[1];
    const int t = threadIdx.x;
    if (!flat_blob_ok(a, order)) {
        if (t == 0) { a.count[0] = 0; a.count[1] = 1; }  // (uniform) not a blob the flat cut can use
        return;
    }
    if (t <= nlev) s_ls[t] = order[4 + t];
    // thread t owns entries [t R, t R + R) of both orders (preorder here, F* below); R = 32 or 64
    const int R = ((M + 1023) / 1024 + 31) & ~31;
    const int p0 = t * R;
    {  // covered bits over preorder positions
        uint32_t e[kFlatRun / 2];
        load_run<2>(endv, min(p0, M & ~31), e);
        const int n = max(0, min(R, M - p0));
        int mx = 0;
#pragma unroll
        for (int k = 0; k < kFlatRun; k++)
            if (k < n) mx = max(mx, (int)run_at<2>(e, k));
        int run = block_excl_max(mx, s_w);
        uint32_t wd[2] = {0u, 0u};
#pragma unroll
        for (int k = 0; k < kFlatRun; k++) {
            if (k < n) {
                if (run > p0 + k) wd[k >> 5] |= 1u << (k & 31);
                run = max(run, (int)run_at<2>(e, k));
            }
        }
        if (p0 < M) {
            s_bits[p0 >> 5] = wd[0];
            if (R == 64) s_bits[(p0 >> 5) + 1] = wd[1];
        }
    }
    __syncthreads();
    // alive leaves and condition-false nodes of the thread's run of F* entries
    const int* fn = order + HLGS_CUT_ORDER_HEADER;
    const int n = max(0, min(R, M - p0));
    uint64_t leaf = 0, stop = 0;
    {
        uint32_t pr[kFlatRun / 2], sw[kFlatRun / 4];
        load_run<2>(fn + ((2 * M + 3) & ~3), min(p0, M & ~31), pr);
        load_run<1>(st8, min(p0, M & ~31), sw);
#pragma unroll
        for (int k = 0; k < kFlatRun; k++) {
            const int st = run_at<1>(sw, k), pre = run_at<2>(pr, k);
            const bool alive = k < n && !((s_bits[pre >> 5] >> (pre & 31)) & 1u);
            if (alive && st == 1) leaf |= 1ull << k;
            if (alive && st == 2) stop |= 1ull << k;
        }
    }
    int3 tot;
    const int3 o = block_excl3(make_int3(__popcll(leaf), __popcll(stop), 0), s_w, &tot);
    // (leaves, stops) before each level's first entry
    for (int l = 0; l < nlev; l++) {
        const int sl = s_ls[l];
        if (sl >= p0 && sl < p0 + n) {
            const uint64_t below = (1ull << (sl - p0)) - 1ull;
            s_lev[l] = make_int2(o.x + __popcll(leaf & below), o.y + __popcll(stop & below));
        }
    }
    if (t == 0) s_lev[nlev] = make_int2(tot.x, tot.y);
    __syncthreads();
    a.flat->leaf[t] = leaf;
    a.flat->stop[t] = stop;
    a.flat->off[t] = make_int2(o.x, o.y);
    if (t <= nlev) a.flat->lev[t] = s_lev[t];
    if (t == 0) {
        const bool over = tot.x + tot.y > a.capacity;
        a.count[0] = over ? 0 : tot.x + tot.y;
        a.count[1] = over ? 1 : 0;
    }
}

// Placement, one thread per F* entry (consecutive lanes, consecutive entries: the stores of a wave land in one or two
// runs of consecutive cut positions).  In k_cut_flat_place each thread stored its own run's nodes, 64 scattered
// store instructions per wave from a single workgroup: 45 us of its time.
__global__ void __launch_bounds__(256) k_cut_flat_write(CutArgs a, const int* __restrict__ order)
{
    __shared__ int s_ls[HLGS_CUT_FLAT_MAX_LEVELS + 1];
    __shared__ int2 s_lev[HLGS_CUT_FLAT_MAX_LEVELS + 1];
    const int M = order[0], nlev = order[1];
    if (!flat_blob_ok(a, order) || a.count[1])
        return;  // (uniform) reported by k_cut_flat_place
    const int t = threadIdx.x;
    if (t <= nlev) {
        s_ls[t] = order[4 + t];
        s_lev[t] = a.flat->lev[t];
    }
    __syncthreads();
    const int i = blockIdx.x * 256 + t;
    if (i >= M) return;
    const int R = ((M + 1023) / 1024 + 31) & ~31;
    const int run = i / R, k = i - run * R;
    const uint64_t leaf = a.flat->leaf[run], stop = a.flat->stop[run];
    const bool isl = (leaf >> k) & 1ull, iss = (stop >> k) & 1ull;
    if (!isl && !iss) return;
    int lo = 0, hi = nlev - 1;  // the level holding entry i: last l with s_ls[l] <= i
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_ls[mid] <= i) lo = mid;
        else hi = mid - 1;
    }
    const int2 off = a.flat->off[run];
    const uint64_t below = (1ull << k) - 1ull;
    const int pos = isl ? s_lev[lo].y + off.x + __popcll(leaf & below) : s_lev[lo + 1].x + off.y + __popcll(stop & below);
    a.cut[pos] = order[HLGS_CUT_ORDER_HEADER + i];
}

void launch_upper_cut_flat(const CutArgs& a, const int* order, hipStream_t s)
{
    // the frontier buffers of the level walk hold the per-entry words and the preorder ends
    uint8_t* st8 = reinterpret_cast<uint8_t*>(a.front_a);
    uint16_t* endv = reinterpret_cast<uint16_t*>(a.front_b);
    hipLaunchKernelGGL(k_cut_flat_eval, dim3((a.N + 255) / 256), dim3(256), 0, s, a, order, st8, endv);
    hipLaunchKernelGGL(k_cut_flat_place, dim3(1), dim3(1024), 0, s, a, order, st8, endv);
    hipLaunchKernelGGL(k_cut_flat_write, dim3((a.N + 255) / 256), dim3(256), 0, s, a, order);
}

size_t upper_cut_state_bytes()
{
    const size_t walk = sizeof(CutState) + sizeof(unsigned) * kCutLevelLaunches + sizeof(int) * 3 * kCutMaxBlocks;
    return (walk + 255) / 256 * 256 + sizeof(CutFlat);  // capi.hip places CutFlat at align_up(walk)
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
    const int U = tb.device_only ? 4 : 1;  // 16-byte lanes for device-only tables, 4-byte lanes across the host link
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
    const float* res[kMaxRowTables];  // load only: the resident tables rows may be taken from (see resident_of)
    int words[kMaxRowTables];
};

// Load with resident_of (per host row: the resident row that holds the same Gaussian, or -1): a row still resident
// -- written back by this very step and loaded again, as the upper-tree Gaussians are every step -- is copied from
// the resident tables instead of over the host link.  The write-back has already put the same bits in host storage.
template <bool TO_HOST>
__global__ void __launch_bounds__(256) k_rows_packed(PackTabs tabs, int T, int64_t n, const int* __restrict__ dev_rows,
                                                     const int* __restrict__ host_rows, float* __restrict__ host,
                                                     int hw, const int* __restrict__ resident_of)
{
    const int lane = threadIdx.x & 63;
    float* base[kPackSlots];
    const float* res[kPackSlots];
    int width[kPackSlots], off[kPackSlots];
    bool live[kPackSlots];
#pragma unroll
    for (int m = 0; m < kPackSlots; m++) {
        const int w = lane + 64 * m;
        int start = 0, t = 0;
        while (t < T && w >= start + tabs.words[t]) start += tabs.words[t++];
        live[m] = t < T;  // a data word (else padding, or beyond the row when m * 64 >= hw)
        base[m] = live[m] ? tabs.t[t] : nullptr;
        res[m] = live[m] ? tabs.res[t] : nullptr;
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
            const int64_t rr = resident_of ? resident_of[hr] : -1;  // wave-uniform
            if (rr >= 0) {
#pragma unroll
                for (int m = 0; m < kPackSlots; m++) v[m] = live[m] ? res[m][rr * width[m] + off[m]] : 0.f;
            } else {
#pragma unroll
                for (int m = 0; m < kPackSlots; m++) v[m] = live[m] ? hrow[lane + 64 * m] : 0.f;
            }
#pragma unroll
            for (int m = 0; m < kPackSlots; m++)
                if (live[m]) base[m][dr * width[m] + off[m]] = v[m];
        }
    }
}

void launch_rows_packed(int T, float* const* tabs, const int* words, int64_t n, const int* dev_rows,
                        const int* host_rows, float* host, int hw, bool to_host, hipStream_t s,
                        const float* const* resident, const int* resident_of)
{
    PackTabs pt{};
    for (int t = 0; t < T; t++) {
        pt.t[t] = tabs[t];
        pt.res[t] = resident ? resident[t] : nullptr;
        pt.words[t] = words[t];
    }
    // 4 waves (rows) per block, grid-stride above.  The write-back's stores cross the host link, and while they are in
    // flight every kernel beside it waits longer for memory -- a 4-element torch add beside it took 160 us, the
    // rasterizer's preprocess 73 -> 190-240 us -- in proportion to how many of them are outstanding.  24 workgroups
    // (96 waves) keep it at ~0.6 ms, inside the step it overlaps, with a small fraction of that pressure: config #5
    // 2.30 ms per step at 128 workgroups, 2.13-2.16 at 16-24 (round 6, tools/c5_trace.sh; 8 workgroups took 1.5 ms
    // and delayed the next step's load).  The load keeps the large grid: with 256 workgroups (fewer host reads in
    // flight) it took 513 against 392 us.
    constexpr int64_t kWriteBackBlocks = 24;
    const int64_t blocks = std::min<int64_t>((n + 3) / 4, to_host ? kWriteBackBlocks : 2048);
    if (blocks <= 0) return;
    if (to_host) hipLaunchKernelGGL(k_rows_packed<true>, dim3((unsigned)blocks), dim3(256), 0, s, pt, T, n, dev_rows, host_rows, host, hw, (const int*)nullptr);
    else hipLaunchKernelGGL(k_rows_packed<false>, dim3((unsigned)blocks), dim3(256), 0, s, pt, T, n, dev_rows, host_rows, host, hw, resident_of);
}

// Compaction inside device memory (dst_rows = identity, every table device-only): dst_t[i] = src_t[src_rows[i]].
// Lane = one 16-byte chunk of the destination (aligned store).  Its four source words lie in rows r .. r_end; when
// those rows are consecutive in the source too (src_rows[r_end] - src_rows[r] = r_end - r, which holds inside the
// long runs of kept rows) they are one contiguous 16-byte load at 4-byte alignment, otherwise four word loads.
// Round 6: one 1-D grid over every table's chunks -- block b copies kCompactChunks consecutive chunks of one table
// (CompactTabs::bstart, the blocks of the tables before it) -- instead of a 2-D grid of 2,048 blocks per table, in which
// the narrow tables (opacity, 3-float rows: a few hundred blocks of work) left most of their blocks idle and the wide
// SH tables took ~13 grid-stride chunks per thread.
constexpr int kCompactU = 4;                      // chunks per thread, their loads issued together
constexpr int kCompactChunks = 256 * kCompactU;   // chunks per block
constexpr int kCompactTables = 20;                // the cache's 18 tables (a smaller kernel argument block)
struct CompactTabs {
    RowCopy t[kCompactTables];
    int bstart[kCompactTables + 1];                // first block of each table; bstart[T] = the grid
};
__global__ void __launch_bounds__(256) k_rows_compact(CompactTabs tabs, int T, int64_t n, const int* __restrict__ src_rows)
{
    int t = 0;  // this block's table (uniform): the last table whose first block is <= blockIdx.x
    for (int j = 1; j < T; j++) t += (int)blockIdx.x >= tabs.bstart[j];
    const RowCopy& tb = tabs.t[t];
    const int64_t words = tb.row_bytes >> 2;
    const uint32_t* __restrict__ src = static_cast<const uint32_t*>(tb.src);
    uint32_t* __restrict__ dst = static_cast<uint32_t*>(tb.dst);
    const int64_t total = n * words;
    // chunk u of this thread: block chunk base + 256 u + thread, so a wave's lanes take consecutive chunks
    const int64_t w0 = ((int64_t)(blockIdx.x - tabs.bstart[t]) * kCompactChunks + threadIdx.x) * 4;
    if (w0 >= total) return;
    int64_t rr[kCompactU], kk[kCompactU], re[kCompactU];
    {
        constexpr int64_t S = 256 * 4;  // words between a thread's chunks
        const int64_t dr = S / words, dk = S - dr * words;
        int64_t r1 = w0 / words, k1 = w0 - r1 * words;
#pragma unroll
        for (int u = 0; u < kCompactU; u++) {
            rr[u] = r1;
            kk[u] = k1;
            re[u] = r1 + (k1 + 3) / words;
            r1 += dr;
            k1 += dk;
            while (k1 >= words) { k1 -= words; r1++; }
        }
    }
    int s0[kCompactU], s1[kCompactU];
#pragma unroll
    for (int u = 0; u < kCompactU; u++) {
        const bool in = w0 + u * 1024 < total;
        s0[u] = in ? src_rows[rr[u]] : 0;
        s1[u] = in ? src_rows[min(re[u], n - 1)] : 0;
    }
    uint4 v[kCompactU];
    bool fast[kCompactU];
#pragma unroll
    for (int u = 0; u < kCompactU; u++) {
        const int64_t wu = w0 + u * 1024;
        fast[u] = wu + 4 <= total && s1[u] - s0[u] == re[u] - rr[u];
        if (fast[u]) v[u] = *reinterpret_cast<const uint4_a4*>(src + (int64_t)s0[u] * words + kk[u]);
    }
#pragma unroll
    for (int u = 0; u < kCompactU; u++) {
        const int64_t wu = w0 + u * 1024;
        if (wu >= total) continue;
        if (fast[u]) {
            *reinterpret_cast<uint4*>(dst + wu) = v[u];
        } else {
            int64_t r2 = rr[u], k2 = kk[u];
            for (int q = 0; q < 4 && wu + q < total; q++) {
                dst[wu + q] = src[(int64_t)src_rows[r2] * words + k2];
                if (++k2 == words) { k2 = 0; r2++; }
            }
        }
    }
}

void launch_rows_multi(int T, const RowCopy* tabs, int64_t n, const int* src_rows, const int* dst_rows, hipStream_t s)
{
    bool compact = src_rows && !dst_rows && T <= kCompactTables;
    for (int t = 0; t < T && compact; t++)
        compact = tabs[t].device_only && (reinterpret_cast<uintptr_t>(tabs[t].dst) & 15u) == 0;
    if (compact) {
        CompactTabs ct{};
        int64_t blocks = 0;
        for (int t = 0; t < T; t++) {
            ct.t[t] = tabs[t];
            ct.bstart[t] = (int)blocks;
            const int64_t chunks = (n * (tabs[t].row_bytes >> 2) + 3) / 4;
            blocks += (chunks + kCompactChunks - 1) / kCompactChunks;
        }
        ct.bstart[T] = (int)blocks;
        if (blocks > 0 && blocks < (1ll << 31))
            hipLaunchKernelGGL(k_rows_compact, dim3((unsigned)blocks), dim3(256), 0, s, ct, T, n, src_rows);
        if (blocks < (1ll << 31)) return;
    }
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

// A workgroup barrier that orders LDS only: global loads issued before it stay in flight (__syncthreads waits for
// every outstanding memory operation, vmcnt(0), which would drain k_cache_lists' prefetches at each scan).
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
// exclusive prefixes of two flags over the 1024-thread block in one pass (per-wave counts packed 16 + 16 bits)
__device__ __forceinline__ void block_excl2(int fa, int fb, int* s_w, int& pa, int& pb, int& ta, int& tb)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t ba = __ballot(fa), bb = __ballot(fb), below = (1ull << lane) - 1ull;
    lds_barrier();
    if (lane == 0) s_w[w] = __popcll(ba) | (__popcll(bb) << 16);
    lds_barrier();
    int before = 0, t = 0;
    for (int i = 0; i < 16; i++) {
        const int c = s_w[i];
        if (i < w) before += c;
        t += c;
    }
    pa = (before & 0xffff) + __popcll(ba & below);
    pb = (before >> 16) + __popcll(bb & below);
    ta = t & 0xffff;
    tb = t >> 16;
}

// Cut-entry fields k_cache_lists' first loop reads (v < 0: past the cut's end)
struct CutEntry {
    int v, leaf_n, fc, gid;
    float x, y, z;
};
__device__ __forceinline__ CutEntry cut_entry(const CacheArgs& a, int v)
{
    CutEntry e{v, 1, -1, 0, 0.f, 0.f, 0.f};
    if (v >= 0) {
        e.leaf_n = a.nodes[6 * v + 2];
        e.fc = a.nodes[6 * v + 3];
        e.gid = a.nodes[6 * v + 5];
        e.x = a.xyz[3 * v];
        e.y = a.xyz[3 * v + 1];
        e.z = a.xyz[3 * v + 2];
    }
    return e;
}

constexpr int kListsLdsSpts = 4096;  // the cut's SPT ids searched from LDS up to this many
__global__ void __launch_bounds__(1024) k_cache_lists(CacheArgs a)
{
#pragma clang fp contract(off)
    __shared__ int s_w[16];
    __shared__ int s_spt[kListsLdsSpts];
    // 1. leaves of the cut, in cut order: SPT leaves (first_child >= 0, with their camera distance) and
    //    upper-tree Gaussians to render (first_child <= 0; a leaf holding SPT 0 is in both lists, as in the
    //    reference's two masks).  Software-pipelined: while one 1024-entry chunk is scanned and written, the next
    //    chunk's node fields and the cut entries of the one after are in flight (one workgroup: it waits for every
    //    load it does not overlap).
    int ns = 0, nu = 0;
    const int n_cut = a.n_cut_dev ? (a.n_cut_dev[1] ? 0 : min(a.n_cut_dev[0], a.n_cut)) : a.n_cut;
    auto cut_at = [&](int i) -> int { return i < n_cut ? a.cut[i] : -1; };
    CutEntry cur = cut_entry(a, cut_at(threadIdx.x));
    int v_next = cut_at(1024 + threadIdx.x);
    for (int c0 = 0; c0 < n_cut; c0 += 1024) {
        const CutEntry nxt = cut_entry(a, v_next);
        v_next = cut_at(c0 + 2048 + threadIdx.x);
        const bool leaf = cur.v >= 0 && cur.leaf_n == 0;
        const bool is_s = leaf && cur.fc >= 0, is_u = leaf && cur.fc <= 0;
        int ps, pu, ts, tu;
        block_excl2(is_s, is_u, s_w, ps, pu, ts, tu);
        if (is_s) {
            float d2 = INFINITY;  // nearest camera
            for (int g = 0; g < a.nviews; g++) {
                const float dx = cur.x - a.campos[3 * g], dy = cur.y - a.campos[3 * g + 1],
                            dz = cur.z - a.campos[3 * g + 2];
                d2 = fminf(d2, dx * dx + dy * dy + dz * dz);
            }
            a.spt_idx[ns + ps] = cur.fc;
            a.spt_dist[ns + ps] = sqrtf(d2) * a.dmul;
            if (ns + ps < kListsLdsSpts) s_spt[ns + ps] = cur.fc;
        }
        if (is_u) a.upper[nu + pu] = cur.gid;
        ns += ts;
        nu += tu;
        cur = nxt;
    }
    __syncthreads();
    // 2. previous SPTs: torch.searchsorted (lower bound; the list is in cut order, not sorted, and the search
    //    runs on it as it is), equal id and isclose distance -> kept, with the reference's segment bounds.  The
    //    search reads the LDS copy of the cut's SPT ids when they fit.
    const bool spt_lds = ns <= kListsLdsSpts;
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
                if (!((spt_lds ? s_spt[mid] : a.spt_idx[mid]) >= pv)) lo = mid + 1;
                else hi = mid;
            }
            keep = lo < ns && (spt_lds ? s_spt[lo] : a.spt_idx[lo]) == pv && is_close(a.spt_dist[lo], a.prev_dist[j], a.rtol, a.atol);
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
            v = spt_lds ? s_spt[k] : a.spt_idx[k];
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
        a.sizes[5] = a.n_cut_dev ? (a.n_cut_dev[1] || a.n_cut_dev[0] > a.n_cut) : 0;  // the cut overflowed
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
