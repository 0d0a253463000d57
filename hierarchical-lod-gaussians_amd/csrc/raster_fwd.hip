// raster_fwd.hip -- forward rasterizer kernels for gfx950.
//
// Reference semantics (submodules/hierarchy-rasterizer/cuda_rasterizer; the preprocess is in preprocess.hip):
//   k_tile_ranges     <- identifyTileRanges  rasterizer_impl.cu:120-142 (from the tile-count scan)
//   k_scatter_keys    <- duplicateWithKeys   rasterizer_impl.cu:70-115
//   k_tile_sort / k_merge_runs <- cub::DeviceRadixSort::SortPairs rasterizer_impl.cu:355-363
//   k_blend_fwd       <- renderCUDA<3>       forward.cu:450-596
//
// Binning is re-designed for MI355X: instead of one 45-bit global LSD radix sort (6+ passes over R
// 12-byte pairs) instances are counted per tile in the preprocess, scattered once into their tile's
// segment, and each segment is sorted in LDS by the total order (depth bits, Gaussian index).  That
// is exactly the order CUB's stable sort of (tile | depth) produces from the reference's
// Gaussian-ordered duplicate list, so point_list is identical.
#include <algorithm>

#include "hlgs_internal.h"
#include "hlgs_math.h"

namespace hlgs {

// ------------------------------------------------------------------------------------------------
// Tile binning with block-level LDS histograms.  A block owns BG consecutive Gaussians (bin_gauss); its
// instances are counted per tile in LDS and each non-empty bin costs one coalesced device atomic,
// instead of one lane-scattered atomic per (Gaussian, tile) instance.
// ------------------------------------------------------------------------------------------------
// s_pre[k] = exclusive prefix of tiles_touched over the block's BG Gaussians (0 past P), s_pre[BG] =
// the block's total: thread t scans its BG / 1024 consecutive entries, then the 1024 thread totals are scanned.
// Every binning block has 1024 threads, so a thread takes four Gaussians at 4,096 per block and one at 1,024 (round 5,
// config #5's count / scatter: 512-thread blocks of 2,048 78 / 87 us, 1024-thread blocks of 2,048 61 / 70 us, of
// 1,024 51 / 57 us, the plan 16 -> 22 us for the doubled histogram rows).
// The rect sizes thread t scans (Gaussians J t .. J t + J - 1 of the block, J = BG / 1024), loaded apart from the
// scan so that a kernel can issue them together with its other first-round loads.
template <int BG>
__device__ __forceinline__ void block_rect_sizes(int P, const Geom& g, uint32_t (&a)[BG / 1024])
{
    const int g0 = blockIdx.x * BG, t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < BG / 1024; k++) {
        const int idx = g0 + (BG / 1024) * t + k;
        a[k] = idx < P ? g.tiles_touched[idx] : 0u;
    }
}
template <int BG>
__device__ __forceinline__ void block_rect_prefix(const uint32_t (&a)[BG / 1024], uint32_t* s_pre, uint32_t* s_w)
{
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t sum = 0, mx = 0;
#pragma unroll
    for (int k = 0; k < BG / 1024; k++) {
        sum += a[k];
        mx = max(mx, a[k]);
    }
    for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
    if (lane == 0) atomicMax(&s_w[(1024) / 64], mx);
    uint32_t x = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t base = 0, total = 0;
    for (int i = 0; i < (1024) / 64; i++) {
        const uint32_t c = s_w[i];
        if (i < w) base += c;
        total += c;
    }
    uint32_t run = base + x - sum;
#pragma unroll
    for (int k = 0; k < BG / 1024; k++) {
        s_pre[(BG / 1024) * t + k] = run;
        run += a[k];
    }
    if (t == 0) s_pre[BG] = total;
    __syncthreads();
}

// the block's longest rect (s_w[(1024) / 64], zeroed before block_rect_prefix)
constexpr uint32_t kNarrowRect = 64;

// Calls f(idx, x, y, qm, dbits) for every binned instance (Gaussian idx, tile (x, y)) of the block's Gaussians: every
// tile of the rect, or for the alt rasterizer the tiles alt_tile_keep leaves (rasterizer_impl.cu:147-179 of
// alt-rasterizer).  KEYS: dbits = the Gaussian's depth bits (the sort key's high word); MASKS: qm = the instance's
// footprint quadrant mask, from the masks the preprocess left in Geom::qmask (rect_tile_mask); otherwise 0.
// Without wide rects each thread takes BG / 1024 Gaussians and loads everything they need before its first call, so the
// key stores issued by f never have to drain for a later load (vmcnt counts loads and stores alike).  With a wide
// rect the block's instances are numbered Gaussian by Gaussian (s_pre) and each thread takes one contiguous run of
// them, so a Gaussian whose rect spans thousands of tiles is spread over the whole block instead of serialising one
// thread.
struct GIn {
    float2 xy;
    int2 ext;
    float4 co;
    uint32_t masks, dbits;
};
template <bool KEYS, bool MASKS>
__device__ __forceinline__ void gauss_in(const Geom& g, bool alt, int idx, GIn& v)
{
    v.xy = g.means2D[idx];
    v.ext = g.rects[idx];
    v.co = make_float4(0.f, 0.f, 0.f, 0.f);
    if (alt) {
        const float4 r0 = g.splat[4 * (size_t)idx], r1 = g.splat[4 * (size_t)idx + 1];
        v.co = make_float4(r0.z, r0.w, r1.x, r1.y);
    }
    v.masks = MASKS ? g.qmask[idx] : 0u;
    v.dbits = KEYS ? __float_as_uint(g.depths[idx]) : 0u;
}
// The narrow path's inputs (Gaussians threadIdx.x + j 1024 of the block, every one below P, culled or not), issued at
// the top of a kernel with its other first-round loads; for_each_instance then reads no Gaussian input itself.
template <int BG, bool MASKS>
__device__ __forceinline__ void prefetch_instances(const Geom& g, bool alt, int P, GIn (&in)[BG / 1024])
{
    const int g0 = blockIdx.x * BG;
#pragma unroll
    for (int j = 0; j < BG / 1024; j++) {  // past P: Gaussian P - 1 again (not used), so the loads need no branch
        const int idx = min(g0 + (int)threadIdx.x + j * (1024), P - 1);
        gauss_in<false, MASKS>(g, alt, idx, in[j]);
    }
}

template <int BG, bool KEYS, bool MASKS, typename F>
__device__ __forceinline__ void for_each_instance(const Geom& g, int P, int gx, int gy, bool alt, const uint32_t* s_pre,
                                                  const uint32_t* s_w, const GIn (&pre)[BG / 1024], F&& f)
{
    const int g0 = blockIdx.x * BG;
    auto gauss = [&](int idx, GIn& v) { gauss_in<KEYS, MASKS>(g, alt, idx, v); };
    auto qmask = [&](uint32_t masks, uint32_t r) { return MASKS ? rect_tile_mask(masks, r) : 0u; };
    if (s_w[(1024) / 64] <= kNarrowRect) {  // no wide rect in this block: one thread per Gaussian
        constexpr int J = BG / 1024;  // Gaussians per thread
        GIn in[J];
        bool live[J];
#pragma unroll
        for (int j = 0; j < J; j++) {
            const int k = threadIdx.x + j * (1024);
            live[j] = s_pre[k + 1] != s_pre[k];
            in[j] = pre[j];
        }
#pragma unroll
        for (int j = 0; j < J; j++) {
            if (!live[j]) continue;
            const int idx = g0 + threadIdx.x + j * (1024);
            const GIn& v = in[j];
            int x0, y0, x1, y1;
            tile_rect(v.xy.x, v.xy.y, v.ext.x, v.ext.y, gx, gy, x0, y0, x1, y1);
            uint32_t r = 0;
            if (alt) {
                const AltKeep thr = alt_keep_prep(v.co);
                for (int y = y0; y < y1; y++)
                    for (int x = x0; x < x1; x++, r++)
                        if (alt_tile_keep(v.xy.x, v.xy.y, v.co, thr, x, y)) f(idx, x, y, qmask(v.masks, r), v.dbits);
            } else {
                for (int y = y0; y < y1; y++)
                    for (int x = x0; x < x1; x++, r++) f(idx, x, y, qmask(v.masks, r), v.dbits);
            }
        }
        return;
    }
    const uint32_t total = s_pre[BG];
    const uint32_t chunk = (total + (1024) - 1) / (1024);
    uint32_t i = threadIdx.x * chunk;
    const uint32_t iend = min(total, i + chunk);
    if (i >= iend) return;
    int lo = 0, hi = BG - 1;  // last k with s_pre[k] <= i: the Gaussian holding instance i
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_pre[mid] <= i) lo = mid;
        else hi = mid - 1;
    }
    // the instances of Gaussian k from i on, up to the run's end
    auto walk = [&](int k, const GIn& v) {
        const uint32_t b = s_pre[k], e = s_pre[k + 1];
        const int idx = g0 + k;
        int x0, y0, x1, y1;
        tile_rect(v.xy.x, v.xy.y, v.ext.x, v.ext.y, gx, gy, x0, y0, x1, y1);
        const int w = x1 - x0;
        const uint32_t local = i - b;
        int ty = (int)(local / (uint32_t)w), tx = (int)local - ty * w;
        const uint32_t stop = min(iend, e);
        if (alt) {
            const AltKeep thr = alt_keep_prep(v.co);
            for (; i < stop; i++) {
                if (alt_tile_keep(v.xy.x, v.xy.y, v.co, thr, x0 + tx, y0 + ty))
                    f(idx, x0 + tx, y0 + ty, qmask(v.masks, i - b), v.dbits);
                if (++tx == w) { tx = 0; ty++; }
            }
        } else {
            for (; i < stop; i++) {
                f(idx, x0 + tx, y0 + ty, qmask(v.masks, i - b), v.dbits);
                if (++tx == w) { tx = 0; ty++; }
            }
        }
    };
    // the run's first kWidePre Gaussians are loaded together (a run crosses several small Gaussians when one wide
    // rect puts its whole block on this path), the rest one by one
    constexpr int kWidePre = 4;
    GIn pv[kWidePre];
#pragma unroll
    for (int u = 0; u < kWidePre; u++) gauss(min(g0 + lo + u, P - 1), pv[u]);  // clamped: no branch before the loads
#pragma unroll
    for (int u = 0; u < kWidePre; u++) {
        if (i >= iend) return;
        if (s_pre[lo + u + 1] != s_pre[lo + u]) walk(lo + u, pv[u]);
    }
    for (int k = lo + kWidePre; i < iend; k++) {
        if (s_pre[k + 1] == s_pre[k]) continue;
        GIn v;
        gauss(g0 + k, v);
        walk(k, v);
    }
}

// hist != nullptr (bin_histogram): the block's per-tile counts are stored as row blockIdx.x of hist (coalesced), and
// k_tile_offsets turns the rows into per-(block, tile) offsets and tile totals; otherwise they are added to
// tile_count with one device atomic per non-empty tile.  zero_words: k_tile_offsets_plan's look-back words and the
// plan's failure / completion words (misc[kMiscFail], misc[kMiscDone]), cleared by block 0 for this frame.
template <int BG, bool DROP>
__global__ void __launch_bounds__(1024) k_count_tiles(int P, const int* __restrict__ radii, Geom g,
                                                             uint32_t* __restrict__ tile_count, int gx, int gy, int alt,
                                                             uint32_t* __restrict__ block_tot, uint32_t* __restrict__ hist,
                                                             uint32_t* __restrict__ zero_words, int n_zero,
                                                             uint32_t* __restrict__ misc)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t s_hist[];
    __shared__ uint32_t s_pre[BG + 1];
    __shared__ uint32_t s_w[(1024) / 64 + 1];
    const int T = gx * gy;
    // every input in the first round trip (the rect sizes for the scan and the narrow walk's Gaussians)
    uint32_t sizes[BG / 1024];
    block_rect_sizes<BG>(P, g, sizes);
    GIn pre[BG / 1024];
    prefetch_instances<BG, DROP>(g, alt, P, pre);
    for (int t = threadIdx.x; t < T; t += (1024)) s_hist[t] = 0;
    if (threadIdx.x == 0) s_w[(1024) / 64] = 0;
    __syncthreads();
    block_rect_prefix<BG>(sizes, s_pre, s_w);
    if (threadIdx.x == 0) block_tot[blockIdx.x] = s_pre[BG];
    if (zero_words && blockIdx.x == 0) {  // k_tile_offsets_plan's look-back words, failure and completion words
        for (int i = threadIdx.x; i < n_zero; i += 1024) zero_words[i] = 0u;
        if (threadIdx.x == 0) { misc[kMiscFail] = 0u; misc[kMiscDone] = 0u; }
    }
    for_each_instance<BG, false, DROP>(g, P, gx, gy, alt, s_pre, s_w, pre, [&](int, int x, int y, uint32_t qm, uint32_t) {
        if (!DROP || qm) atomicAdd(&s_hist[y * gx + x], 1u);
    });
    __syncthreads();
    if (hist) {
        uint32_t* row = hist + (size_t)blockIdx.x * T;
        for (int t = threadIdx.x; t < T; t += (1024)) row[t] = s_hist[t];
        return;
    }
    for (int t = threadIdx.x; t < T; t += (1024)) {
        const uint32_t c = s_hist[t];
        if (c) atomicAdd(&tile_count[t], c);
    }
}

// A tile segment holds the count blocks' runs in XCD-grouped block order (xcd_unmap), not in block order,
// so that the runs next to each other in memory are written by scatter blocks of the same XCD (workgroups go to XCDs
// round robin): their partial lines meet in that XCD's L2 and leave it whole, instead of as partial lines from eight
// L2s.  The order inside a segment is free (k_tile_sort orders it).
// The histogram rows of logical positions i, i + 1, ... in that order, stepped without a division per row.
struct HistRows {
    int i, x, k, q, r;
    __device__ HistRows(int i0, int nb) : i(i0), x(0), k(0), q(nb / 8), r(nb % 8)
    {
        const int b = xcd_unmap(i0, nb);
        x = b % 8;
        k = b / 8;
    }
    __device__ int row() const { return x + 8 * k; }
    __device__ void next()
    {
        i++;
        if (++k == (x < r ? q + 1 : q)) { x++; k = 0; }
    }
};
// The count blocks' histogram rows (nb x T) -> in place, each block's exclusive offset inside every tile's segment (the
// blocks in order), and tile_count[t] = the tile's total.  32 tiles per workgroup (128-byte row segments), 32 row
// groups of 32 threads; each thread takes a contiguous run of blocks down its tile's column, issues all of a run's
// loads before adding (up to 8 held in registers, so the offsets are written without a second read), and the 32 run
// totals of a tile are scanned in LDS.  With it the binning has no device atomics and a tile's segment holds the
// blocks' runs in block order.
template <int K>  // histogram rows per thread held in registers: 8, or 24 for the 1,024-Gaussian blocks' longer columns
__global__ void __launch_bounds__(1024) k_tile_offsets(uint32_t* __restrict__ hist, int nb, int T,
                                                       uint32_t* __restrict__ tile_count)
{
    __shared__ uint32_t s_part[32][33];
    const int c = threadIdx.x & 31, r = threadIdx.x >> 5;
    const int t = blockIdx.x * 32 + c;
    const int run = (nb + 31) / 32, b0 = r * run, b1 = min(nb, b0 + run);
    uint32_t v[K];
    int rows[K];
    uint32_t sum = 0;
    if (t < T) {
        if (run <= K) {
            HistRows it(b0, nb);
#pragma unroll
            for (int k = 0; k < K; k++) {
                rows[k] = it.row();
                it.next();
            }
#pragma unroll
            for (int k = 0; k < K; k++) v[k] = b0 + k < b1 ? hist[(size_t)rows[k] * T + t] : 0u;
#pragma unroll
            for (int k = 0; k < K; k++) sum += v[k];
        } else {
            HistRows it(b0, nb);
            for (int b = b0; b < b1; b++, it.next()) sum += hist[(size_t)it.row() * T + t];
        }
    }
    s_part[r][c] = sum;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) {
        const uint32_t x = s_part[i][c];
        if (i < r) off += x;
        tot += x;
    }
    if (t >= T) return;
    if (run <= K) {
#pragma unroll
        for (int k = 0; k < K; k++)
            if (b0 + k < b1) {
                hist[(size_t)rows[k] * T + t] = off;
                off += v[k];
            }
    } else {
        HistRows it(b0, nb);
        for (int b = b0; b < b1; b++, it.next()) {
            uint32_t* h = hist + (size_t)it.row() * T + t;
            const uint32_t x = *h;
            *h = off;
            off += x;
        }
    }
    if (r == 0) tile_count[t] = tot;
}

// Same block -> Gaussian mapping as k_count_tiles: reserve the block's run inside every tile segment
// with one returning atomic per bin, then hand out slots from LDS.  Slot order inside a tile is
// irrelevant: k_tile_sort orders each segment by (depth, index) afterwards.
// hist != nullptr: the block's base inside each tile segment is ranges[t].x + its k_tile_offsets offset, so the block
// walks its instances once (no count walk, no returning device atomics).
template <int BG, bool PACK>
__global__ void __launch_bounds__(1024) k_scatter_keys_lds(int P, const int* __restrict__ radii, Geom g,
                                                                  const uint2* __restrict__ ranges, uint32_t* cursor,
                                                                  uint64_t* __restrict__ keys, int gx, int gy, int alt,
                                                                  Guard gd, const uint32_t* __restrict__ block_tot,
                                                                  const uint32_t* __restrict__ hist)
{
    if (guard_fail(gd)) return;
    // 4-byte entries only (the low words of the sort keys): the tile sort gathers each entry's depth itself, so the
    // scattered stores -- about one per block and tile, each into its own line -- carry half the bytes
    uint32_t* __restrict__ ents = reinterpret_cast<uint32_t*>(keys);
    extern __shared__ __attribute__((aligned(16))) uint32_t s_hist[];
    __shared__ uint32_t s_base;
    __shared__ uint32_t s_pre[BG + 1];
    __shared__ uint32_t s_w[(1024) / 64 + 1];
    const int T = gx * gy;
    uint32_t* s_cnt = s_hist;      // per-tile count, then the block's base inside the tile segment
    uint32_t* s_rank = s_hist + T; // per-tile running rank
    // The first round trip carries every input the block needs: the rect sizes for the scan, the preceding blocks'
    // totals, the first kPreTiles of this thread's tile bases (the tile's range start + this block's histogram offset)
    // and the narrow walk's Gaussians.  (Issued one after another, the five rounds of loads had been the kernel's time.)
    constexpr int kPreTiles = 8;
    uint32_t sizes[BG / 1024];
    block_rect_sizes<BG>(P, g, sizes);
    // (every load unconditional, clamped into range, so that the compiler issues them back to back)
    uint32_t part = block_tot[min((int)threadIdx.x, max((int)blockIdx.x - 1, 0))];  // preceding block threadIdx.x
    uint32_t trange[kPreTiles], trow[kPreTiles];
    const uint32_t* row = hist ? hist + (size_t)blockIdx.x * T : nullptr;
    if (hist) {
#pragma unroll
        for (int k = 0; k < kPreTiles; k++) {
            const int t = min((int)threadIdx.x + k * (1024), T - 1);
            trange[k] = ranges[t].x;
            trow[k] = row[t];
        }
    }
    GIn pre[BG / 1024];
    prefetch_instances<BG, PACK>(g, alt, P, pre);
    if (threadIdx.x == 0) { s_w[(1024) / 64] = 0; s_base = 0; }
    if (hist) {
        for (int t = threadIdx.x; t < T; t += (1024)) s_rank[t] = 0;
    } else {
        for (int t = threadIdx.x; t < T; t += (1024)) { s_cnt[t] = 0; s_rank[t] = 0; }
    }
    __syncthreads();
    block_rect_prefix<BG>(sizes, s_pre, s_w);
    {  // point_offsets (the inclusive scan of tiles_touched) = the block's base + the block-local prefix; the base is
       // the sum of the preceding count blocks' totals (k_count_tiles): thread i adds block i's, and i + 1024 ... too
        if ((int)threadIdx.x >= (int)blockIdx.x) part = 0;
        for (int i = threadIdx.x + 1024; i < (int)blockIdx.x; i += 1024) part += block_tot[i];
        if (part) atomicAdd(&s_base, part);
        __syncthreads();
        const int g0 = blockIdx.x * BG, g1 = min(P, g0 + BG);
        const uint32_t base = s_base;
        for (int idx = g0 + (int)threadIdx.x; idx < g1; idx += (1024)) {
            const int k = idx - g0;
            g.point_offsets[idx] = base + s_pre[k + 1];
        }
    }
    if (hist) {
#pragma unroll
        for (int k = 0; k < kPreTiles; k++) {
            const int t = (int)threadIdx.x + k * (1024);
            if (t < T) s_cnt[t] = trange[k] + trow[k];
        }
        for (int t = threadIdx.x + kPreTiles * (1024); t < T; t += (1024)) s_cnt[t] = ranges[t].x + row[t];
    } else {
        for_each_instance<BG, false, PACK>(g, P, gx, gy, alt, s_pre, s_w, pre, [&](int, int x, int y, uint32_t qm, uint32_t) {
            if (!(g.drop && !qm)) atomicAdd(&s_cnt[y * gx + x], 1u);
        });
        __syncthreads();
        for (int t = threadIdx.x; t < T; t += (1024)) {
            const uint32_t c = s_cnt[t];
            s_cnt[t] = c ? ranges[t].x + atomicAdd(&cursor[t], c) : 0u;
        }
    }
    __syncthreads();
    if (!alt && s_w[(1024) / 64] <= kNarrowRect) {
        // Narrow rects (for_each_instance's one-thread-per-Gaussian path): each thread's instances in groups of four,
        // the four rank atomics issued together and then the four key stores -- one at a time, every store waits for
        // its atomic's return.
        const int g0 = blockIdx.x * BG;
        constexpr int J = BG / 1024;
        bool live[J];
#pragma unroll
        for (int j = 0; j < J; j++) {
            const int k = threadIdx.x + j * (1024);
            live[j] = s_pre[k + 1] != s_pre[k];
        }
#pragma unroll
        for (int j = 0; j < J; j++) {
            if (!live[j]) continue;
            const uint32_t idx = (uint32_t)(g0 + threadIdx.x + j * (1024));
            const uint32_t gmask = pre[j].masks;
            int x0, y0, x1, y1;
            tile_rect(pre[j].xy.x, pre[j].xy.y, pre[j].ext.x, pre[j].ext.y, gx, gy, x0, y0, x1, y1);
            const int w = x1 - x0, n = w * (y1 - y0);
            int tx = 0, ty = 0;
            for (int c = 0; c < n; c += 4) {
                uint32_t pos[4], ent[4];
                bool use[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int r = c + u;
                    const uint32_t qm = PACK ? rect_tile_mask(gmask, (uint32_t)r) : 0u;
                    use[u] = r < n && !(g.drop && !qm);
                    const int tile = (y0 + ty) * gx + x0 + tx;
                    if (use[u]) pos[u] = s_cnt[tile] + atomicAdd(&s_rank[tile], 1u);
                    ent[u] = PACK ? (idx << kEntryShift) | qm : idx;
                    if (++tx == w) { tx = 0; ty++; }
                }
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (use[u]) ents[pos[u]] = ent[u];
            }
        }
        return;
    }
    for_each_instance<BG, false, PACK>(g, P, gx, gy, alt, s_pre, s_w, pre, [&](int idx, int x, int y, uint32_t qm, uint32_t) {
        if (g.drop && !qm) return;  // the footprint reaches none of the tile's quadrants
        const int tile = y * gx + x;
        const uint32_t r = atomicAdd(&s_rank[tile], 1u);
        ents[s_cnt[tile] + r] = PACK ? ((uint32_t)idx << kEntryShift) | qm : (uint32_t)idx;
    });
}

// ranges[t] = [incl[t] - count[t], incl[t]); misc[0] = R, misc[1] = max count; cursor reset for the scatter.
// misc[2] = point_offsets[P - 1]: instances over all tile rects (record slots; == misc[0] unless culled).
// misc[kMiscPack], misc[kMiscDrop] = the frame's FrameOpts (flags = pack | drop << 1), so the backward decodes the lists
// as they were written and a caller can read which binning the frame used.
__global__ void __launch_bounds__(256) k_tile_ranges(const uint32_t* __restrict__ count, uint32_t* incl_and_cursor,
                                                     uint2* __restrict__ ranges, uint32_t* __restrict__ misc, int T,
                                                     const uint32_t* __restrict__ point_offsets, int P, uint32_t flags)
{
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= T) return;
    const uint32_t c = count[t], e = incl_and_cursor[t];
    ranges[t] = make_uint2(e - c, e);
    incl_and_cursor[t] = 0;
    if (t == T - 1) {
        misc[0] = e;
        misc[2] = P > 0 ? point_offsets[P - 1] : 0u;
        misc[kMiscPack] = flags & 1u;
        misc[kMiscDrop] = flags >> 1;
    }
    if (c) atomicMax(&misc[1], c);
}

// Binning plan of the LDS-histogram path, one 1024-thread block: the sum of the count blocks' instance totals
// (record slots; each k_scatter_keys_lds block sums its predecessors' totals for its base and adds its local prefix to
// form point_offsets), the tile ranges from the per-tile counts, cursor reset, and misc[0..2] = R, longest list,
// record slots -- mirrored into the caller's pinned host words, so the host reads R without a copy.
// Replaces two device-wide scans, k_tile_ranges and the read-back copy (seven launches).
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_w, uint32_t& total)
{
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) s_w[wid] = x;
    __syncthreads();
    uint32_t woff = 0;
    total = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); w++) {
        const uint32_t c = s_w[w];
        if (w < wid) woff += c;
        total += c;
    }
    __syncthreads();
    return woff + x - v;
}

// Scan of n counts by one 1024-thread block, each thread over a contiguous run of up to kPlanRun entries (one
// block-wide scan of the run totals instead of a loop of them).  plan_load issues a run's loads; both of k_plan's
// inputs are loaded before either is scanned, so the block waits for one round trip, not two.
constexpr int kPlanRun = 16;  // 16 x 1024 >= kBinMaxTiles
struct PlanRun {
    uint32_t v[kPlanRun];
    int i0, run, n;
};
__device__ __forceinline__ void plan_load(const uint32_t* in, int n, PlanRun& r)
{
    r.n = n;
    r.run = (n + 1023) / 1024;  // <= kPlanRun (checked by the launcher)
    r.i0 = (int)threadIdx.x * r.run;
#pragma unroll
    for (int k = 0; k < kPlanRun; k++) r.v[k] = (k < r.run && r.i0 + k < n) ? in[r.i0 + k] : 0u;
}
template <typename F>
__device__ __forceinline__ uint32_t plan_scan(const PlanRun& r, uint32_t* s_w, uint32_t& mx, F&& emit)
{
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < kPlanRun; k++) {
        sum += r.v[k];
        mx = max(mx, r.v[k]);
    }
    uint32_t total;
    uint32_t ex = block_excl_scan(sum, s_w, total);
#pragma unroll
    for (int k = 0; k < kPlanRun; k++) {
        if (k < r.run && r.i0 + k < r.n) emit(r.i0 + k, ex, r.v[k]);
        ex += r.v[k];
    }
    return total;
}

// The plan's words for the host in its pinned read-back slot (capi.hip plan_words_ready).
__device__ __forceinline__ void plan_host_words(uint32_t* host, uint32_t seq, uint32_t R, uint32_t mx, uint32_t slots)
{
    uint64_t* h = reinterpret_cast<uint64_t*>(host);
    const uint64_t tag = (uint64_t)seq << 32;
    h[0] = tag | R;
    h[1] = tag | mx;
    h[2] = tag | slots;
}

__global__ void __launch_bounds__(1024) k_plan(uint32_t* __restrict__ block_tot, int nb,
                                               const uint32_t* __restrict__ count, uint32_t* __restrict__ cursor,
                                               uint2* __restrict__ ranges, int T, uint32_t* __restrict__ misc,
                                               uint32_t* host, uint32_t seq, uint32_t flags)
{
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_max;
    if (threadIdx.x == 0) s_max = 0;
    PlanRun rb, rc;
    plan_load(block_tot, nb, rb);
    plan_load(count, T, rc);
    uint32_t mx = 0, unused = 0;
    const uint32_t slots = plan_scan(rb, s_w, unused, [&](int, uint32_t, uint32_t) {});  // the scatter sums its own base
    const uint32_t R = plan_scan(rc, s_w, mx, [&](int t, uint32_t ex, uint32_t c) {
        ranges[t] = make_uint2(ex, ex + c);
        if (cursor) cursor[t] = 0;  // only the atomic scatter (no histogram rows) hands out slots from cursors
    });
    for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off, 64));
    if ((threadIdx.x & 63) == 0) atomicMax(&s_max, mx);
    __syncthreads();
    if (threadIdx.x == 0) {
        misc[0] = R;
        misc[1] = s_max;
        misc[2] = slots;
        misc[kMiscPack] = flags & 1u;
        misc[kMiscDrop] = flags >> 1;
        // the host polls these words instead of putting an event (a queue barrier) here: three 64-bit words, each
        // carrying the frame's sequence number in its high half, written by single-copy-atomic stores, so the host
        // waits until all three carry it and the kernel needs no system-scope release to order them
        if (host) plan_host_words(host, seq, R, s_max, slots);
    }
}

// k_tile_offsets and k_plan in one launch (the default plan): each block turns its 32 tiles' histogram columns into
// block offsets as k_tile_offsets does, publishes its tiles' total and longest list in one 64-bit word (flags[b]:
// high half 1 << 31 | max, low half total; zeroed by k_count_tiles), and sums its predecessors' published totals for
// its ranges (a decoupled look-back: every block publishes before it waits, and blocks are dispatched in order, so a
// waiting block's predecessors are all running or done).  The last block, which sees every predecessor's word, also
// sums the count blocks' totals (record slots) and writes misc and the host words; the totals stay as they are (each
// scatter block sums its predecessors' for its base), so no block reads what another rewrites.  One launch and one
// dependent round trip instead of two launches, the second a single block.
//
// Every poll is bounded (`polls` sc1 loads per word, ~0.1 s by default), so a word that never arrives cannot hang the
// queue.  A block whose look-back times out sets misc[kMiscFail] before it counts itself done (misc[kMiscDone], a
// release increment after its ranges); the last block waits for every other block to be done, then reports R = ~0u if
// any block failed (or the wait itself timed out).  The host then re-plans the frame with the two launches that need no
// inter-block wait (k_tile_offsets + k_plan, capi.hip replan), and the render kernels queued behind the failed plan
// exit at once (Guard: R exceeds every capacity).  hlgs_set_plan_polls lowers the bound for the tests that force it.
template <int K>  // as k_tile_offsets
__global__ void __launch_bounds__(1024) k_tile_offsets_plan(uint32_t* __restrict__ hist, int nb, int T,
                                                            uint32_t* __restrict__ tile_count, uint2* __restrict__ ranges,
                                                            uint32_t* __restrict__ block_tot, uint64_t* flags,
                                                            uint32_t* misc, uint32_t* host, uint32_t seq, uint32_t fopts,
                                                            uint32_t polls)
{
    __shared__ uint32_t s_part[32][33];
    __shared__ uint32_t s_ex[32];
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_sum, s_max, s_agg, s_bmax, s_fail;
    const int c = threadIdx.x & 31, r = threadIdx.x >> 5;
    const int t = blockIdx.x * 32 + c;
    const int NB = (T + 31) / 32;
    const bool last = (int)blockIdx.x == NB - 1;
    const int run = (nb + 31) / 32, b0 = r * run, b1 = min(nb, b0 + run);
    uint32_t v[K];
    int rows[K];
    uint32_t sum = 0;
    if (threadIdx.x == 0) { s_sum = 0; s_max = 0; s_fail = 0; }
    if (t < T) {
        if (run <= K) {
            HistRows it(b0, nb);
#pragma unroll
            for (int k = 0; k < K; k++) {
                rows[k] = it.row();
                it.next();
            }
#pragma unroll
            for (int k = 0; k < K; k++) v[k] = b0 + k < b1 ? hist[(size_t)rows[k] * T + t] : 0u;
#pragma unroll
            for (int k = 0; k < K; k++) sum += v[k];
        } else {
            HistRows it(b0, nb);
            for (int b = b0; b < b1; b++, it.next()) sum += hist[(size_t)it.row() * T + t];
        }
    }
    s_part[r][c] = sum;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) {
        const uint32_t x = s_part[i][c];
        if (i < r) off += x;
        tot += x;
    }
    if (r == 0) s_ex[c] = t < T ? tot : 0u;  // the block's 32 tile totals
    __syncthreads();
    if (threadIdx.x == 0) {  // their exclusive prefix, total and longest list, published at once
        uint32_t x[32], a = 0, m = 0;
#pragma unroll
        for (int i = 0; i < 32; i++) x[i] = s_ex[i];
#pragma unroll
        for (int i = 0; i < 32; i++) {
            s_ex[i] = a;
            a += x[i];
            m = max(m, x[i]);
        }
        s_agg = a;
        s_bmax = m;
        __hip_atomic_store(&flags[blockIdx.x], ((uint64_t)(0x80000000u | m) << 32) | a, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (t < T) {
        if (run <= K) {
#pragma unroll
            for (int k = 0; k < K; k++)
                if (b0 + k < b1) {
                    hist[(size_t)rows[k] * T + t] = off;
                    off += v[k];
                }
        } else {
            HistRows it(b0, nb);
            for (int b = b0; b < b1; b++, it.next()) {
                uint32_t* h = hist + (size_t)it.row() * T + t;
                const uint32_t x = *h;
                *h = off;
                off += x;
            }
        }
        if (r == 0 && tile_count) tile_count[t] = tot;
    }
    uint32_t slots = 0;
    if (last) {  // the count blocks' totals summed (record slots), ahead of the look-back wait
        PlanRun rb;
        plan_load(block_tot, nb, rb);
        uint32_t unused = 0;
        slots = plan_scan(rb, s_w, unused, [&](int, uint32_t, uint32_t) {});
    }
    // look-back: thread i < blockIdx.x polls block i's word (sc1 loads, bounded)
    if ((int)threadIdx.x < (int)blockIdx.x) {
        uint64_t w = 0;
        for (uint32_t n = 0; n < polls; n++) {
            w = __hip_atomic_load(&flags[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (w >> 63) break;
            __builtin_amdgcn_s_sleep(2);
        }
        if (!(w >> 63)) s_fail = 1u;
        atomicAdd(&s_sum, (uint32_t)w);
        atomicMax(&s_max, (uint32_t)(w >> 32) & 0x7fffffffu);
    }
    __syncthreads();
    const uint32_t E = s_sum;
    if (r == 0 && t < T) ranges[t] = make_uint2(E + s_ex[c], E + s_ex[c] + tot);
    if (!last) {
        __syncthreads();  // the block's ranges are written
        if (threadIdx.x == 0) {
            if (s_fail) __hip_atomic_fetch_or(&misc[kMiscFail], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&misc[kMiscDone], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    if (threadIdx.x == 0) {  // misc and the host words (the scatter sums its own base)
        bool ok = !s_fail;
        uint32_t done = 0;
        for (uint32_t n = 0; ok && n < polls; n++) {  // every other block done (bounded)
            done = __hip_atomic_load(&misc[kMiscDone], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            if (done == (uint32_t)(NB - 1)) break;
            __builtin_amdgcn_s_sleep(2);
        }
        ok = ok && done == (uint32_t)(NB - 1) &&
             __hip_atomic_load(&misc[kMiscFail], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0u;
        // a failed look-back reports R = ~0u: the host re-plans the frame (k_tile_offsets + k_plan)
        const uint32_t R = ok ? E + s_agg : ~0u, mx = max(s_max, s_bmax);
        misc[0] = R;
        misc[1] = mx;
        misc[2] = slots;
        misc[kMiscPack] = fopts & 1u;
        misc[kMiscDrop] = fopts >> 1;
        if (host) plan_host_words(host, seq, R, mx, slots);
    }
}

// One thread per Gaussian: drop (depth, index) keys into each touched tile's segment.
__global__ void __launch_bounds__(256) k_scatter_keys(int P, const int* __restrict__ radii, Geom g,
                                                      const uint2* __restrict__ ranges, uint32_t* cursor,
                                                      uint64_t* __restrict__ keys, int gx, int gy, int alt, Guard gd,
                                                      int pack)
{
    if (guard_fail(gd)) return;
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= P || radii[idx] <= 0) return;
    const float2 xy = g.means2D[idx];
    const int2 ext = g.rects[idx];
    int x0, y0, x1, y1;
    tile_rect(xy.x, xy.y, ext.x, ext.y, gx, gy, x0, y0, x1, y1);
    uint32_t* __restrict__ ents = reinterpret_cast<uint32_t*>(keys);  // entries only, as k_scatter_keys_lds
    const float4 r0 = g.splat[4 * (size_t)idx], r1 = g.splat[4 * (size_t)idx + 1];
    const float4 co = make_float4(r0.z, r0.w, r1.x, r1.y);
    const AltKeep kthr = alt ? alt_keep_prep(co) : AltKeep{0.f, 0.f, 0.f};
    const uint32_t masks = pack ? g.qmask[idx] : 0u;
    uint32_t r = 0;
    for (int y = y0; y < y1; y++)
        for (int x = x0; x < x1; x++, r++) {
            if (alt && !alt_tile_keep(xy.x, xy.y, co, kthr, x, y)) continue;
            if (g.drop && !rect_tile_mask(masks, r)) continue;
            const int tile = y * gx + x;
            const uint32_t slot = atomicAdd(&cursor[tile], 1u);
            ents[ranges[tile].x + slot] = pack ? ((uint32_t)idx << kEntryShift) | rect_tile_mask(masks, r) : (uint32_t)idx;
        }
}

// The sort key of a binned entry: the Gaussian's depth bits above the entry (depths are positive, so their bits order
// as the floats do; the entry orders equal depths by Gaussian index, CUB's stable order, App. A-4).
struct KeySrc {
    const uint32_t* ents;  // the scatter's entries (the keys buffer's first 4 R bytes)
    const float* depths;   // Geom::depths
    int pack;              // entries carry quadrant masks (pack_entries): index = entry >> kEntryShift
    __device__ __forceinline__ uint64_t operator()(uint32_t p) const
    {
        const uint32_t e = ents[p];
        return ((uint64_t)depth_bits(e) << 32) | e;
    }
    __device__ __forceinline__ uint32_t depth_bits(uint32_t e) const
    {
        return __float_as_uint(depths[pack ? e >> kEntryShift : e]);
    }
};
// A tile's keys from position base on: the register sorts read all of a lane's entries first and then gather all of
// their depths, two rounds of independent loads (a per-key entry -> depth chain would wait once per key).
struct KeyView {
    KeySrc ks;
    uint32_t base;
    __device__ __forceinline__ uint32_t entry(uint32_t e) const { return ks.ents[base + e]; }
    __device__ __forceinline__ uint32_t depth_bits(uint32_t ent) const { return ks.depth_bits(ent); }
};

// One pass of M consecutive bitonic substages (distances step 2^(M-1) .. step) of stage kk on group g: the 2^M keys
// at base + t step (base = g with M zero bits inserted at step's bit), compare-exchanged in registers.
template <int M>
__device__ __forceinline__ void bitonic_group(uint64_t* s, uint32_t g, uint32_t step, uint32_t kk)
{
    const uint32_t low = step - 1u, base = ((g & ~low) << M) | (g & low);
    uint64_t v[1 << M];
#pragma unroll
    for (int t = 0; t < (1 << M); t++) v[t] = s[base + (uint32_t)t * step];
    const bool asc = (base & kk) == 0;
#pragma unroll
    for (int sub = 0; sub < M; sub++) {
        const int d = 1 << (M - 1 - sub);
#pragma unroll
        for (int t = 0; t < (1 << M); t++) {
            if (t & d) continue;
            const uint64_t x = v[t], y = v[t + d];
            const bool sw = (x > y) == asc;
            v[t] = sw ? y : x;
            v[t + d] = sw ? x : y;
        }
    }
#pragma unroll
    for (int t = 0; t < (1 << M); t++) s[base + (uint32_t)t * step] = v[t];
}

// One 256-thread block per tile: bitonic sort of the tile's keys in LDS.  Tiles longer than kSortCap
// are sorted in kSortCap runs here and merged by k_merge_runs.
__global__ void __launch_bounds__(256) k_tile_sort(const uint2* __restrict__ ranges, KeySrc ks, uint64_t* runs,
                                                   uint32_t* __restrict__ point_list, int T, Guard gd)
{
    if (guard_fail(gd)) return;
    __shared__ uint64_t s[kSortCap];
    const int tile = xcd_remap(blockIdx.x, T);
    const uint2 r = ranges[tile];
    const uint32_t cnt = r.y - r.x;
    if (cnt <= (uint32_t)kWaveSortCap) return;  // sorted by k_tile_sort_wave
    const int tid = threadIdx.x;
    const bool big = cnt > (uint32_t)kSortCap;
    for (uint32_t c0 = 0; c0 < cnt; c0 += kSortCap) {
        const uint32_t n = min((uint32_t)kSortCap, cnt - c0);
        uint32_t np = 2;
        while (np < n) np <<= 1;
        {  // all of a thread's entries, then all of their depths: two rounds of loads, not one chain per key
            constexpr int EPT = kSortCap / 256;
            uint32_t en[EPT], dp[EPT];
#pragma unroll
            for (int k = 0; k < EPT; k++) en[k] = ks.ents[r.x + c0 + min(tid + 256u * k, n - 1)];
#pragma unroll
            for (int k = 0; k < EPT; k++) dp[k] = ks.depth_bits(en[k]);
#pragma unroll
            for (int k = 0; k < EPT; k++) {
                const uint32_t i = tid + 256u * k;
                if (i < np) s[i] = i < n ? ((uint64_t)dp[k] << 32) | en[k] : ~0ull;
            }
        }
        __syncthreads();
        // Three substages per pass over the LDS (distances j, j/2, j/4): a thread loads the 8 keys those substages
        // connect, runs the 12 compare-exchanges in registers and stores the 8 back, a third of the LDS traffic and
        // barriers of one substage per pass.  Passes whose largest distance j is below the quarter seg = np / 4 stay
        // inside one wave's quarter of the array (their 2j-blocks are aligned in it): each wave runs its own quarter's
        // groups with no block barrier, its own LDS order (lgkmcnt(0)) separating the passes.
        const uint32_t seg = np >> 2, wv = (uint32_t)(tid >> 6), ln = (uint32_t)(tid & 63);
        for (uint32_t kk = 2; kk <= np; kk <<= 1)
            for (uint32_t j = kk >> 1; j > 0;) {
                const int m = min(3, 32 - __clz(j));  // substages in this pass (j = 1 or 2 leaves fewer)
                const uint32_t step = j >> (m - 1), ng = np >> m;
                auto pass = [&](uint32_t g) {
                    if (m == 3) bitonic_group<3>(s, g, step, kk);
                    else if (m == 2) bitonic_group<2>(s, g, step, kk);
                    else bitonic_group<1>(s, g, step, kk);
                };
                if (j >= seg) {  // block-uniform
                    __syncthreads();
                    for (uint32_t g = tid; g < ng; g += 256) pass(g);
                    __syncthreads();
                } else {
                    const uint32_t gpw = seg >> m, g0 = wv * gpw;
                    for (uint32_t g = g0 + ln; g < g0 + gpw; g += 64) pass(g);
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                }
                j >>= m;
            }
        __syncthreads();
        if (big)  // sorted runs into the second key buffer (the entries of other tiles still occupy the first)
            for (uint32_t i = tid; i < n; i += 256) runs[r.x + c0 + i] = s[i];
        else
            for (uint32_t i = tid; i < n; i += 256) point_list[r.x + c0 + i] = (uint32_t)s[i];
        __syncthreads();
    }
}

// {a, b} = {x, x of lane l ^ PL} (in either order) for a 64-bit key, without the LDS: DPP within 16-lane rows for
// PL = 1, 2 (quad_perm), 4 (row_ror:12 into banks 0 and 2, row_ror:4 into banks 1 and 3; row_ror:n reads lane l - n
// of the row) and 8 (row_ror:8); permlane16 / permlane32 swaps of two copies for 16 and 32, which leave each lane its
// own value in one register and its partner's in the other.  A compare-exchange only needs the pair's min and max, so
// the order does not matter.  (ds_bpermute, which __shfl_xor compiles to, is an LDS round trip per 32-bit half.)
template <int PL>
__device__ __forceinline__ void lane_pair64(uint64_t x, uint64_t& a, uint64_t& b)
{
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    if constexpr (PL == 16 || PL == 32) {
        const auto l = PL == 16 ? __builtin_amdgcn_permlane16_swap(lo, lo, false, false)
                                : __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        const auto h = PL == 16 ? __builtin_amdgcn_permlane16_swap(hi, hi, false, false)
                                : __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        a = ((uint64_t)h[0] << 32) | l[0];
        b = ((uint64_t)h[1] << 32) | l[1];
    } else {
        auto mv = [](uint32_t v) -> uint32_t {
            if constexpr (PL == 1) return __builtin_amdgcn_update_dpp(0u, v, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
            if constexpr (PL == 2) return __builtin_amdgcn_update_dpp(0u, v, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
            if constexpr (PL == 8) return __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xF, 0xF, false);  // row_ror:8
            const uint32_t t = __builtin_amdgcn_update_dpp(0u, v, 0x12C, 0xF, 0x5, false);            // row_ror:12
            return __builtin_amdgcn_update_dpp(t, v, 0x124, 0xF, 0xA, false);                          // row_ror:4
        };
        a = x;
        b = ((uint64_t)mv(hi) << 32) | mv(lo);
    }
}
template <int PL>
__device__ __forceinline__ uint64_t lane_cx64(uint64_t x, bool take_min)
{
    uint64_t a, b;
    lane_pair64<PL>(x, a, b);
    return ((a < b) == take_min) ? a : b;
}

// Per-tile sort of 64 * KPL keys by one wave, entirely in registers (~0 pads): afterwards lane l's slot i holds sorted
// position l * KPL + i.  Bitonic stages with partner distance < KPL are compare-exchanges inside a lane, longer ones
// exchange with lane l ^ (j / KPL) (lane_pair64).  No LDS, no barriers.  The keys may start in any lanes and slots.
template <int KPL>
__device__ __forceinline__ void wave_sort_regs(uint64_t (&v)[KPL], int lane)
{
    constexpr uint32_t NP = 64u * KPL;
#pragma unroll
    for (uint32_t kk = 2; kk <= NP; kk <<= 1) {
#pragma unroll
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
            if (j >= (uint32_t)KPL) {
                const int pl = (int)(j / KPL);
                const bool lower = (lane & pl) == 0;
#pragma unroll
                for (int i = 0; i < KPL; i++) {
                    const uint32_t e = (uint32_t)lane * KPL + i;
                    const bool asc = (e & kk) == 0;
                    const bool take_min = lower == asc;
                    switch (pl) {  // a constant once the stages are unrolled
                    case 1: v[i] = lane_cx64<1>(v[i], take_min); break;
                    case 2: v[i] = lane_cx64<2>(v[i], take_min); break;
                    case 4: v[i] = lane_cx64<4>(v[i], take_min); break;
                    case 8: v[i] = lane_cx64<8>(v[i], take_min); break;
                    case 16: v[i] = lane_cx64<16>(v[i], take_min); break;
                    default: v[i] = lane_cx64<32>(v[i], take_min); break;
                    }
                }
            } else {
#pragma unroll
                for (int i = 0; i < KPL; i++) {
                    if (i & j) continue;
                    const int k = i | (int)j;
                    const uint32_t e = (uint32_t)lane * KPL + i;
                    const bool asc = (e & kk) == 0;
                    const uint64_t x = v[i], y = v[k];
                    const bool sw = (x > y) == asc;
                    v[i] = sw ? y : x;
                    v[k] = sw ? x : y;
                }
            }
        }
    }
}
// Keys l + 64 i (i < K, the ones below n) of the tile segment at base into v[i] of lane l: all of the lane's entries
// are loaded first, then all of their depths (two rounds of independent loads, not an entry -> depth chain per key).
// Consecutive lanes read consecutive entries.
template <int K>
__device__ __forceinline__ void wave_keys_load(const KeySrc& ks, uint32_t base, uint32_t n, uint64_t (&v)[K], int lane)
{
    uint32_t en[K], dp[K];
#pragma unroll
    for (int i = 0; i < K; i++) en[i] = ks.ents[base + min((uint32_t)lane + 64u * i, n - 1)];  // n >= 1
#pragma unroll
    for (int i = 0; i < K; i++) dp[i] = ks.depth_bits(en[i]);
#pragma unroll
    for (int i = 0; i < K; i++) v[i] = (uint32_t)lane + 64u * i < n ? ((uint64_t)dp[i] << 32) | en[i] : ~0ull;
}
// The first K slots of v sorted as 64 K keys (the ones from the strided load that reach m), stored by st(e, key) for e < m.
template <int K, int KMAX, typename ST>
__device__ __forceinline__ void wave_sort_first(const uint64_t (&v)[KMAX], uint32_t m, ST&& st, int lane)
{
    uint64_t w[K];
#pragma unroll
    for (int i = 0; i < K; i++) w[i] = v[i];
    wave_sort_regs<K>(w, lane);
#pragma unroll
    for (int i = 0; i < K; i++) {
        const uint32_t e = (uint32_t)lane * K + i;
        if (e < m) st(e, w[i]);
    }
}
// n in (64 KH, 128 KH]: the first A = 64 KH keys sorted with KH keys per lane and the other m = n - A with the fewest
// that hold them, both into LDS, then merged -- each lane finds the start of its run of ceil(n / 64) outputs on the
// merge path (binary search) and merges the run.  A 300-key tile then costs a 256-key and a 64-key register sort
// instead of a 512-key one (the mean configs[1] list is 258 keys).  Both runs' keys are loaded before either is
// sorted, so the wave waits for the entries and the depths once.  Keys are unique, so the merge is the same total order.
template <int KH>
__device__ __forceinline__ void wave_sort_split(const KeySrc& ks, uint32_t base, uint32_t n,
                                                uint32_t* __restrict__ out, int lane, uint64_t* s)
{
    constexpr uint32_t A = 64u * KH;
    const uint32_t m = n - A;  // 1 .. A
    uint64_t va[KH], vb[KH];
    {
        uint32_t ea[KH], eb[KH], da[KH], db[KH];
#pragma unroll
        for (int i = 0; i < KH; i++) ea[i] = ks.ents[base + lane + 64u * i];
#pragma unroll
        for (int i = 0; i < KH; i++) eb[i] = ks.ents[base + A + min((uint32_t)lane + 64u * i, m - 1)];
#pragma unroll
        for (int i = 0; i < KH; i++) da[i] = ks.depth_bits(ea[i]);
#pragma unroll
        for (int i = 0; i < KH; i++) db[i] = ks.depth_bits(eb[i]);
#pragma unroll
        for (int i = 0; i < KH; i++) {
            va[i] = ((uint64_t)da[i] << 32) | ea[i];
            vb[i] = (uint32_t)lane + 64u * i < m ? ((uint64_t)db[i] << 32) | eb[i] : ~0ull;
        }
    }
    wave_sort_regs<KH>(va, lane);
#pragma unroll
    for (int i = 0; i < KH; i++) s[(uint32_t)lane * KH + i] = va[i];
    auto stb = [&](uint32_t e, uint64_t v) { s[A + e] = v; };
    if (m <= 64) wave_sort_first<1>(vb, m, stb, lane);
    else if constexpr (KH >= 2) {
        if (m <= 128) wave_sort_first<2>(vb, m, stb, lane);
        else if constexpr (KH >= 4) {
            if (m <= 256) wave_sort_first<4>(vb, m, stb, lane);
            else if constexpr (KH >= 8) wave_sort_first<8>(vb, m, stb, lane);
        }
    }
    __syncthreads();  // one wave: the LDS stores before the loads
    const uint32_t per = (n + 63u) / 64u, k0 = min(n, (uint32_t)lane * per), k1 = min(n, k0 + per);
    uint32_t lo = k0 > m ? k0 - m : 0u, hi = min(k0, A);  // A keys among the first k0 outputs
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s[mid] < s[A + (k0 - mid - 1)]) lo = mid + 1;
        else hi = mid;
    }
    uint32_t i = lo, j = k0 - lo;
    for (uint32_t k = k0; k < k1; k++) {
        const bool takeA = j >= m || (i < A && s[i] < s[A + j]);
        const uint64_t v = takeA ? s[i] : s[A + j];
        out[base + k] = (uint32_t)v;
        if (takeA) i++;
        else j++;
    }
}
// Tiles of up to kWaveSortCap instances: one wave each (k_tile_sort handles the longer ones).
__global__ void __launch_bounds__(64) k_tile_sort_wave(const uint2* __restrict__ ranges, KeySrc ks,
                                                       uint32_t* __restrict__ point_list, int T, Guard gd)
{
    if (guard_fail(gd)) return;
    const int tile = xcd_remap(blockIdx.x, T);
    const uint2 r = ranges[tile];
    const uint32_t n = r.y - r.x;
    const int lane = threadIdx.x;
    if (n == 0 || n > (uint32_t)kWaveSortCap) return;
    __shared__ uint64_t s_sort[kWaveSortCap + 1];  // + 1: the merge may read one past the second run
    if (n <= 64) {
        uint64_t v[1];
        wave_keys_load<1>(ks, r.x, n, v, lane);
        wave_sort_regs<1>(v, lane);
        if ((uint32_t)lane < n) point_list[r.x + lane] = (uint32_t)v[0];
    }
    else if (n <= 128) wave_sort_split<1>(ks, r.x, n, point_list, lane, s_sort);
    else if (n <= 256) wave_sort_split<2>(ks, r.x, n, point_list, lane, s_sort);
    else if (n <= 512) wave_sort_split<4>(ks, r.x, n, point_list, lane, s_sort);
    else wave_sort_split<8>(ks, r.x, n, point_list, lane, s_sort);
}

// Merge pass for long tiles: element of run r finds its rank in the partner run by binary search.
__global__ void __launch_bounds__(256) k_merge_runs(const uint2* __restrict__ ranges, const uint64_t* __restrict__ src,
                                                    uint64_t* __restrict__ dst, uint32_t* __restrict__ point_list,
                                                    uint32_t L, int last)
{
    const int tile = blockIdx.y;
    const uint2 r = ranges[tile];
    const uint32_t cnt = r.y - r.x;
    if (cnt <= (uint32_t)kSortCap) return;
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= cnt) return;
    const uint64_t key = src[r.x + i];
    const uint32_t run = i / L, a = i - run * L;
    const uint32_t prun = run ^ 1u;
    uint32_t out = i;
    const uint64_t pstart64 = (uint64_t)prun * L;
    if (pstart64 < cnt) {
        const uint32_t ps = (uint32_t)pstart64, pe = min(cnt, ps + L);
        uint32_t lo = ps, hi = pe;  // count partner keys < key (keys are unique)
        while (lo < hi) {
            uint32_t mid = (lo + hi) >> 1;
            if (src[r.x + mid] < key) lo = mid + 1; else hi = mid;
        }
        out = min(run, prun) * L + a + (lo - ps);
    }
    dst[r.x + out] = key;
    if (last) point_list[r.x + out] = (uint32_t)key;
}

struct FwdArgs {
    const uint2* ranges;
    const uint32_t* point_list;
    int W, H, gx, T;
    const float4* splat;
    float* final_T;
    uint32_t* n_contrib;
    const float* bg;
    float* out_color;
    float* out_invdepth;
    int* seen;
    float* split_state;  // Img::split_state (null: not sampled)
    int pack;            // point_list entries are packed (pack_entries)
};

// ------------------------------------------------------------------------------------------------
// Front-to-back blend.  One wave64 per 8x8 quadrant of a 16x16 tile, one pixel per lane; the four
// quadrant waves of a tile are independent blocks placed on one XCD (xcd_remap) so the tile's splat
// reads hit the same L2.  Each 64-splat batch is staged in LDS; a ballot builds the wave-uniform bit
// set of the batch's splats whose alpha >= 1/255 footprint reaches this quadrant, and only those are
// visited (scalar find-first-set loop).  Skipped pairs are exactly the ones the reference discards.
// Round 5 measured per-row 4x4 sub-block lists instead (raster_fwd_sub4.hip, tools/variants/INDEX.md): a third fewer
// iterations, but 209 against 151 us -- per-lane LDS addresses and the row bookkeeping cost more VALU than the
// iterations saved.
// ------------------------------------------------------------------------------------------------
template <bool INTERP, bool DEPTH, bool SEEN>  // SEEN: A.seen is set (the per-splat mask is only kept then)
__global__ void __launch_bounds__(64) k_blend_fwd(FwdArgs A, Guard gd)
{
    if (guard_fail(gd)) return;
    __shared__ float4 s_xy[64];   // x, y, 1/depth, alpha threshold on e2
    __shared__ float4 s_co[64];   // conic_q, opacity
    __shared__ float4 s_col[64];  // r, g, b, 1/kids (hierarchy mode) or 1-based list position
    __shared__ float s_t[64];     // interpolation t
    const int L = xcd_remap(blockIdx.x, 4 * A.T);
    const int tile = L >> 2, q = L & 3;
    const int lane = threadIdx.x;
    const int qx0 = (tile % A.gx) * HLGS_TILE + 8 * (q & 1), qy0 = (tile / A.gx) * HLGS_TILE + 8 * (q >> 1);
    const int px = qx0 + (lane & 7), py = qy0 + (lane >> 3);
    const float pxf = (float)px, pyf = (float)py;
    const float fqx = (float)qx0, fqy = (float)qy0;
    const uint2 range = A.ranges[tile];

    float Tt = 1.0f, C0 = 0.f, C1 = 0.f, C2 = 0.f, D = 0.f;
    uint32_t last = 0;
    // Backward chunk boundaries (bwd_chunk_len): at each, the transmittance is stored at once and the colour /
    // inverse depth blended so far is kept, so that the end can store what was blended behind the boundary.
    const uint32_t clen = bwd_chunk_len(range.y - range.x);
    float* st = A.split_state ? A.split_state + (size_t)tile * kBwdSplits * kSplitFloats + q * 5 * 64 + lane : nullptr;
    uint32_t next_split = range.x + clen, nsplit = 0;
    float S0[kBwdSplits][4];
    // per-lane predicates are kept as wave masks (the wave is always full): compares are ballots of one v_cmp
    // each, their combinations scalar mask operations, and selects read them back with inverse_ballot
    uint64_t done = __builtin_amdgcn_ballot_w64(!(px < A.W && py < A.H));
    // Software pipeline over batches: while batch b is blended, the records of batch b+1 and the list entries of
    // batch b+2 are in flight.  Every lane issues every load (a lane with nothing to stage reads record 0, a lane
    // past the list end re-reads the list's last entry), so the loads retire in a fixed order and the wait at the top
    // of a batch is for the records alone, not for everything in flight as after a branch round a load.
    const bool any = range.x < range.y;  // wave-uniform
    const uint32_t lastpos = any ? range.y - 1 : range.x;
    auto entry_at = [&](uint32_t p) -> uint32_t { return any ? A.point_list[p < range.y ? p : lastpos] : 0u; };
    auto decode = [&](uint32_t e, uint32_t p, uint32_t& id) -> bool {
        bool s = p < range.y;
        if (A.pack) {
            s = s && ((e >> q) & 1u);
            e >>= kEntryShift;
        }
        id = e;
        return s;
    };
    uint32_t cur_id, nxt_entry = entry_at(range.x + 64 + lane);
    bool cur_stage = decode(entry_at(range.x + lane), range.x + lane, cur_id);
    float4 R0, R1, R2, R3;
    {
        const float4* rec = A.splat + 4 * (size_t)(cur_stage ? cur_id : 0u);
        R0 = rec[0]; R1 = rec[1]; R2 = rec[2]; R3 = rec[3];
    }
    for (uint32_t base = range.x; base < range.y; base += 64) {
        if (done == ~0ull) break;
        if (base == next_split && st) {  // wave-uniform; never past kBwdSplits boundaries (bwd_chunk_len)
            st[nsplit * kSplitFloats] = Tt;
#pragma unroll
            for (int k = 0; k < kBwdSplits; k++)
                if (k == (int)nsplit) { S0[k][0] = C0; S0[k][1] = C1; S0[k][2] = C2; S0[k][3] = D; }
            nsplit++;
            next_split += clen;
        }
        const uint32_t pos = base + lane;
        uint32_t my_id = 0;
        bool hit = false;
        {
            my_id = cur_id;
            const float4 co = make_float4(R0.z, R0.w, R1.x, R1.y);
            // packed entries (pack_entries) carry the quadrant mask: only the splats reaching this quadrant are staged
            hit = cur_stage && (A.pack || touches_quad(R0.x, R0.y, co, R3.w, fqx, fqy));
            // unconditional: lanes that stage nothing write slots no lane visits
            s_xy[lane] = make_float4(R0.x, R0.y, DEPTH ? R2.y : 0.f, R3.w);
            s_co[lane] = conic_q(co);
            // .w: 1/kids in hierarchy mode, otherwise the splat's 1-based position in the tile list (n_contrib value)
            s_col[lane] = make_float4(R1.z, R1.w, R2.x, INTERP ? R2.w : __uint_as_float(base - range.x + lane + 1));
            if (INTERP) s_t[lane] = R2.z;
            cur_stage = decode(nxt_entry, pos + 64, cur_id);
            const float4* rec = A.splat + 4 * (size_t)(cur_stage ? cur_id : 0u);
            R0 = rec[0]; R1 = rec[1]; R2 = rec[2]; R3 = rec[3];
            nxt_entry = entry_at(pos + 128);
        }
        uint64_t todo = __ballot(hit);
        __syncthreads();
        uint64_t seen_mask = 0;
        // Two visited splats per iteration: their falloffs, exponentials and alphas are independent of the pixel
        // state, so both chains are in flight together; only the short transmittance / colour updates run in list
        // order (the second sees the first's Tt and done).
        auto front = [&](int j, float& e2, float& alpha) {
            const float4 xy = s_xy[j];
            const float4 co = s_co[j];
            e2 = splat_e2(co, xy.x - pxf, xy.y - pyf);  // power * log2(e)
            const float my_alpha = fminf(0.99f, co.w * __builtin_amdgcn_exp2f(e2));
            alpha = my_alpha;
            if (INTERP) {
                const float tt = s_t[j];
                alpha = tt * my_alpha + (1.0f - tt) * (1.0f - __powf(1.0f - my_alpha, s_col[j].w));
            }
        };
        auto back = [&](int j, float e2, float alpha) {
            const float4 xy = s_xy[j];
            const float4 c = s_col[j];
            const float test_T = Tt * (1 - alpha);
            // alpha >= 1/255 (alpha_e2_threshold); a NaN e2 passes both tests, as in the reference
            const uint64_t valid = ~done & ~__builtin_amdgcn_ballot_w64(e2 > 0.0f) & ~__builtin_amdgcn_ballot_w64(e2 < xy.w);
            const uint64_t tlow = __builtin_amdgcn_ballot_w64(test_T < 0.0001f);
            const uint64_t blended = valid & ~tlow;
            done |= valid & tlow;  // the pixel stops; this splat is not blended into it
            const bool bl = __builtin_amdgcn_inverse_ballot_w64(blended);
            const float wgt = bl ? alpha * Tt : 0.f;
            C0 = fmaf(c.x, wgt, C0);
            C1 = fmaf(c.y, wgt, C1);
            C2 = fmaf(c.z, wgt, C2);
            if (DEPTH) D = fmaf(xy.z, wgt, D);
            Tt = bl ? test_T : Tt;
            last = bl ? (INTERP ? base - range.x + (uint32_t)j + 1 : __float_as_uint(c.w)) : last;
            if (SEEN && blended) seen_mask |= 1ull << j;
        };
        if (__builtin_popcountll(todo) & 1) {  // an odd count: the first splat alone, then pairs in list order
            int j;  // find-first-set and clear it: two SALU instead of four
            asm("s_ff1_i32_b64 %0, %1\n\ts_bitset0_b64 %1, %0" : "=&s"(j), "+s"(todo));
            float e2a, aa;
            front(j, e2a, aa);
            back(j, e2a, aa);
        }
        while (todo) {
            int j, k;
            asm("s_ff1_i32_b64 %0, %1\n\ts_bitset0_b64 %1, %0" : "=&s"(j), "+s"(todo));
            asm("s_ff1_i32_b64 %0, %1\n\ts_bitset0_b64 %1, %0" : "=&s"(k), "+s"(todo));
            float e2a, aa, e2b, ab;
            front(j, e2a, aa);
            front(k, e2b, ab);
            back(j, e2a, aa);
            back(k, e2b, ab);
        }
        if (SEEN && ((seen_mask >> lane) & 1ull)) A.seen[my_id] = 1;
        __syncthreads();
    }
    if (px < A.W && py < A.H) {
        const size_t HW = (size_t)A.H * A.W;
        const size_t pid = (size_t)A.W * py + px;
        A.final_T[pid] = Tt;
        A.n_contrib[pid] = last;
        A.out_color[pid] = C0 + Tt * A.bg[0];
        A.out_color[HW + pid] = C1 + Tt * A.bg[1];
        A.out_color[2 * HW + pid] = C2 + Tt * A.bg[2];
        if (DEPTH) A.out_invdepth[pid] = D;
    }
#pragma unroll
    for (int k = 0; k < kBwdSplits; k++)
        if (k < (int)nsplit) {
            float* sk = st + k * kSplitFloats;
            sk[64] = C0 - S0[k][0];
            sk[128] = C1 - S0[k][1];
            sk[192] = C2 - S0[k][2];
            if (DEPTH) sk[256] = D - S0[k][3];
        }
}

// rasterizer_impl.cu:54-66 with auxiliary.h:164-189 (prefiltered = false)
__global__ void __launch_bounds__(256) k_mark_visible(int P, const float* __restrict__ means, const float* view,
                                                      uint8_t* __restrict__ present)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    const f3 p = mk(means[3 * i], means[3 * i + 1], means[3 * i + 2]);
    present[i] = !(xform43(p, view).z <= 0.2f);
}

// utils.cu:6-36 (MCMC relocation, eq. 9 of 3DGS-as-MCMC)
__global__ void __launch_bounds__(256) k_relocation(int P, const float* __restrict__ op_old, const float* __restrict__ sc_old,
                                                    const int* __restrict__ N, const float* __restrict__ binoms,
                                                    int n_max, float* __restrict__ op_new, float* __restrict__ sc_new)
{
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= P) return;
    const int n = N[idx];
    float denom = 0.0f;
    const float on = 1.0f - powf(1.0f - op_old[idx], 1.0f / n);
    op_new[idx] = on;
    for (int i = 1; i <= n; ++i)
        for (int k = 0; k <= i - 1; ++k) {
            const float b = binoms[(i - 1) * n_max + k];
            const float term = (float)(((k & 1) ? -1.0 : 1.0) / sqrt((double)(k + 1)) * pow((double)on, k + 1));
            denom += b * term;
        }
    const float coeff = op_old[idx] / denom;
    for (int i = 0; i < 3; ++i) sc_new[3 * idx + i] = coeff * sc_old[3 * idx + i];
}

// ------------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------------
// LDS-histogram binning with the one-block plan: tile grids up to kBinMaxTiles and up to kPlanRun * 1024 blocks of
// bin_gauss(P) Gaussians (67M); anything larger takes the generic per-Gaussian path.
// Gaussians per binning block: 4,096, or 1,024 when 4,096 would leave fewer than ~200 blocks for the 256 CUs.  The
// switch sits at 768 blocks of 1,024 (786,432 Gaussians), the most the register runs of k_tile_offsets<24> /
// k_tile_offsets_plan<24> hold (ceil(nb / 32) <= 24); above it 4,096 gives >= 193 blocks (at 200 x 4,096
// the frames of 786,433-819,199 Gaussians took the serial per-row fallback).
int bin_gauss(int P) { return P > 768 * 1024 ? 4096 : 1024; }

bool lds_binning(int P, int gx, int gy)
{
    return gx * gy <= kBinMaxTiles && (long)(P + bin_gauss(P) - 1) / bin_gauss(P) <= (long)kPlanRun * 1024;
}

// Dynamic LDS above 64 KiB must be opted into per kernel (idempotent; done once per process).
static void allow_big_lds()
{
    static bool done = false;
    if (done) return;
    // the kernels' static LDS (the block's rect prefix, ~16 KiB) comes out of the same 160 KiB
    const int dyn = 2 * (int)sizeof(uint32_t) * kBinMaxTiles;
    const hipFuncAttribute A = hipFuncAttributeMaxDynamicSharedMemorySize;
#define HLGS_BIG(...) (void)hipFuncSetAttribute((const void*)__VA_ARGS__, A, dyn)
    HLGS_BIG(k_count_tiles<4096, false>); HLGS_BIG(k_count_tiles<1024, false>);
    HLGS_BIG(k_count_tiles<4096, true>); HLGS_BIG(k_count_tiles<1024, true>);
    HLGS_BIG(k_scatter_keys_lds<4096, true>); HLGS_BIG(k_scatter_keys_lds<1024, true>);
    HLGS_BIG(k_scatter_keys_lds<4096, false>); HLGS_BIG(k_scatter_keys_lds<1024, false>);
#undef HLGS_BIG
    hipGetLastError();
    done = true;
}

// Scratch for the count blocks' histogram rows: the image buffer's split state (written only later, by the forward
// blend), when nb x T words fit in it; nullptr -> the device-atomic binning.
uint32_t* bin_histogram(const Img& im, int P, int gx, int gy)
{
    const size_t T = (size_t)gx * gy, nb = (size_t)(P + bin_gauss(P) - 1) / bin_gauss(P);
    if (lds_binning(P, gx, gy) && nb * T <= T * kBwdSplits * (size_t)kSplitFloats)
        return reinterpret_cast<uint32_t*>(im.split_state);
    return nullptr;
}

// The fused plan's look-back words live in the tile cursors (unused by the histogram binning): ceil(T / 32) 64-bit
// words, within the cursors' align_up(4 T) bytes for every T >= 1.
static uint64_t* plan_flags(const Img& im) { return reinterpret_cast<uint64_t*>(im.tile_cursor); }
// fused: the plan that follows is k_tile_offsets_plan (it needs its look-back words cleared); otherwise, with histogram
// rows, k_tile_offsets runs here and k_plan after it (the re-plan of a frame whose fused plan failed, capi.hip).
void launch_count_tiles(int P, const int* radii, const Geom& g, const Img& im, int gx, int gy, bool alt,
                        hipStream_t s, uint32_t* hist, bool fused)
{
    const int T = gx * gy;
    const size_t lds = sizeof(uint32_t) * (size_t)T;
    allow_big_lds();
    const int bg = bin_gauss(P);
    fused = fused && hist;
    uint32_t* zw = fused ? im.tile_cursor : nullptr;
    const int nz = fused ? 2 * ((T + 31) / 32) : 0;
#define HLGS_CNT(BG, D) hipLaunchKernelGGL((k_count_tiles<BG, D>), dim3((P + BG - 1) / BG), dim3(1024), lds, s, P, \
                                          radii, g, im.tile_count, gx, gy, (int)alt, g.scan_tmp, hist, zw, nz, im.misc)
    if (bg == 4096) { if (g.drop) HLGS_CNT(4096, true); else HLGS_CNT(4096, false); }
    else { if (g.drop) HLGS_CNT(1024, true); else HLGS_CNT(1024, false); }
#undef HLGS_CNT
    if (hist && !fused) {
        const int nb = (P + bg - 1) / bg;
        if (nb <= 32 * 8) hipLaunchKernelGGL(k_tile_offsets<8>, dim3((T + 31) / 32), dim3(1024), 0, s, hist, nb, T, im.tile_count);
        else hipLaunchKernelGGL(k_tile_offsets<24>, dim3((T + 31) / 32), dim3(1024), 0, s, hist, nb, T, im.tile_count);
    }
}

void launch_plan(int P, const Geom& g, const Img& im, int gx, int gy, uint32_t* host, uint32_t seq, hipStream_t s,
                 bool fused)
{
    const int T = gx * gy;
    static_assert(kPlanRun * 1024 >= kBinMaxTiles, "one k_plan block covers every LDS-binned tile grid");
    uint32_t* hist = bin_histogram(im, P, gx, gy);
    const int nb = (P + bin_gauss(P) - 1) / bin_gauss(P);
    if (hist && fused) {
        if (nb <= 32 * 8)
            hipLaunchKernelGGL(k_tile_offsets_plan<8>, dim3((T + 31) / 32), dim3(1024), 0, s, hist, nb, T, im.tile_count,
                               im.ranges, g.scan_tmp, plan_flags(im), im.misc, host, seq, FrameOpts{g.pack, g.drop, 0}.flags(), g.polls);
        else
            hipLaunchKernelGGL(k_tile_offsets_plan<24>, dim3((T + 31) / 32), dim3(1024), 0, s, hist, nb, T, im.tile_count,
                               im.ranges, g.scan_tmp, plan_flags(im), im.misc, host, seq, FrameOpts{g.pack, g.drop, 0}.flags(), g.polls);
        return;
    }
    uint32_t* cursor = hist ? nullptr : im.tile_cursor;
    hipLaunchKernelGGL(k_plan, dim3(1), dim3(1024), 0, s, g.scan_tmp, nb, im.tile_count, cursor, im.ranges, T, im.misc,
                       host, seq, FrameOpts{g.pack, g.drop, 0}.flags());
}

void launch_tile_ranges(const Img& im, int T, const uint32_t* point_offsets, int P, uint32_t flags, hipStream_t s)
{
    hipLaunchKernelGGL(k_tile_ranges, dim3((T + 255) / 256), dim3(256), 0, s, im.tile_count, im.tile_cursor,
                       im.ranges, im.misc, T, point_offsets, P, flags);
}

void launch_binning(const hlgs_raster_args& a, const int* radii, const Geom& g, const Img& im, const Bin& b,
                    int gx, int gy, uint32_t max_count, hipStream_t s, bool timing, Guard gd)
{
    const int T = gx * gy;
    const int alt = a.variant == HLGS_VARIANT_ALT;
    if (timing) stage_mark(s, 3, true);
    if (lds_binning(a.P, gx, gy)) {
        allow_big_lds();
#define HLGS_SCATTER(BG, PK)                                                                                       \
    hipLaunchKernelGGL((k_scatter_keys_lds<BG, PK>), dim3((a.P + BG - 1) / BG), dim3(1024),                           \
                       2 * sizeof(uint32_t) * (size_t)T, s, a.P, radii, g, im.ranges, im.tile_cursor, b.keys, gx, gy, alt, \
                       gd, g.scan_tmp, bin_histogram(im, a.P, gx, gy))
        const bool pk = g.pack;
        if (bin_gauss(a.P) == 4096) { if (pk) HLGS_SCATTER(4096, true); else HLGS_SCATTER(4096, false); }
        else { if (pk) HLGS_SCATTER(1024, true); else HLGS_SCATTER(1024, false); }
#undef HLGS_SCATTER
    } else
        hipLaunchKernelGGL(k_scatter_keys, dim3((a.P + 255) / 256), dim3(256), 0, s, a.P, radii, g, im.ranges,
                           im.tile_cursor, b.keys, gx, gy, alt, gd, g.pack);
    if (timing) { stage_mark(s, 3, false); stage_mark(s, 4, true); }
    const KeySrc ks{reinterpret_cast<const uint32_t*>(b.keys), g.depths, g.pack};
    hipLaunchKernelGGL(k_tile_sort_wave, dim3(T), dim3(64), 0, s, im.ranges, ks, b.point_list, T, gd);
    if (max_count > (uint32_t)kWaveSortCap)
        hipLaunchKernelGGL(k_tile_sort, dim3(T), dim3(256), 0, s, im.ranges, ks, b.keys2, b.point_list, T, gd);
    if (max_count > (uint32_t)kSortCap) {  // the runs are in keys2; every entry has been read by now
        uint64_t* src = b.keys2;
        uint64_t* dst = b.keys;
        for (uint32_t L = kSortCap; L < max_count; L <<= 1) {
            const int last = (L << 1) >= max_count;
            hipLaunchKernelGGL(k_merge_runs, dim3((max_count + 255) / 256, T), dim3(256), 0, s, im.ranges, src, dst,
                               b.point_list, L, last);
            uint64_t* t = src; src = dst; dst = t;
        }
    }
    if (timing) stage_mark(s, 4, false);
}

void launch_blend_fwd(const hlgs_raster_args& a, const Geom& g, const Img& im, const Bin& b, int gx, int gy,
                      float* out_color, float* out_invdepth, int* seen, hipStream_t s, Guard gd)
{
    const int T = gx * gy;
    const bool interp = a.ts != nullptr && a.kids != nullptr;
    const bool depth = out_invdepth != nullptr;
    FwdArgs A{im.ranges, b.point_list, a.W, a.H, gx, T, g.splat, im.final_T, im.n_contrib, a.bg, out_color,
              out_invdepth, seen, im.split_state, g.pack};
#define HLGS_BLEND(I, Dp)                                                                                         \
    do {                                                                                                          \
        if (seen) hipLaunchKernelGGL((k_blend_fwd<I, Dp, true>), dim3(4 * T), dim3(64), 0, s, A, gd);           \
        else hipLaunchKernelGGL((k_blend_fwd<I, Dp, false>), dim3(4 * T), dim3(64), 0, s, A, gd);               \
    } while (0)
    if (interp) { if (depth) HLGS_BLEND(true, true); else HLGS_BLEND(true, false); }
    else { if (depth) HLGS_BLEND(false, true); else HLGS_BLEND(false, false); }
#undef HLGS_BLEND
}

void launch_mark_visible(int P, const float* means, const float* view, uint8_t* present, hipStream_t s)
{
    hipLaunchKernelGGL(k_mark_visible, dim3((P + 255) / 256), dim3(256), 0, s, P, means, view, present);
}

void launch_relocation(int P, const float* oo, const float* so, const int* N, const float* binoms, int n_max,
                       float* on, float* sn, hipStream_t s)
{
    hipLaunchKernelGGL(k_relocation, dim3((P + 255) / 256), dim3(256), 0, s, P, oo, so, N, binoms, n_max, on, sn);
}

}  // namespace hlgs
