// lod.hip -- hierarchical level-of-detail selection and child/parent interpolation for gfx950.
//
// Reference semantics (submodules/gaussianhierarchy/runtime_switching.cu):
//   k_mark_dynamic / k_put_dynamic   <- markNodesForSizeDynamic :533-582, putRenderIndicesDynamic :95-108
//   k_weights_dynamic                <- computeTsIndexedDynamic :637-684
//   k_mark_static / k_put_static     <- markNodesForSize :495-529, putRenderIndices :68-93
//   k_weights_static                 <- computeTsIndexed :588-634
//   k_spt_bsearch / k_spt_populate   <- binary_search_SPTs :784-810, populate_SPT :812-856,
//                                       DeviceSelect::If :944-950, ExclusiveSum :973-986
//   k_lod_interp_fwd / _bwd          <- gaussian_renderer/__init__.py:304-339 (render_post lerp) and its autograd
#include <float.h>

#include "hlgs_internal.h"
#include "hlgs_math.h"

namespace hlgs {

// ---- dynamic hierarchy: HierarchyNode {depth, parent, child_count, first_child, next_sibling, max_side_length}
__device__ __forceinline__ float gauss_dist(const float* p, float vx, float vy, float vz)
{
    const float d0 = vx - p[0], d1 = vy - p[1], d2 = vz - p[2];
    return sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
}
__device__ __forceinline__ bool in_cone(const float* p, float vx, float vy, float vz, float zx, float zy, float zz)
{
    const float d0 = vx - p[0], d1 = vy - p[1], d2 = vz - p[2];
    const float n = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
    const float c = d0 / n * zx + d1 / n * zy + d2 / n * zz;
    return c < -0.5f;
}
__device__ __forceinline__ float size_dyn(const float* p, const float* s, float vx, float vy, float vz)
{
    const float md = gauss_dist(p, vx, vy, vz);
    if (md < 0.0f) return 0;
    return fmaxf(s[0], fmaxf(s[1], s[2])) / md;
}

__global__ void __launch_bounds__(256) k_mark_dynamic(int N, const int* __restrict__ nodes, const float* __restrict__ pos,
                                                      const float* __restrict__ scales, const float* __restrict__ vp,
                                                      float zx, float zy, float zz, float target,
                                                      uint32_t* __restrict__ counts)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    const float vx = vp[0], vy = vp[1], vz = vp[2];
    const int* nd = nodes + 6 * i;
    uint32_t c = 0;
    if (in_cone(pos + 3 * i, vx, vy, vz, zx, zy, zz)) {
        const float size = size_dyn(pos + 3 * i, scales + 3 * i, vx, vy, vz);
        const int depth = nd[0], parent = nd[1], nchild = nd[2];
        if (depth < 0) c = 0;
        else if (size >= target && nchild == 0) c = 1;
        else if (parent >= 0) {
            const float ps = size_dyn(pos + 3 * parent, scales + 3 * parent, vx, vy, vz);
            if (ps >= target && size < target) c = 1;
        }
    }
    counts[i] = c;
}

__global__ void __launch_bounds__(256) k_put_dynamic(int N, const int* __restrict__ nodes, const uint32_t* __restrict__ counts,
                                                     const uint32_t* __restrict__ incl, int* __restrict__ render_indices,
                                                     int* __restrict__ parent_indices, int* __restrict__ nodes_for)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N || counts[i] == 0) return;
    const uint32_t off = incl[i] - 1;
    render_indices[off] = i;
    nodes_for[off] = i;
    const int parent = nodes[6 * i + 1];
    if (parent != -1) parent_indices[off] = parent;
}

__global__ void __launch_bounds__(256) k_weights_dynamic(int n, const int* __restrict__ idx, const int* __restrict__ nodes,
                                                         const float* __restrict__ pos, const float* __restrict__ scales,
                                                         float vx, float vy, float vz, float target,
                                                         float* __restrict__ ts, int* __restrict__ kids)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int id = idx[i];
    const int parent = nodes[6 * id + 1];
    float t;
    if (parent < 0) t = 1.0f;
    else {
        const float ps = size_dyn(pos + 3 * parent, scales + 3 * parent, vx, vy, vz);
        if (ps > 2.0f * target) t = 1.0f;
        else {
            const float s = size_dyn(pos + 3 * id, scales + 3 * id, vx, vy, vz);
            const float start = fmaxf(0.5f * ps, s);
            const float diff = ps - start;
            if (diff <= 0) t = 1.0f;
            else {
                const float td = fmaxf(0.0f, target - start);
                t = fmaxf(1.0f - (td / diff), 0.0f);
            }
        }
    }
    ts[i] = t;
    kids[i] = parent < 0 ? 1 : nodes[6 * parent + 2];
}

// ---- static (.hier) hierarchy: Node {depth, parent, start, count_leafs, count_merged, start_children,
// count_children}, Box {minn xyzw, maxx xyzw}
__device__ __forceinline__ float size_box(const float* b, float vx, float vy, float vz)
{
    const bool inside = vx >= b[0] && vx <= b[4] && vy >= b[1] && vy <= b[5] && vz >= b[2] && vz <= b[6];
    if (inside) return FLT_MAX;
    const float c0 = fmaxf(b[0], fminf(b[4], vx)), c1 = fmaxf(b[1], fminf(b[5], vy)), c2 = fmaxf(b[2], fminf(b[6], vz));
    const float d0 = vx - c0, d1 = vy - c1, d2 = vz - c2;
    return b[3] / sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
}

__global__ void __launch_bounds__(256) k_mark_static(int N, const int* __restrict__ nodes, const float* __restrict__ boxes,
                                                     const float* __restrict__ vp, float target,
                                                     uint32_t* __restrict__ counts)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    const float vx = vp[0], vy = vp[1], vz = vp[2];
    const int* nd = nodes + 7 * i;
    const float size = size_box(boxes + 8 * i, vx, vy, vz);
    int c = 0;
    if (size >= target) c = nd[3];
    else if (nd[1] != -1) {
        const float ps = size_box(boxes + 8 * nd[1], vx, vy, vz);
        if (ps >= target) {
            c = nd[3];
            if (nd[0] != 0) c += nd[4];
        }
    }
    counts[i] = (uint32_t)c;
}

__global__ void __launch_bounds__(256) k_put_static(int N, const int* __restrict__ nodes, const uint32_t* __restrict__ counts,
                                                    const uint32_t* __restrict__ incl, int* __restrict__ render_indices,
                                                    int* __restrict__ parent_indices, int* __restrict__ nodes_for)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    const uint32_t c = counts[i];
    if (c == 0) return;
    const uint32_t off = incl[i] - c;
    const int* nd = nodes + 7 * i;
    const int pg = nd[1] != -1 ? nodes[7 * nd[1] + 2] : -1;
    for (uint32_t k = 0; k < c; k++) {
        render_indices[off + k] = nd[2] + (int)k;
        if (parent_indices) parent_indices[off + k] = pg;
        if (nodes_for) nodes_for[off + k] = i;
    }
}

__global__ void __launch_bounds__(256) k_weights_static(int n, const int* __restrict__ idx, const int* __restrict__ nodes,
                                                        const float* __restrict__ boxes, float vx, float vy, float vz,
                                                        float target, float* __restrict__ ts, int* __restrict__ kids)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int id = idx[i];
    const int parent = nodes[7 * id + 1];
    float t;
    if (parent == -1) t = 1.0f;
    else {
        const float ps = size_box(boxes + 8 * parent, vx, vy, vz);
        if (ps > 2.0f * target) t = 1.0f;
        else {
            const float s = size_box(boxes + 8 * id, vx, vy, vz);
            const float start = fmaxf(0.5f * ps, s);
            const float diff = ps - start;
            if (diff <= 0) t = 1.0f;
            else {
                const float td = fmaxf(0.0f, target - start);
                t = fmaxf(1.0f - (td / diff), 0.0f);
            }
        }
    }
    ts[i] = t;
    kids[i] = parent == -1 ? 1 : nodes[7 * parent + 6];
}

// ---- SPT cut
__global__ void __launch_bounds__(256) k_spt_bsearch(int s, const int* __restrict__ starts, const float* __restrict__ smax,
                                                     const int* __restrict__ sidx, const float* __restrict__ sdist,
                                                     uint32_t* __restrict__ sizes)
{
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= s) return;
    const int index = sidx[k];
    const float d = sdist[k];
    int low = starts[index], high = starts[index + 1];
    int pivot = (low + high) / 2;
    while (high - low > 1) {
        if (smax[pivot] > d) low = pivot;
        else high = pivot;
        pivot = (low + high) / 2;
    }
    sizes[k] = (uint32_t)(high - starts[index]);
}

__global__ void __launch_bounds__(256) k_spt_populate(int s, int E, int n, const int* __restrict__ gidx,
                                                      const int* __restrict__ starts, const float* __restrict__ smin,
                                                      const int* __restrict__ sidx, const float* __restrict__ sdist,
                                                      const uint32_t* __restrict__ sizes, const uint32_t* __restrict__ incl,
                                                      int compat, int* __restrict__ result, uint32_t* __restrict__ keep,
                                                      uint32_t* __restrict__ counts)
{
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= n) return;
    auto prefix = [&](int k) { return (int)(incl[k] - sizes[k]); };
    int ii;
    if (compat) {  // populate_SPT's search, including its `>=` boundary attribution (App. A-10)
        int low = 0, high = s;
        ii = s / 2;
        while (high - low > 1) {
            if (prefix(ii) >= idx) high = ii;
            else low = ii;
            ii = (high + low) / 2;
        }
    } else {  // intended semantics (scene/gaussian_model.py:163-181): largest k with prefix[k] <= idx
        int low = 0, high = s;
        while (high - low > 1) {
            const int mid = (low + high) / 2;
            if (prefix(mid) <= idx) low = mid; else high = mid;
        }
        ii = low;
    }
    const int g = starts[sidx[ii]] + (idx - prefix(ii));
    uint32_t kp = 0;
    int v = 0;
    if (g < E && smin[g] < sdist[ii]) {
        atomicAdd(&counts[ii], 1u);
        v = gidx[g];
        kp = (!compat || v != 0) ? 1u : 0u;
    }
    result[idx] = v;
    keep[idx] = kp;
}

__global__ void __launch_bounds__(256) k_compact(int n, const int* __restrict__ result, const uint32_t* __restrict__ keep,
                                                 const uint32_t* __restrict__ incl, int* __restrict__ cut)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n || !keep[i]) return;
    cut[incl[i] - 1] = result[i];
}

__global__ void __launch_bounds__(256) k_excl_from_incl(int s, const uint32_t* __restrict__ counts,
                                                        const uint32_t* __restrict__ incl, int* __restrict__ out)
{
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k < s) out[k] = (int)(incl[k] - counts[k]);
}

// ---- render_post lerp: one thread per output row
// render_post lerp, one row per 16-lane group (four rows per wave): the group's lanes walk the row's SH floats
// with unit stride, so every load / store / atomic instruction covers a contiguous 64-byte segment of one row
// instead of one float in each of 64 rows.  Lanes 0-2 also do the mean, 3-5 the scale, 6-9 the rotation (the
// sign of <q_child, q_parent> from the whole quaternions), 10 the opacity.  Rows [0, S) are the uninterpolated
// skybox prefix.
struct LerpRow {
    int o, c, p;
    float t, u;
    bool skip;
};
__device__ __forceinline__ LerpRow lerp_row(int S, int n, const int* __restrict__ ridx, const int* __restrict__ pidx,
                                            const float* __restrict__ w)
{
    LerpRow r;
    r.o = blockIdx.x * 16 + (threadIdx.x >> 4);
    r.skip = r.o >= S + n;
    r.c = r.p = r.o;
    r.t = 1.f;
    r.u = 0.f;
    if (!r.skip && r.o >= S) {
        const int i = r.o - S;
        r.c = ridx[i];
        r.p = pidx[i];
        r.t = w[i];
        r.u = 1 - w[i];
    }
    return r;
}

__global__ void __launch_bounds__(256) k_lod_interp_fwd(int S, int n, int M3, const int* __restrict__ ridx,
                                                        const int* __restrict__ pidx, const float* __restrict__ w,
                                                        const float* __restrict__ means, const float* __restrict__ scales,
                                                        const float* __restrict__ rots, const float* __restrict__ opac,
                                                        const float* __restrict__ shs, float* __restrict__ om,
                                                        float* __restrict__ osc, float* __restrict__ orot,
                                                        float* __restrict__ oop, float* __restrict__ osh)
{
    const LerpRow r = lerp_row(S, n, ridx, pidx, w);
    if (r.skip) return;
    const int l = threadIdx.x & 15;
    const bool sky = r.o < S;
    if (shs) {
        const float* sc = shs + (size_t)M3 * r.c;
        const float* sp = shs + (size_t)M3 * r.p;
        float* so = osh + (size_t)M3 * r.o;
        for (int k = l; k < M3; k += 16) so[k] = sky ? sc[k] : r.t * sc[k] + r.u * sp[k];
    }
    if (l < 3) {
        om[3 * r.o + l] = sky ? means[3 * r.c + l] : r.t * means[3 * r.c + l] + r.u * means[3 * r.p + l];
    } else if (l < 6) {
        const int k = l - 3;
        osc[3 * r.o + k] = sky ? scales[3 * r.c + k] : r.t * scales[3 * r.c + k] + r.u * scales[3 * r.p + k];
    } else if (l < 10) {
        const int k = l - 6;
        const float4 rc = reinterpret_cast<const float4*>(rots)[r.c];
        float v = (&rc.x)[k];
        if (!sky) {
            const float4 rp = reinterpret_cast<const float4*>(rots)[r.p];
            float dotv = 0.f;
            dotv += rc.x * rp.x;
            dotv += rc.y * rp.y;
            dotv += rc.z * rp.z;
            dotv += rc.w * rp.w;
            const float pk = dotv < 0 ? -(&rp.x)[k] : (&rp.x)[k];
            v = r.t * v + r.u * pk;
        }
        orot[4 * r.o + k] = v;
    } else if (l == 10) {
        oop[r.o] = sky ? opac[r.c] : r.t * opac[r.c] + r.u * opac[r.p];
    }
}

// Degree-3 rows (M3 = 48) with every load of the row issued at once: lanes 0-11 of the group take one float4 of the
// child's and the parent's SH row each, lane 12 the mean, 13 the scale, 14 the rotation, 15 the opacity, so the
// group waits for one gather latency instead of one per loop step.  Same arithmetic as k_lod_interp_fwd.
__global__ void __launch_bounds__(256) k_lod_interp_fwd48(int S, int n, const int* __restrict__ ridx,
                                                          const int* __restrict__ pidx, const float* __restrict__ w,
                                                          const float* __restrict__ means,
                                                          const float* __restrict__ scales,
                                                          const float* __restrict__ rots, const float* __restrict__ opac,
                                                          const float* __restrict__ shs, float* __restrict__ om,
                                                          float* __restrict__ osc, float* __restrict__ orot,
                                                          float* __restrict__ oop, float* __restrict__ osh)
{
    const LerpRow r = lerp_row(S, n, ridx, pidx, w);
    if (r.skip) return;
    const int l = threadIdx.x & 15;
    const bool sky = r.o < S;
    const float t = r.t, u = r.u;
    // every lane issues the same four dword loads for the child and four for the parent, at lane-specific addresses
    // (lanes 0-11 a float4 of the SH row, 12 the mean, 13 the scale, 14 the rotation, 15 the opacity; short fields
    // repeat their last element): no divergent load paths, so one gather latency per row
    const float* base = l < 12 ? shs + 48 * (size_t)r.c + 4 * l
                      : l == 12 ? means + 3 * (size_t)r.c
                      : l == 13 ? scales + 3 * (size_t)r.c
                      : l == 14 ? rots + 4 * (size_t)r.c : opac + r.c;
    const float* pbase = l < 12 ? shs + 48 * (size_t)r.p + 4 * l
                       : l == 12 ? means + 3 * (size_t)r.p
                       : l == 13 ? scales + 3 * (size_t)r.p
                       : l == 14 ? rots + 4 * (size_t)r.p : opac + r.p;
    const int kmax = (l < 12 || l == 14) ? 3 : (l == 15 ? 0 : 2);
    float cv[4], pv[4];
#pragma unroll
    for (int k = 0; k < 4; k++) cv[k] = base[min(k, kmax)];
#pragma unroll
    for (int k = 0; k < 4; k++) pv[k] = sky ? 0.f : pbase[min(k, kmax)];
    const float4 c = make_float4(cv[0], cv[1], cv[2], cv[3]);
    float4 p = make_float4(pv[0], pv[1], pv[2], pv[3]);
    float4 v = c;
    if (!sky) {
        if (l == 14) {
            float dotv = 0.f;
            dotv += c.x * p.x;
            dotv += c.y * p.y;
            dotv += c.z * p.z;
            dotv += c.w * p.w;
            if (dotv < 0) p = make_float4(-p.x, -p.y, -p.z, -p.w);
        }
        v = make_float4(t * c.x + u * p.x, t * c.y + u * p.y, t * c.z + u * p.z, t * c.w + u * p.w);
    }
    if (l < 12) reinterpret_cast<float4*>(osh + (size_t)48 * r.o)[l] = v;
    else if (l == 14) reinterpret_cast<float4*>(orot)[r.o] = v;
    else if (l == 15) oop[r.o] = v.x;
    else {
        float* dst = l == 12 ? om : osc;
        dst[3 * r.o] = v.x;
        dst[3 * r.o + 1] = v.y;
        dst[3 * r.o + 2] = v.z;
    }
}

// Autograd of the lerp: d_child += t g, d_parent += (1 - t) g (the parent's rotation gradient negated where the
// forward flipped its sign), d_sky = g for the prefix rows.  A node can be a selected child, the parent of
// several selected nodes and, with non-monotone sizes, both.  Instead of float atomics on zero-initialised
// gradients (torch's index_add in the reference's autograd), every node's contributions are gathered: the 2n
// (node, row, role) entries are bucketed by node (counting sort: k_lerp_count, scan, k_lerp_fill), and
// k_lerp_gather walks each node's bucket in (row, role) order and writes all of its gradient row -- untouched
// nodes get zeros, so no memset is needed and the result is bitwise deterministic.
__global__ void __launch_bounds__(256) k_lerp_count(int n, const int* __restrict__ ridx, const int* __restrict__ pidx,
                                                    uint32_t* __restrict__ cnt)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    atomicAdd(&cnt[ridx[i]], 1u);
    atomicAdd(&cnt[pidx[i]], 1u);
}

__global__ void __launch_bounds__(256) k_lerp_fill(int n, const int* __restrict__ ridx, const int* __restrict__ pidx,
                                                   const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ incl,
                                                   uint32_t* __restrict__ cur, uint32_t* __restrict__ list,
                                                   const float* __restrict__ rots, uint32_t* __restrict__ flip)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int c = ridx[i], p = pidx[i];
    if (flip) {  // the forward's rotation sign flip of row i (<q_child, q_parent> < 0), for the gather kernels
        const float4 rc = reinterpret_cast<const float4*>(rots)[c], rp = reinterpret_cast<const float4*>(rots)[p];
        float dotv = 0.f;
        dotv += rc.x * rp.x;
        dotv += rc.y * rp.y;
        dotv += rc.z * rp.z;
        dotv += rc.w * rp.w;
        flip[i] = dotv < 0 ? 1u : 0u;
    }
    list[incl[c] - cnt[c] + atomicAdd(&cur[c], 1u)] = 2u * (uint32_t)i;       // child role
    list[incl[p] - cnt[p] + atomicAdd(&cur[p], 1u)] = 2u * (uint32_t)i + 1u;  // parent role
}

// One wave per 64 consecutive nodes: the wave first stores zero rows for all of them with full-wave coalesced
// stores, then its four 16-lane groups take the touched nodes (bucket non-empty or skybox) four at a time, walk
// each bucket in (row, role) order and overwrite the node's row.
template <int KSH>  // SH floats handled per lane: ceil(M3 / 16) <= KSH
__global__ void __launch_bounds__(64) k_lerp_gather(int P, int S, int M3, const int* __restrict__ ridx,
                                                    const float* __restrict__ w, const float* __restrict__ rots,
                                                    const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ incl,
                                                    const uint32_t* __restrict__ list, const float* __restrict__ gm,
                                                    const float* __restrict__ gsc, const float* __restrict__ grot,
                                                    const float* __restrict__ gop, const float* __restrict__ gsh,
                                                    float* __restrict__ dm, float* __restrict__ dsc,
                                                    float* __restrict__ drot, float* __restrict__ dop,
                                                    float* __restrict__ dsh)
{
    const int lane = threadIdx.x;
    const int v0 = blockIdx.x * 64;
    const int nv = min(64, P - v0);
    // zero rows (every output row is written by this kernel)
    for (int e = lane; e < 3 * nv; e += 64) { dm[3 * (size_t)v0 + e] = 0.f; dsc[3 * (size_t)v0 + e] = 0.f; }
    for (int e = lane; e < 4 * nv; e += 64) drot[4 * (size_t)v0 + e] = 0.f;
    if (lane < nv) dop[v0 + lane] = 0.f;
    if (dsh)
        for (int e = lane; e < M3 * nv; e += 64) dsh[(size_t)M3 * v0 + e] = 0.f;
    const int my_v = v0 + lane;
    const uint32_t my_k = lane < nv ? cnt[my_v] : 0u;
    const uint32_t my_start = lane < nv ? incl[my_v] - my_k : 0u;
    uint64_t todo = __ballot(lane < nv && (my_k > 0 || my_v < S));
    // make the zero stores visible before the overwrites (same wave, same addresses: program order suffices for
    // a single lane, but rows are overwritten by other lanes)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_waitcnt(0);
    const int grp = lane >> 4, l = lane & 15;
    while (todo) {
        // the group's node: the grp-th remaining set bit
        uint64_t m = todo;
        for (int q = 0; q < grp && m; q++) m &= m - 1;
        const bool have = m != 0;
        const int src = have ? __builtin_ctzll(m) : 0;
        // consume four bits
        for (int q = 0; q < 4 && todo; q++) todo &= todo - 1;
        const uint32_t k = __shfl(my_k, src, 64), start = __shfl(my_start, src, 64);
        if (!have) continue;
        const int v = v0 + src;
        float acc_sh[KSH];
#pragma unroll
        for (int j = 0; j < KSH; j++) acc_sh[j] = 0.f;
        float acc = 0.f;  // lane 0-2 mean, 3-5 scale, 6-9 rotation, 10 opacity
        auto small_grad = [&](int o) -> float {
            if (l < 3) return gm[3 * o + l];
            if (l < 6) return gsc[3 * o + l - 3];
            if (l < 10) return grot[4 * o + l - 6];
            if (l == 10) return gop[o];
            return 0.f;
        };
        if (v < S) {  // skybox prefix: identity
            acc += small_grad(v);
#pragma unroll
            for (int j = 0; j < KSH; j++)
                if (gsh && l + 16 * j < M3) acc_sh[j] += gsh[(size_t)M3 * v + l + 16 * j];
        }
        uint32_t prev = 0xffffffffu;
        for (uint32_t e = 0; e < k; e++) {
            uint32_t best = 0xffffffffu;  // next entry in (row, role) order: buckets hold a handful of entries
            for (uint32_t q = 0; q < k; q++) {
                const uint32_t x = list[start + q];
                if ((prev == 0xffffffffu || x > prev) && x < best) best = x;
            }
            prev = best;
            const int row = (int)(best >> 1);
            const bool parent = best & 1u;
            const int o = S + row;
            const float t = w[row];
            const float f = parent ? 1 - t : t;
            const float g = small_grad(o);
            if (parent && l >= 6 && l < 10) {
                const float4 rc = reinterpret_cast<const float4*>(rots)[ridx[row]];
                const float4 rp = reinterpret_cast<const float4*>(rots)[v];
                float dotv = 0.f;
                dotv += rc.x * rp.x;
                dotv += rc.y * rp.y;
                dotv += rc.z * rp.z;
                dotv += rc.w * rp.w;
                acc += (dotv < 0 ? -1.0f : 1.0f) * (f * g);
            } else {
                acc += f * g;
            }
#pragma unroll
            for (int j = 0; j < KSH; j++)
                if (gsh && l + 16 * j < M3) acc_sh[j] += f * gsh[(size_t)M3 * o + l + 16 * j];
        }
        if (l < 3) dm[3 * v + l] = acc;
        else if (l < 6) dsc[3 * v + l - 3] = acc;
        else if (l < 10) drot[4 * v + l - 6] = acc;
        else if (l == 10) dop[v] = acc;
#pragma unroll
        for (int j = 0; j < KSH; j++)
            if (dsh && l + 16 * j < M3) dsh[(size_t)M3 * v + l + 16 * j] = acc_sh[j];
    }
}

// Degree-3 rows (M3 = 48).  The small upstream gradients of each interpolated row (mean 3, scale 3, rotation 4,
// opacity 1) are first packed into one 12-float row (k_lerp_pack), so every lane of a 16-lane group issues the same single
// float4 load per entry: lanes 0-11 one float4 of the SH row, lanes 12-14 the packed small row (lane 15 idles).
// A group owns two consecutive nodes; their bucket bounds, then their bucket entries (up to kLerpUnroll each, put in
// (row, role) order in registers), then every weight, sign flag and gradient load of every entry are issued as three
// rounds; a longer bucket takes the serial next-minimum walk.  Untouched nodes store zero rows.  Sums run in the
// (sky, then (row, role) ascending) order of k_lerp_gather; a parent entry's rotation sign comes from k_lerp_fill.
constexpr int kLerpUnroll = 3;
constexpr int kLerpNodes = 2;
__global__ void __launch_bounds__(256) k_lerp_pack(int n, int S, const float* __restrict__ gm,
                                                   const float* __restrict__ gsc, const float* __restrict__ grot,
                                                   const float* __restrict__ gop, float4* __restrict__ packed)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int o = S + i;
    const float4 r = reinterpret_cast<const float4*>(grot)[o];
    packed[3 * i] = make_float4(gm[3 * o], gm[3 * o + 1], gm[3 * o + 2], gsc[3 * o]);
    packed[3 * i + 1] = make_float4(gsc[3 * o + 1], gsc[3 * o + 2], r.x, r.y);
    packed[3 * i + 2] = make_float4(r.z, r.w, gop[o], 0.f);
}
// gradient of interpolated row `row` (output row S + row) in the lane's packed layout
__device__ __forceinline__ const float4* lerp_src(int l, int S, int row, const float* __restrict__ gsh,
                                                  const float4* __restrict__ packed)
{
    return l < 12 ? reinterpret_cast<const float4*>(gsh + (size_t)48 * (S + row)) + l
                  : packed + 3 * (size_t)row + min(l - 12, 2);
}
// skybox output row v (< S) in the same lane layout, read field by field (a short prefix)
__device__ __forceinline__ float4 lerp_sky(int l, int v, const float* __restrict__ gm, const float* __restrict__ gsc,
                                           const float* __restrict__ grot, const float* __restrict__ gop,
                                           const float* __restrict__ gsh)
{
    if (l < 12) return reinterpret_cast<const float4*>(gsh + (size_t)48 * v)[l];
    if (l == 12) return make_float4(gm[3 * v], gm[3 * v + 1], gm[3 * v + 2], gsc[3 * v]);
    if (l == 13) return make_float4(gsc[3 * v + 1], gsc[3 * v + 2], grot[4 * v], grot[4 * v + 1]);
    if (l == 14) return make_float4(grot[4 * v + 2], grot[4 * v + 3], gop[v], 0.f);
    return make_float4(0.f, 0.f, 0.f, 0.f);
}
// rotation components in the packed layout: lane 13 .z .w, lane 14 .x .y
__device__ __forceinline__ void lerp_acc(float4& acc, float f, float4 g, bool neg, int l)
{
    const float sx = (neg && l == 14) ? -1.0f : 1.0f, sy = sx;
    const float sz = (neg && l == 13) ? -1.0f : 1.0f, sw = sz;
    acc.x += sx * (f * g.x);
    acc.y += sy * (f * g.y);
    acc.z += sz * (f * g.z);
    acc.w += sw * (f * g.w);
}

__global__ void __launch_bounds__(256) k_lerp_gather48(int P, int S, const float* __restrict__ w,
                                                       const uint32_t* __restrict__ flip,
                                                       const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ incl,
                                                       const uint32_t* __restrict__ list, const float4* __restrict__ packed,
                                                       const float* __restrict__ gm, const float* __restrict__ gsc,
                                                       const float* __restrict__ grot, const float* __restrict__ gop,
                                                       const float* __restrict__ gsh, float* __restrict__ dm,
                                                       float* __restrict__ dsc, float* __restrict__ drot,
                                                       float* __restrict__ dop, float* __restrict__ dsh)
{
    const int v0 = (blockIdx.x * 16 + (threadIdx.x >> 4)) * kLerpNodes;
    if (v0 >= P) return;
    const int l = threadIdx.x & 15;
    uint32_t k[kLerpNodes], st[kLerpNodes];
#pragma unroll
    for (int j = 0; j < kLerpNodes; j++) {
        const int v = v0 + j;
        k[j] = v < P ? cnt[v] : 0u;
        st[j] = v < P ? incl[v] - k[j] : 0u;
    }
    uint32_t e[kLerpNodes][kLerpUnroll];
#pragma unroll
    for (int j = 0; j < kLerpNodes; j++)
#pragma unroll
        for (int q = 0; q < kLerpUnroll; q++) e[j][q] = (q < (int)k[j] && k[j] <= kLerpUnroll) ? list[st[j] + q] : ~0u;
    float4 acc[kLerpNodes];
#pragma unroll
    for (int j = 0; j < kLerpNodes; j++) {
        acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (v0 + j < S) acc[j] = lerp_sky(l, v0 + j, gm, gsc, grot, gop, gsh);  // skybox prefix: identity
#pragma unroll
        for (int i = 1; i < kLerpUnroll; i++)  // insertion sort in registers (entries are distinct; ~0 pads last)
#pragma unroll
            for (int q = i; q > 0; q--) {
                const uint32_t x = e[j][q - 1], y = e[j][q];
                e[j][q - 1] = min(x, y);
                e[j][q] = max(x, y);
            }
    }
    float4 g[kLerpNodes][kLerpUnroll];
    float f[kLerpNodes][kLerpUnroll];
    bool neg[kLerpNodes][kLerpUnroll];
#pragma unroll
    for (int j = 0; j < kLerpNodes; j++)
#pragma unroll
        for (int q = 0; q < kLerpUnroll; q++) {
            f[j][q] = 0.f;
            neg[j][q] = false;
            g[j][q] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (e[j][q] != ~0u) {
                const int row = (int)(e[j][q] >> 1);
                const bool par = e[j][q] & 1u;
                const float t = w[row];
                f[j][q] = par ? 1 - t : t;
                neg[j][q] = par && flip[row];
                g[j][q] = *lerp_src(l, S, row, gsh, packed);
            }
        }
#pragma unroll
    for (int j = 0; j < kLerpNodes; j++) {
        const int v = v0 + j;
        if (v >= P) break;
        if (k[j] <= kLerpUnroll) {
#pragma unroll
            for (int q = 0; q < kLerpUnroll; q++)
                if (e[j][q] != ~0u) lerp_acc(acc[j], f[j][q], g[j][q], neg[j][q], l);
        } else {
            uint32_t prev = ~0u;
            for (uint32_t q = 0; q < k[j]; q++) {
                uint32_t best = ~0u;
                for (uint32_t x = 0; x < k[j]; x++) {
                    const uint32_t y = list[st[j] + x];
                    if ((prev == ~0u || y > prev) && y < best) best = y;
                }
                prev = best;
                const int row = (int)(best >> 1);
                const bool par = best & 1u;
                const float t = w[row];
                lerp_acc(acc[j], par ? 1 - t : t, *lerp_src(l, S, row, gsh, packed), par && flip[row], l);
            }
        }
        const float4 a = acc[j];
        if (l < 12) reinterpret_cast<float4*>(dsh + (size_t)48 * v)[l] = a;
        else if (l == 12) { dm[3 * v] = a.x; dm[3 * v + 1] = a.y; dm[3 * v + 2] = a.z; dsc[3 * v] = a.w; }
        else if (l == 13) { dsc[3 * v + 1] = a.x; dsc[3 * v + 2] = a.y; drot[4 * v] = a.z; drot[4 * v + 1] = a.w; }
        else if (l == 14) { drot[4 * v + 2] = a.x; drot[4 * v + 3] = a.y; dop[v] = a.z; }
    }
}

// ---- host launchers
static inline dim3 g256(long n) { return dim3((unsigned)((n + 255) / 256)); }

void launch_expand_dynamic(int N, float target, const int* nodes, const float* pos, const float* scales, const float* vp,
                           const float* vd, int* ri, int* pi, int* ni, uint32_t* counts, uint32_t* incl, uint32_t* tmp,
                           hipStream_t s)
{
    hipLaunchKernelGGL(k_mark_dynamic, g256(N), dim3(256), 0, s, N, nodes, pos, scales, vp, vd[0], vd[1], vd[2], target,
                       counts);
    scan_inclusive_u32(counts, incl, (size_t)N, tmp, s);
    hipLaunchKernelGGL(k_put_dynamic, g256(N), dim3(256), 0, s, N, nodes, counts, incl, ri, pi, ni);
}

void launch_weights_dynamic(int n, const int* idx, float target, const int* nodes, const float* pos,
                            const float* scales, const float* vp, float* ts, int* kids, hipStream_t s)
{
    hipLaunchKernelGGL(k_weights_dynamic, g256(n), dim3(256), 0, s, n, idx, nodes, pos, scales, vp[0], vp[1], vp[2],
                       target, ts, kids);
}

void launch_expand_static(int N, float target, const int* nodes, const float* boxes, const float* vp, int* ri, int* pi,
                          int* ni, uint32_t* counts, uint32_t* incl, uint32_t* tmp, hipStream_t s)
{
    hipLaunchKernelGGL(k_mark_static, g256(N), dim3(256), 0, s, N, nodes, boxes, vp, target, counts);
    scan_inclusive_u32(counts, incl, (size_t)N, tmp, s);
    hipLaunchKernelGGL(k_put_static, g256(N), dim3(256), 0, s, N, nodes, counts, incl, ri, pi, ni);
}

void launch_weights_static(int n, const int* idx, float target, const int* nodes, const float* boxes, const float* vp,
                           float* ts, int* kids, hipStream_t s)
{
    hipLaunchKernelGGL(k_weights_static, g256(n), dim3(256), 0, s, n, idx, nodes, boxes, vp[0], vp[1], vp[2], target,
                       ts, kids);
}

void launch_spt_prepare(int s_, const int* starts, const float* smax, const int* sidx, const float* sdist,
                        uint32_t* sizes, uint32_t* incl, uint32_t* tmp, hipStream_t s)
{
    hipLaunchKernelGGL(k_spt_bsearch, g256(s_), dim3(256), 0, s, s_, starts, smax, sidx, sdist, sizes);
    scan_inclusive_u32(sizes, incl, (size_t)s_, tmp, s);
}

void launch_spt_finish(int s_, int E, int n, const int* gidx, const int* starts, const float* smin, const int* sidx,
                       const float* sdist, int compat, const uint32_t* sizes, const uint32_t* incl, uint32_t* counts,
                       uint32_t* counts_incl, uint32_t* tmp_s, int* result, uint32_t* keep, uint32_t* keep_incl,
                       uint32_t* tmp_n, int* cut, int* counts_prefix, hipStream_t s)
{
    hipMemsetAsync(counts, 0, sizeof(uint32_t) * (size_t)s_, s);
    if (n > 0) {
        hipLaunchKernelGGL(k_spt_populate, g256(n), dim3(256), 0, s, s_, E, n, gidx, starts, smin, sidx, sdist, sizes,
                           incl, compat, result, keep, counts);
        scan_inclusive_u32(keep, keep_incl, (size_t)n, tmp_n, s);
        hipLaunchKernelGGL(k_compact, g256(n), dim3(256), 0, s, n, result, keep, keep_incl, cut);
    }
    scan_inclusive_u32(counts, counts_incl, (size_t)s_, tmp_s, s);
    hipLaunchKernelGGL(k_excl_from_incl, g256(s_), dim3(256), 0, s, s_, counts, counts_incl, counts_prefix);
}

void launch_lod_interp_fwd(int S, int n, int M3, const int* ridx, const int* pidx, const float* w, const float* means,
                           const float* scales, const float* rots, const float* opac, const float* shs, float* om,
                           float* osc, float* orot, float* oop, float* osh, hipStream_t s)
{
    if (M3 == 48 && shs) {
        hipLaunchKernelGGL(k_lod_interp_fwd48, dim3((unsigned)(((long)S + n + 15) / 16)), dim3(256), 0, s, S, n, ridx,
                           pidx, w, means, scales, rots, opac, shs, om, osc, orot, oop, osh);
        return;
    }
    hipLaunchKernelGGL(k_lod_interp_fwd, dim3((unsigned)(((long)S + n + 15) / 16)), dim3(256), 0, s, S, n, M3, ridx,
                       pidx, w, means, scales,
                       rots, opac, shs, om, osc, orot, oop, osh);
}

size_t lerp_bwd_scratch_elems(int P, int n)
{
    return 4 * align_up(sizeof(uint32_t) * (size_t)P) / 4 + align_up(sizeof(uint32_t) * scan_scratch_elems(P)) / 4 +
           align_up(sizeof(uint32_t) * 2 * (size_t)n) / 4 + align_up(sizeof(float) * 12 * (size_t)n) / 4;
}

void launch_lod_interp_bwd(int P, int S, int n, int M3, const int* ridx, const int* pidx, const float* w,
                           const float* rots, const float* gm, const float* gsc, const float* grot, const float* gop,
                           const float* gsh, float* dm, float* dsc, float* drot, float* dop, float* dsh, void* scratch,
                           hipStream_t s)
{
    char* p = static_cast<char*>(scratch);
    auto take = [&](size_t count) {
        uint32_t* r = reinterpret_cast<uint32_t*>(p);
        p += align_up(count * sizeof(uint32_t));
        return r;
    };
    uint32_t* cnt = take(P);
    uint32_t* cur = take(P);
    uint32_t* incl = take(P);
    uint32_t* flip = take(P);  // per-row rotation sign flip (n <= P)
    uint32_t* tmp = take(scan_scratch_elems(P));
    uint32_t* list = take(2 * (size_t)n);
    float4* packed = reinterpret_cast<float4*>(take(12 * (size_t)n));  // k_lerp_pack rows (degree-3 path)
    hipMemsetAsync(cnt, 0, sizeof(uint32_t) * (size_t)P, s);
    hipMemsetAsync(cur, 0, sizeof(uint32_t) * (size_t)P, s);
    if (n > 0) hipLaunchKernelGGL(k_lerp_count, g256(n), dim3(256), 0, s, n, ridx, pidx, cnt);
    scan_inclusive_u32(cnt, incl, (size_t)P, tmp, s);
    const bool fast = M3 == 48 && gsh && dsh;
    if (n > 0)
        hipLaunchKernelGGL(k_lerp_fill, g256(n), dim3(256), 0, s, n, ridx, pidx, cnt, incl, cur, list, rots,
                           fast ? flip : nullptr);
    if (fast) {
        if (n > 0) hipLaunchKernelGGL(k_lerp_pack, g256(n), dim3(256), 0, s, n, S, gm, gsc, grot, gop, packed);
        const long groups = ((long)P + kLerpNodes - 1) / kLerpNodes;
        hipLaunchKernelGGL(k_lerp_gather48, dim3((unsigned)((groups + 15) / 16)), dim3(256), 0, s, P, S, w, flip, cnt,
                           incl, list, packed, gm, gsc, grot, gop, gsh, dm, dsc, drot, dop, dsh);
        return;
    }
    const dim3 grid((unsigned)(((long)P + 63) / 64));
#define HLGS_LG(K) hipLaunchKernelGGL((k_lerp_gather<K>), grid, dim3(64), 0, s, P, S, M3, ridx, w, rots, cnt, incl, list, \
                                      gm, gsc, grot, gop, gsh, dm, dsc, drot, dop, dsh)
    if (M3 <= 16) HLGS_LG(1);
    else if (M3 <= 32) HLGS_LG(2);
    else if (M3 <= 48) HLGS_LG(3);
    else HLGS_LG(4);
#undef HLGS_LG
}

// get_morton_indices (gaussianhierarchy/morton.cu:9-42, bound at torch_interface.cpp:246-260): 63-bit Morton
// code of each position normalised to the [min, max] box and scaled by 2^21; the float -> int64 conversion
// truncates and only bits 0..20 of each coordinate are interleaved, as the reference does.
__global__ void __launch_bounds__(256) k_morton(int P, const float* __restrict__ xyz, const float* __restrict__ mn,
                                                const float* __restrict__ mx, int64_t* __restrict__ codes)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    const float bx = mx[0] - mn[0], by = mx[1] - mn[1], bz = mx[2] - mn[2];
    const float px = (xyz[3 * i] - mn[0]) / bx * (float)(1 << 21);
    const float py = (xyz[3 * i + 1] - mn[1]) / by * (float)(1 << 21);
    const float pz = (xyz[3 * i + 2] - mn[2]) / bz * (float)(1 << 21);
    const int64_t q[3] = {(int64_t)px, (int64_t)py, (int64_t)pz};
    int64_t code = 0;
#pragma unroll
    for (int b = 0; b < 21; ++b) {
        code |= (q[0] >> b & 1) << (3 * b);
        code |= (q[1] >> b & 1) << (3 * b + 1);
        code |= (q[2] >> b & 1) << (3 * b + 2);
    }
    codes[i] = code;
}

void launch_morton(int P, const float* xyz, const float* mn, const float* mx, int64_t* codes, hipStream_t s)
{
    hipLaunchKernelGGL(k_morton, g256(P), dim3(256), 0, s, P, xyz, mn, mx, codes);
}

}  // namespace hlgs
