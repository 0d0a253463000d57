// spt_build.cpp -- host-side construction of the sequential point trees (SPTs) and the upper tree of the SPT
// streaming step: GaussianModel.build_hierarchical_SPT and get_min_distance (scene/gaussian_model.py:184-352),
// restated as one pass over host arrays instead of a Python loop of small device ops per SPT.
//
// Steps (gaussian_model.py line numbers):
//   :186-187  upper tree / cut = cut_hierarchy_on_condition(nodes, prod(exp(scale)) > SPT_Root_Volume) from the
//             hierarchy root (the reference's default root_node = 100000 = its skybox size): visited nodes form
//             the upper tree, leaves and nodes failing the condition the cut.
//   :203-257  for every cut node with children: a breadth-first walk of its subtree (first children, then their
//             next siblings, zeros dropped) recording per node [id, min distance, max distance] with
//             min = min(get_min_distance + |x - centre|, parent's min) and max = the parent's min; the SPT is kept
//             if it has more than min_SPT_Size rows (sorted by max distance, descending, ties in walk order),
//             otherwise its nodes join the upper tree.
//   :259-290  upper tree: sorted indices, node rows remapped to upper-tree positions, SPT leaves store the SPT
//             number in first_child, plain leaves -1; min_distance_squared from the parent's min distance.
//   :292-310  bounding-sphere radii: 3 x max scale at leaves, the SPT walk's radius at SPT leaves, propagated
//             upward as max over the two children of child radius + centre distance.
// float32 arithmetic throughout, in the reference's operation order.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/hlgs.h"

namespace hlgs {
int fail_msg(int code, const std::string& msg);  // capi.hip
}

struct hlgs_spt_result {
    std::vector<int> starts, gidx, roots;
    std::vector<float> smax, smin;
    std::vector<int> up_nodes;  // U x 6
    std::vector<float> up_xyz, up_scaling, min_d2, radii;
};

namespace {

constexpr int kDepth = 0, kParent = 1, kChildCount = 2, kFirstChild = 3, kNextSibling = 4, kMaxSide = 5;

struct Ctx {
    int G;
    const int* nodes;
    const float* xyz;
    const float* sc;  // log scales
    float tg;
    const int* nd(int i) const { return nodes + 6 * (size_t)i; }
    float es(int i, int k) const { return expf(sc[3 * (size_t)i + k]); }
    float max_es(int i) const { return std::max(es(i, 0), std::max(es(i, 1), es(i, 2))); }
    // get_min_distance (gaussian_model.py:334-352); `single` selects the one-node branch (leaf -> -1e6)
    float min_distance(int i, bool single) const
    {
        if (nd(i)[kChildCount] == 0) return single ? -1000000.f : -1000000000.f;
        const float s0 = es(i, 0), s1 = es(i, 1), s2 = es(i, 2);
        return sqrtf(s0 * s1 + s0 * s2 + s1 * s2) / tg;
    }
    float dist(int i, const float* c) const
    {
        const float d0 = xyz[3 * (size_t)i] - c[0], d1 = xyz[3 * (size_t)i + 1] - c[1], d2 = xyz[3 * (size_t)i + 2] - c[2];
        return sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
    }
};

int search_sorted(const std::vector<int>& a, int v)  // torch.searchsorted (left)
{
    return (int)(std::lower_bound(a.begin(), a.end(), v) - a.begin());
}

}  // namespace

extern "C" {

int hlgs_spt_build(int G, const int* nodes, const float* xyz, const float* log_scales, int root, float spt_root_volume,
                   float target_granularity, int min_spt_size, int use_bounding_spheres, hlgs_spt_result** out)
{
    if (!out) return hlgs::fail_msg(HLGS_ERR_ARG, "null result");
    *out = nullptr;
    if (G <= 0 || root < 0 || root >= G || !nodes || !xyz || !log_scales)
        return hlgs::fail_msg(HLGS_ERR_ARG, "invalid hierarchy arguments");
    Ctx c{G, nodes, xyz, log_scales, target_granularity};
    auto bad = [&](int v) { return v < 0 || v >= G; };
    // ---- upper tree and cut (cut_hierarchy_on_condition, return_upper_tree=True)
    std::vector<int> upper, cut, stack{root}, next;
    while (!stack.empty()) {
        upper.insert(upper.end(), stack.begin(), stack.end());
        std::vector<int> inner;
        for (int v : stack) (c.nd(v)[kChildCount] == 0 ? cut : inner).push_back(v);
        std::vector<int> expand;
        for (int v : inner) {
            const float vol = c.es(v, 0) * c.es(v, 1) * c.es(v, 2);
            if (vol > spt_root_volume) expand.push_back(v);
        }
        for (int v : inner) {
            const float vol = c.es(v, 0) * c.es(v, 1) * c.es(v, 2);
            if (!(vol > spt_root_volume)) cut.push_back(v);
        }
        next.clear();
        for (int v : expand) next.push_back(c.nd(v)[kFirstChild]);
        const size_t nf = next.size();
        for (size_t i = 0; i < nf; i++) {
            if (bad(next[i])) return hlgs::fail_msg(HLGS_ERR_ARG, "child index out of range");
            next.push_back(c.nd(next[i])[kNextSibling]);
        }
        for (int v : next)
            if (bad(v)) return hlgs::fail_msg(HLGS_ERR_ARG, "child index out of range");
        stack.swap(next);
        if (upper.size() > (size_t)G * 4) return hlgs::fail_msg(HLGS_ERR_ARG, "hierarchy walk does not terminate");
    }
    auto* r = new hlgs_spt_result();
    r->starts.push_back(0);
    std::vector<int> spt_nodes, leaf_spt_children;
    std::vector<float> bsr_list;
    // ---- one SPT per cut node with children
    for (int cn : cut) {
        if (c.nd(cn)[kChildCount] == 0) continue;
        const float* centre = xyz + 3 * (size_t)cn;
        std::vector<int> ids{cn};
        std::vector<float> mins{c.min_distance(cn, true)}, maxs{1000000000000.f};
        std::vector<int> st{cn};
        std::vector<float> maxd{mins[0]};
        float bsr = c.max_es(cn) * 3.0f;
        std::vector<int> extra;
        while (true) {
            std::vector<int> first, all;
            for (int v : st) first.push_back(c.nd(v)[kFirstChild]);
            for (int f : first) all.push_back(f);
            for (int f : first) all.push_back(bad(f) ? 0 : c.nd(f)[kNextSibling]);
            std::vector<int> s2;
            for (int v : all)
                if (v > 0) s2.push_back(v);
            if (s2.empty()) break;
            for (int v : s2)
                if (bad(v)) { delete r; return hlgs::fail_msg(HLGS_ERR_ARG, "child index out of range"); }
            float mcd = -INFINITY;
            std::vector<float> cdist(s2.size());
            for (size_t i = 0; i < s2.size(); i++) {
                cdist[i] = c.dist(s2[i], centre);
                mcd = std::max(mcd, cdist[i] + c.max_es(s2[i]) * 3.0f);
            }
            bsr = std::max(bsr, mcd);
            std::vector<float> md;
            for (size_t i = 0; i < first.size(); i++)
                if (first[i] > 0) md.push_back(maxd[i]);
            const size_t half = md.size();
            for (size_t i = 0; i < half; i++) md.push_back(md[i]);
            if (md.size() != s2.size()) { delete r; return hlgs::fail_msg(HLGS_ERR_ARG, "SPT build needs a binary hierarchy"); }
            std::vector<float> nmin(s2.size());
            for (size_t i = 0; i < s2.size(); i++) {
                const float m = c.min_distance(s2[i], s2.size() == 1) + cdist[i];  // numel == 1: scalar branch
                nmin[i] = m < md[i] ? m : md[i];
                ids.push_back(s2[i]);
                mins.push_back(nmin[i]);
                maxs.push_back(md[i]);
            }
            maxd = nmin;
            extra.insert(extra.end(), s2.begin(), s2.end());
            st = s2;
        }
        if ((int)ids.size() > min_spt_size) {
            bsr_list.push_back(bsr);
            std::vector<int> order(ids.size());
            std::iota(order.begin(), order.end(), 0);
            std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return maxs[a] > maxs[b]; });
            leaf_spt_children.push_back((int)r->roots.size());
            spt_nodes.push_back(cn);
            for (int o : order) {
                r->smax.push_back(maxs[o]);
                r->smin.push_back(mins[o]);
                r->gidx.push_back(ids[o]);
            }
            r->starts.push_back(r->starts.back() + (int)ids.size());
            r->roots.push_back(cn);
        } else {
            upper.insert(upper.end(), extra.begin(), extra.end());
        }
    }
    // ---- upper tree arrays
    std::sort(upper.begin(), upper.end());
    const int U = (int)upper.size();
    r->up_nodes.resize(6 * (size_t)U);
    r->up_xyz.resize(3 * (size_t)U);
    r->up_scaling.resize(3 * (size_t)U);
    for (int i = 0; i < U; i++) {
        memcpy(&r->up_nodes[6 * (size_t)i], c.nd(upper[i]), 6 * sizeof(int));
        memcpy(&r->up_xyz[3 * (size_t)i], xyz + 3 * (size_t)upper[i], 3 * sizeof(float));
        memcpy(&r->up_scaling[3 * (size_t)i], log_scales + 3 * (size_t)upper[i], 3 * sizeof(float));
    }
    auto un = [&](int i) { return &r->up_nodes[6 * (size_t)i]; };
    std::vector<int> cut_spt(spt_nodes.size());
    std::vector<char> is_spt_leaf(U, 0);
    for (size_t k = 0; k < spt_nodes.size(); k++) {
        cut_spt[k] = search_sorted(upper, spt_nodes[k]);
        un(cut_spt[k])[kChildCount] = 0;
        un(cut_spt[k])[kFirstChild] = leaf_spt_children[k];
        is_spt_leaf[cut_spt[k]] = 1;
    }
    for (int i = 0; i < U; i++) {
        un(i)[kMaxSide] = upper[i];
        un(i)[kParent] = search_sorted(upper, un(i)[kParent]);
    }
    un(0)[kParent] = -1;
    for (int i = 0; i < U; i++)
        if (!is_spt_leaf[i]) un(i)[kFirstChild] = un(i)[kFirstChild] == 0 ? -1 : search_sorted(upper, un(i)[kFirstChild]);
    for (int i = 0; i < U; i++)
        if (un(i)[kNextSibling] > 0) un(i)[kNextSibling] = search_sorted(upper, un(i)[kNextSibling]);
    // min distance of the parent, squared (the parent of the root is read at index -1, i.e. the last row, and then
    // overwritten)
    r->min_d2.resize(U);
    for (int i = 0; i < U; i++) {
        int p = un(i)[kParent];
        if (p < 0) p += U;
        const int g = un(p)[kMaxSide];
        const float m = c.min_distance(g, false);
        r->min_d2[i] = m * m;
    }
    r->min_d2[0] = 1000000000000.f;
    if (use_bounding_spheres) {
        r->radii.assign(U, 0.f);
        for (int i = 0; i < U; i++)
            if (un(i)[kFirstChild] == -1) {
                const float* s = &r->up_scaling[3 * (size_t)i];
                r->radii[i] = std::max(expf(s[0]), std::max(expf(s[1]), expf(s[2]))) * 3;
            }
        for (size_t k = 0; k < cut_spt.size(); k++) r->radii[cut_spt[k]] = bsr_list[k];
        std::vector<int> level;
        for (int i = 0; i < U; i++)
            if (un(i)[kChildCount] == 0) level.push_back(i);
        auto udist = [&](int a, int b) {
            const float* pa = &r->up_xyz[3 * (size_t)a];
            const float* pb = &r->up_xyz[3 * (size_t)b];
            const float d0 = pa[0] - pb[0], d1 = pa[1] - pb[1], d2 = pa[2] - pb[2];
            return sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
        };
        int guard = 0;
        while (!level.empty() && guard++ < 4 * U + 8) {
            std::vector<int> parents;
            for (int v : level)
                if (un(v)[kParent] >= 0) parents.push_back(un(v)[kParent]);
            std::vector<float> vals(parents.size());
            for (size_t k = 0; k < parents.size(); k++) {  // all reads before the writes, as the vectorised assignment
                const int p = parents[k], f = un(p)[kFirstChild];
                const int s2 = (f >= 0 && f < U) ? un(f)[kNextSibling] : -1;
                if (f < 0 || f >= U || s2 < 0 || s2 >= U) { delete r; return hlgs::fail_msg(HLGS_ERR_ARG, "upper tree is not binary"); }
                vals[k] = std::max(r->radii[f] + udist(p, f), r->radii[s2] + udist(p, s2));
            }
            for (size_t k = 0; k < parents.size(); k++) r->radii[parents[k]] = vals[k];
            level.swap(parents);
        }
    }
    *out = r;
    return HLGS_OK;
}

int hlgs_spt_result_sizes(const hlgs_spt_result* r, int* n_spt, int* n_entries, int* n_upper)
{
    if (!r) return hlgs::fail_msg(HLGS_ERR_ARG, "null result");
    *n_spt = (int)r->roots.size();
    *n_entries = (int)r->gidx.size();
    *n_upper = (int)r->up_xyz.size() / 3;
    return HLGS_OK;
}

int hlgs_spt_result_copy(const hlgs_spt_result* r, int* starts, float* smax, float* smin, int* gidx, int* roots,
                         int* up_nodes, float* up_xyz, float* up_scaling, float* min_d2, float* radii)
{
    if (!r) return hlgs::fail_msg(HLGS_ERR_ARG, "null result");
    auto cp = [](void* dst, const void* src, size_t bytes) { if (dst && bytes) memcpy(dst, src, bytes); };
    cp(starts, r->starts.data(), r->starts.size() * sizeof(int));
    cp(smax, r->smax.data(), r->smax.size() * sizeof(float));
    cp(smin, r->smin.data(), r->smin.size() * sizeof(float));
    cp(gidx, r->gidx.data(), r->gidx.size() * sizeof(int));
    cp(roots, r->roots.data(), r->roots.size() * sizeof(int));
    cp(up_nodes, r->up_nodes.data(), r->up_nodes.size() * sizeof(int));
    cp(up_xyz, r->up_xyz.data(), r->up_xyz.size() * sizeof(float));
    cp(up_scaling, r->up_scaling.data(), r->up_scaling.size() * sizeof(float));
    cp(min_d2, r->min_d2.data(), r->min_d2.size() * sizeof(float));
    cp(radii, r->radii.data(), r->radii.size() * sizeof(float));
    return HLGS_OK;
}

void hlgs_spt_result_free(hlgs_spt_result* r) { delete r; }

// Walk order of the upper tree for the flat coarse cut (hlgs_upper_tree_cut_views_ordered_device).  The reference's
// walk (cut_hierarchy_on_condition, gaussian_model.py:364-404) keeps a frontier per level: the expanding nodes'
// first children in order, then those children's next siblings in order.  Whatever the view, a level's frontier is a
// subsequence of the frontier of the walk in which every node with children expands (F*, by induction: both halves
// of the next frontier keep the order of their parents).  So the cut is, level by level, the leaves of F*'s level
// that are alive (no ancestor culled or stopped), then its alive condition-false nodes, each in F* order.  Aliveness
// is a subtree test: with the walk's binary tree numbered in preorder, a node is dead iff it lies strictly inside
// the preorder interval of a non-expanding node.
// Blob (int32): [0] M = entries of F*, [1] levels, [2] usable, [3] N (the node count it was built for: the cut kernels
// reject a blob whose N differs), [4 .. 4 + levels] the levels' first entries
// (the last = M), then from HLGS_CUT_ORDER_HEADER: node[M], preorder position[M], preorder end[M] (position + subtree
// size), all in F* order.
size_t hlgs_upper_tree_order_size(int N)  // (64 words of room past the last array: whole 64-entry runs are read)
{
    return sizeof(int) * (HLGS_CUT_ORDER_HEADER + 3 * (size_t)(N > 0 ? N : 0) + 68);
}

int hlgs_upper_tree_order(int N, const int* nodes, void* order)
{
    if (N < 0 || !order || (N > 0 && !nodes)) return hlgs::fail_msg(HLGS_ERR_ARG, "bad upper-tree order arguments");
    int* o = static_cast<int*>(order);
    memset(o, 0, sizeof(int) * HLGS_CUT_ORDER_HEADER);
    if (N == 0) return HLGS_OK;
    auto nd = [&](int v) { return nodes + 6 * (size_t)v; };
    // F*: the breadth-first frontiers with every node that has children expanding
    std::vector<int> fs{0}, lev{0};
    std::vector<char> seen(N, 0);
    seen[0] = 1;
    std::vector<int> first, second;
    for (size_t b = 0; b < fs.size();) {
        const size_t e = fs.size();
        first.clear();
        second.clear();
        for (size_t i = b; i < e; i++) {
            const int v = fs[i];
            if (nd(v)[kChildCount] == 0) continue;
            const int fc = nd(v)[kFirstChild];
            if (fc < 0 || fc >= N) return HLGS_OK;  // not walkable as the reference walks it: usable stays 0
            const int ns = nd(fc)[kNextSibling];
            if (ns >= N) return HLGS_OK;
            first.push_back(fc);
            if (ns >= 0) second.push_back(ns);
        }
        for (const std::vector<int>* part : {&first, &second})
            for (int c : *part) {
                if (seen[c]) return HLGS_OK;  // reached twice: not a tree
                seen[c] = 1;
                fs.push_back(c);
            }
        b = e;
        if (fs.size() > e) lev.push_back((int)e);  // the next level starts where this one ended
    }
    const int M = (int)fs.size(), levels = (int)lev.size();
    lev.push_back(M);
    if (M > HLGS_CUT_FLAT_MAX_ENTRIES || levels > HLGS_CUT_FLAT_MAX_LEVELS) return HLGS_OK;
    // preorder positions and subtree sizes of the walk's binary tree (children: first child, then its next sibling)
    std::vector<int> pos(N, -1), size(N, 1);
    for (int i = M - 1; i >= 0; i--) {  // children come after their parent in F*
        const int v = fs[i];
        if (nd(v)[kChildCount] == 0) continue;
        const int fc = nd(v)[kFirstChild], ns = nd(fc)[kNextSibling];
        size[v] += size[fc] + (ns >= 0 ? size[ns] : 0);
    }
    pos[0] = 0;
    for (int i = 0; i < M; i++) {
        const int v = fs[i];
        if (nd(v)[kChildCount] == 0) continue;
        const int fc = nd(v)[kFirstChild], ns = nd(fc)[kNextSibling];
        pos[fc] = pos[v] + 1;
        if (ns >= 0) pos[ns] = pos[v] + 1 + size[fc];
    }
    o[0] = M;
    o[1] = levels;
    o[2] = 1;
    o[3] = N;
    for (int l = 0; l <= levels; l++) o[4 + l] = lev[l];
    int* fn = o + HLGS_CUT_ORDER_HEADER;
    uint16_t* pre16 = reinterpret_cast<uint16_t*>(fn + ((2 * M + 3) & ~3));  // 16-byte aligned
    for (int i = 0; i < M; i++) {
        const int v = fs[i];
        fn[i] = v;
        fn[M + i] = pos[v] | (pos[v] + size[v]) << 16;  // both < 2^16 (M < 2^16)
        pre16[i] = (uint16_t)pos[v];
    }
    return HLGS_OK;
}

}  // extern "C"
