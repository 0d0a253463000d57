"""CPU restatement of the upper-tree coarse cut of the SPT streaming step.

TEST INFRASTRUCTURE ONLY (tests/ import it as the checker of csrc/stream.hip's k_upper_cut).  Restates, as plain
Python over numpy arrays, GaussianModel.cut_hierarchy_on_condition with return_upper_tree=False, root_node=0 and
a leave_out_of_cut_condition (scene/gaussian_model.py:364-404), the frustum_cull_spheres condition
(:80-100) and the LOD distance condition of train_post.py:336: a level-by-level walk of a `stack` that is
filtered by the cull, sends leaves and then condition-false nodes to the cut, and continues with the first
children followed by the first children's next siblings.  float32 arithmetic in the reference's order.

Also restated here (same status: checkers of csrc/stream.hip and csrc/optim.hip, never the product path):
  cache_pass   one pass of train_post.py's SPT-cache bookkeeping (:346-430) -- searchsorted of the previous
               SPTs in the (unsorted) new list, isclose reuse test, Python-slice segment marks, isin, the
               SPT_counts prefix, and the keep / write-back split of render_indices
  adam_dense   OurAdam._single_tensor_adam2 (scene/OurAdam.py:357-448) with the skybox gradient rows zeroed
               (train_post.py:786-791), as float32 torch ops on the CPU
"""
import numpy as np


def frustum_visible(p, r, planes):
    f = np.float32
    for pl in np.asarray(planes, np.float32):
        sd = f(f(f(p[0] * pl[0]) + f(p[1] * pl[1])) + f(p[2] * pl[2])) + pl[3]
        if f(sd + r) < 0:
            return False
    return True


def _d2(p, c):
    f = np.float32
    dx, dy, dz = f(c[0] - p[0]), f(c[1] - p[1]), f(c[2] - p[2])
    return f(f(f(dx * dx) + f(dy * dy)) + f(dz * dz))


def lod_expand(p, md2, cam, dmul):
    """cam: one camera (3,) or a batch of views (G, 3): the nearest camera's squared distance decides."""
    f = np.float32
    d2 = min(_d2(p, c) for c in np.asarray(cam, np.float32).reshape(-1, 3))
    return md2 > f(d2 * f(dmul))


def upper_tree_cut(nodes, xyz, bounds, md2, planes, cam, dmul=1.0, use_frustum=True, use_lod=True):
    """planes (4, 4) and cam (3,) for one view, or (G, 4, 4) and (G, 3) for the union cut of a batch of views
    (visible in any frustum, nearest camera for the LOD condition; DESIGN §7 -- the reference trains one view per
    step, so the batch form has no counterpart there and reduces to it for G = 1)."""
    nodes = np.asarray(nodes)
    xyz = np.asarray(xyz, np.float32)
    pls = None if planes is None else np.asarray(planes, np.float32).reshape(-1, 4, 4)
    stack = [0]
    cut = []
    while stack:
        if use_frustum:
            stack = [v for v in stack if any(frustum_visible(xyz[v], np.float32(bounds[v]), pl) for pl in pls)]
        cut += [v for v in stack if nodes[v, 2] == 0]
        stack = [v for v in stack if nodes[v, 2] > 0]
        if use_lod:
            keep = [lod_expand(xyz[v], np.float32(md2[v]), cam, dmul) for v in stack]
        else:
            keep = [True] * len(stack)
        cut += [v for v, k in zip(stack, keep) if not k]
        stack = [v for v, k in zip(stack, keep) if k]
        first = [int(nodes[v, 3]) for v in stack]
        second = [int(nodes[c, 4]) for c in first]
        stack = first + second
    return np.array(cut, np.int32)


# ---------------------------------------------------------------------------------------------------------------
# SPT construction: GaussianModel.build_hierarchical_SPT / get_min_distance / cut_hierarchy_on_condition
# (scene/gaussian_model.py:184-404) restated with CPU torch float32 tensor operations in the reference's order
# (the reference runs the same operations on the GPU, one SPT at a time).  Sorting uses stable=True (the
# reference's argsort on the device is a stable radix sort).  Parity is against this restatement only: the
# reference ships no hierarchy data and its method needs a CUDA device.
def _min_distance(nodes, scaling, idx, tg):
    import torch
    if idx.numel() == 1:
        i = int(idx.reshape(-1)[0])
        if nodes[i, 2] == 0:
            return torch.tensor(-1000000.0)
        s = torch.exp(scaling[i])
        return torch.sqrt(s[0] * s[1] + s[0] * s[2] + s[1] * s[2]) / tg
    leaves = nodes[idx, 2] == 0
    s = torch.exp(scaling[idx])
    md = torch.sqrt(s[:, 0] * s[:, 1] + s[:, 0] * s[:, 2] + s[:, 1] * s[:, 2]) / tg
    md[leaves] = -1000000000
    return md


def build_spt(nodes, xyz, scaling, root, volume, tg, min_size=100, use_bounding_spheres=True):
    import torch
    nodes = torch.as_tensor(nodes, dtype=torch.int64)
    xyz = torch.as_tensor(xyz, dtype=torch.float32)
    scaling = torch.as_tensor(scaling, dtype=torch.float32)
    # cut_hierarchy_on_condition(nodes, prod(exp(scale)) > volume, root_node=root)
    stack = torch.tensor([root])
    upper = torch.empty(0, dtype=torch.int64)
    cut = torch.empty(0, dtype=torch.int64)
    while len(stack) > 0:
        upper = torch.cat((upper, stack))
        cut = torch.cat((cut, stack[nodes[stack, 2] == 0]))
        stack = stack[nodes[stack, 2] > 0]
        mask = torch.prod(torch.exp(scaling[stack]), dim=-1) > volume
        cut = torch.cat((cut, stack[~mask]))
        stack = stack[mask]
        fc = nodes[stack, 3]
        stack = torch.cat((fc, nodes[fc, 4]))
    starts, smax, smin, gidx, roots, leaf_children, spt_nodes, radii_list = [0], [], [], [], [], [], [], []
    for cn in cut.tolist():
        if nodes[cn, 2] == 0:
            continue
        centre = xyz[cn]
        spt = torch.zeros(1, 3)
        spt[0, 0] = cn
        spt[0, 1] = _min_distance(nodes, scaling, torch.tensor(cn), tg)
        spt[0, 2] = 1000000000000
        ids = [cn]
        st = torch.tensor([cn])
        maxd = spt[0, 1:2].clone()
        bsr = float(torch.max(torch.exp(scaling[cn])) * 3.0)
        extra = []
        while len(st) > 0:
            fc = nodes[st, 3]
            sc = nodes[fc, 4]
            st = torch.cat((fc, sc))
            st = st[st > 0]
            if len(st) == 0:
                break
            cdist = torch.sqrt(torch.sum((xyz[st] - centre) ** 2, dim=1))
            bsr = max(bsr, float(torch.max(cdist + torch.max(torch.exp(scaling[st]), dim=-1)[0] * 3)))
            maxd = maxd[fc > 0]
            mind = _min_distance(nodes, scaling, st, tg) + cdist
            maxd = torch.cat((maxd, maxd))
            rows = torch.zeros(len(st), 3)
            rows[:, 0] = st.float()
            rows[:, 1] = torch.where(mind < maxd, mind, maxd)
            rows[:, 2] = maxd
            maxd = rows[:, 1].clone()
            spt = torch.cat((spt, rows))
            ids += st.tolist()
            extra += st.tolist()
        if len(spt) > min_size:
            radii_list.append(bsr)
            order = torch.argsort(spt[:, -1], descending=True, stable=True)
            leaf_children.append(len(roots))
            spt_nodes.append(cn)
            starts.append(starts[-1] + len(spt))
            smax.append(spt[order, 2])
            smin.append(spt[order, 1])
            gidx.append(torch.tensor(ids)[order])
            roots.append(cn)
        else:
            upper = torch.cat((upper, torch.tensor(extra, dtype=torch.int64)))
    upper = torch.sort(upper)[0]
    un = nodes[upper].clone()
    cut_spt = torch.searchsorted(upper, torch.tensor(spt_nodes, dtype=torch.int64))
    un[cut_spt, 2] = 0
    un[cut_spt, 3] = torch.tensor(leaf_children, dtype=torch.int64)
    uxyz, uscale = xyz[upper], scaling[upper]
    un[:, 5] = upper
    un[:, 1] = torch.searchsorted(upper, un[:, 1].contiguous())
    un[0, 1] = -1
    non_leaf = ~torch.isin(torch.arange(len(un)), cut_spt)
    fcs = un[non_leaf, 3]
    un[non_leaf, 3] = torch.where(fcs == 0, torch.full_like(fcs, -1), torch.searchsorted(upper, fcs))
    fs = un[:, 4] > 0
    un[fs, 4] = torch.searchsorted(upper, un[fs, 4])
    parents = un[un[:, 1], 5]
    md2 = _min_distance(nodes, scaling, parents, tg).square()
    md2[0] = 1000000000000
    radii = None
    if use_bounding_spheres:
        radii = torch.zeros(len(un))
        leaves = torch.where(un[:, 3] == -1)[0]
        radii[leaves] = torch.max(torch.exp(uscale[leaves]), dim=-1)[0] * 3
        radii[cut_spt] = torch.tensor(radii_list, dtype=torch.float32)
        level = torch.where(un[:, 2] == 0)[0]
        while level.numel():
            par = un[level, 1]
            par = par[par >= 0]
            f = un[par, 3]
            s = un[f, 4]
            df = (uxyz[par] - uxyz[f]).square().sum(1).sqrt()
            ds = (uxyz[par] - uxyz[s]).square().sum(1).sqrt()
            radii[par] = torch.maximum(radii[f] + df, radii[s] + ds)
            level = par
    cat = lambda xs, dt: torch.cat(xs).to(dt) if xs else torch.empty(0, dtype=dt)  # noqa: E731
    return dict(SPT_starts=torch.tensor(starts, dtype=torch.int32), SPT_max=cat(smax, torch.float32),
                SPT_min=cat(smin, torch.float32), SPT_gaussian_indices=cat(gidx, torch.int32),
                SPT_root_hierarchy_indices=torch.tensor(roots, dtype=torch.int32), upper_tree_nodes=un.to(torch.int32),
                upper_tree_xyz=uxyz, upper_tree_scaling=uscale, min_distance_squared=md2, bounding_sphere_radii=radii)


# ---------------------------------------------------------------- SPT cache (train_post.py:346-430)
def lower_bound(arr, v):
    """torch.searchsorted(arr, v) (right=False): a plain lower-bound binary search over arr as it is given."""
    lo, hi = 0, len(arr)
    while lo < hi:
        mid = lo + ((hi - lo) >> 1)
        if not arr[mid] >= v:
            lo = mid + 1
        else:
            hi = mid
    return lo


def isclose32(a, b, rtol, atol):
    """torch.isclose on float32 scalars: a == b, or finite |a - b| <= atol + |rtol * b| (scalars in float32)."""
    f = np.float32
    a, b = f(a), f(b)
    if a == b:
        return True
    err = f(abs(f(a - b)))
    allowed = f(f(atol) + f(abs(f(f(rtol) * b))))
    return bool(np.isfinite(err) and err <= allowed)


def spt_distances(xyz, cam, dmul):
    """(upper_tree_xyz[i] - camera_position).pow(2).sum(1).sqrt() * distance_multiplier, float32; for a batch of
    views (cam G x 3) the nearest camera's distance."""
    best = None
    for c in np.asarray(cam, np.float32).reshape(-1, 3):
        d = (np.asarray(xyz, np.float32) - c).astype(np.float32)
        q = (d * d).astype(np.float32)
        s = ((q[:, 0] + q[:, 1]).astype(np.float32) + q[:, 2]).astype(np.float32)
        best = s if best is None else np.minimum(best, s)
    return (np.sqrt(best).astype(np.float32) * np.float32(dmul)).astype(np.float32)


def cache_pass(nodes, xyz, coarse, cam, dmul, prev_idx, prev_dist, prev_counts, render, n_loaded_prev, sky, rtol,
               atol, spt_cut):
    """One pass of the SPT cache bookkeeping.  spt_cut(load_idx, load_dist) -> (cut, counts_prefix) is
    get_spt_cut_cuda's restatement.  Returns a dict of numpy arrays named after the reference's variables."""
    nodes = np.asarray(nodes)
    coarse = np.asarray(coarse, np.int64)
    leaf_nodes = coarse[nodes[coarse, 2] == 0]
    fc = nodes[leaf_nodes, 3]
    spt_idx = fc[fc >= 0].astype(np.int32)
    spt_nodes = leaf_nodes[fc >= 0]
    upper = nodes[leaf_nodes[fc <= 0], 5].astype(np.int32)
    dist = spt_distances(np.asarray(xyz)[spt_nodes].reshape(-1, 3), cam, dmul)
    m, R = len(prev_idx), len(render)
    tail_end = R - n_loaded_prev
    kept = []
    for j in range(m):
        pos = lower_bound(spt_idx, prev_idx[j])
        if pos < len(spt_idx) and spt_idx[pos] == prev_idx[j] and isclose32(dist[pos], prev_dist[j], rtol, atol):
            kept.append(j)
    seg_end = lambda j: int(prev_counts[j + 1]) if j + 1 < m else tail_end  # noqa: E731
    keep = np.zeros(R, bool)
    for j in kept:
        keep[int(prev_counts[j]):seg_end(j)] = True
    keep[:sky] = True
    keep_idx = np.asarray([prev_idx[j] for j in kept], np.int32)
    keep_dist = np.asarray([prev_dist[j] for j in kept], np.float32)
    load = ~np.isin(spt_idx, keep_idx)
    load_idx, load_dist = spt_idx[load], dist[load]
    if len(load_idx):
        cut, counts = spt_cut(load_idx, load_dist)
    else:
        cut, counts = np.zeros(0, np.int32), np.zeros(0, np.int32)
    counts = np.asarray(counts, np.int64) + sky
    prefix, keep_counts = 0, []
    for j in kept:
        keep_counts.append(prefix)
        prefix += seg_end(j) - int(prev_counts[j])
    render = np.asarray(render, np.int32)
    load_from_disk = np.concatenate([np.asarray(cut, np.int32), upper]).astype(np.int32)
    return dict(SPT_indices=np.concatenate([keep_idx, load_idx]).astype(np.int32),
                SPT_distances=np.concatenate([keep_dist, load_dist]).astype(np.float32),
                SPT_counts=np.concatenate([np.asarray(keep_counts, np.int64), counts + prefix]).astype(np.int32),
                keep_mask=keep, write_back_indices=render[~keep], load_from_disk_indices=load_from_disk,
                render_indices=np.concatenate([render[keep], load_from_disk]).astype(np.int32),
                n_kept=len(kept), load_SPT_indices=load_idx, upper_tree_nodes_to_render=upper, prefix=prefix)


# ---------------------------------------------------------------- dense Adam (train_post.py:786-812)
def adam_dense(param, grad, exp_avg, exp_avg_sq, lr, step, sky, beta1=0.9, beta2=0.999, eps=1e-8):
    """In-place float32 torch CPU ops of OurAdam._single_tensor_adam2 (maximize=False, weight_decay=0,
    amsgrad=False, capturable=False) after grad[:sky] = 0; step is the incremented state step."""
    import math
    grad[:sky] = 0
    exp_avg.mul_(beta1).add_(grad, alpha=1 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
    step_size = lr / (1 - beta1 ** step)
    denom = (exp_avg_sq.sqrt() / math.sqrt(1 - beta2 ** step)).add_(eps)
    param.addcdiv_(exp_avg, denom, value=-step_size)
