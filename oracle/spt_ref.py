"""CPU restatement of the upper-tree coarse cut of the SPT streaming step.

TEST INFRASTRUCTURE ONLY (tests/ import it as the checker of csrc/stream.hip's k_upper_cut).  Restates, as plain
Python over numpy arrays, GaussianModel.cut_hierarchy_on_condition with return_upper_tree=False, root_node=0 and
a leave_out_of_cut_condition (scene/gaussian_model.py:364-404), the frustum_cull_spheres condition
(:80-100) and the LOD distance condition of train_post.py:336: a level-by-level walk of a `stack` that is
filtered by the cull, sends leaves and then condition-false nodes to the cut, and continues with the first
children followed by the first children's next siblings.  float32 arithmetic in the reference's order.
"""
import numpy as np


def frustum_visible(p, r, planes):
    f = np.float32
    for pl in np.asarray(planes, np.float32):
        sd = f(f(f(p[0] * pl[0]) + f(p[1] * pl[1])) + f(p[2] * pl[2])) + pl[3]
        if f(sd + r) < 0:
            return False
    return True


def lod_expand(p, md2, cam, dmul):
    f = np.float32
    dx, dy, dz = f(cam[0] - p[0]), f(cam[1] - p[1]), f(cam[2] - p[2])
    d2 = f(f(f(dx * dx) + f(dy * dy)) + f(dz * dz))
    return md2 > f(d2 * f(dmul))


def upper_tree_cut(nodes, xyz, bounds, md2, planes, cam, dmul=1.0, use_frustum=True, use_lod=True):
    nodes = np.asarray(nodes)
    xyz = np.asarray(xyz, np.float32)
    stack = [0]
    cut = []
    while stack:
        if use_frustum:
            stack = [v for v in stack if frustum_visible(xyz[v], np.float32(bounds[v]), planes)]
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
