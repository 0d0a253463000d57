"""The SPT streaming step around the SPT cut: the per-view coarse cut of the upper tree and the
cache traffic of train_post.py's SPT cache, on the HIP path.

  extract_frustum_planes(view_proj)     scene/gaussian_model.py:54-78 (left/right/bottom/top planes, normalised)
  upper_tree_cut(...)                   cut_hierarchy_on_condition over the upper tree with frustum_cull_spheres
                                        and the LOD distance condition (gaussian_model.py:364-404;
                                        train_post.py:326-343), one workgroup on the GPU
  gather_rows(storage, idx) / scatter_rows(storage, idx, values)
                                        storage[idx].cuda() and storage[idx] = values.to(storage)
                                        (train_post.py:439-488); storage may be pinned host memory, which the GPU
                                        reads and writes directly
  build_hierarchical_spt(...)           GaussianModel.build_hierarchical_SPT (gaussian_model.py:184-332) in the
                                        library's host code
  spt_view_cut(...)                     the per-view cut of get_SPT_cut (gaussian_model.py:108-159): coarse cut,
                                        SPT leaves through get_spt_cut_cuda, the cut's non-leaf nodes
"""
import ctypes as C

import torch

from hlgs_core import _lib as L

# HierarchyNode columns (types.h:60-67)
CHILD_COUNT, FIRST_CHILD, NEXT_SIBLING, MAX_SIDE = 2, 3, 4, 5


def extract_frustum_planes(view_proj_matrix):
    m = view_proj_matrix.T
    planes = torch.stack([m[3] + m[0], m[3] - m[0], m[3] + m[1], m[3] - m[1]])
    planes /= torch.norm(planes[:, :3], dim=1, keepdim=True)
    return planes


def upper_tree_order(nodes, device=None):
    """The walk order of an upper tree for the flat coarse cut (hlgs_upper_tree_order, host code): a device int32
    blob, or None when the tree exceeds the flat cut's limits (65,535 nodes on the walk, 64 levels) or is not a tree
    as the reference walks it -- then the cut walks level by level."""
    lib = L.load()
    nd = nodes.detach().to("cpu", torch.int32).contiguous()
    N = int(nd.shape[0])
    blob = torch.zeros(((lib.hlgs_upper_tree_order_size(N) + 3) // 4,), dtype=torch.int32)
    L.check(lib.hlgs_upper_tree_order(N, L.ptr(nd) if N else None, L.ptr(blob)))
    if not int(blob[2]):
        return None
    return blob.to(device if device is not None else nodes.device)


def upper_tree_cut(nodes, xyz, bounds, min_distance_squared, planes, camera_position, distance_multiplier=1.0,
                   use_frustum=True, use_lod=True, order=None):
    """Coarse cut of the upper tree from root 0 (int32 device tensor, the reference's order).  order: the blob of
    upper_tree_order(nodes) for the flat cut (two launches), or None for the level walk; same result."""
    lib = L.load()
    nd = nodes.contiguous().to(torch.int32)
    p = xyz.contiguous().float()
    dev = p.device
    b = bounds.contiguous().float() if bounds is not None else None
    md = min_distance_squared.contiguous().float() if min_distance_squared is not None else None
    pl = planes.detach().to(device=dev, dtype=torch.float32).contiguous() if planes is not None else None
    cam = camera_position.detach().reshape(-1)[:3].to(device=dev, dtype=torch.float32).contiguous()
    L.require_gpu(nd, p)
    N = nd.size(0)
    cut = torch.empty((max(N, 1),), dtype=torch.int32, device=dev)
    scratch = torch.empty(lib.hlgs_upper_cut_scratch_size(N), dtype=torch.uint8, device=dev)
    if order is not None:
        cnt = torch.zeros((2,), dtype=torch.int32, device=dev)
        L.check(lib.hlgs_upper_tree_cut_views_ordered_device(
            N, L.ptr(nd), L.ptr(order), L.ptr(p), L.ptr(b), L.ptr(md), 1, L.ptr(pl), L.ptr(cam),
            float(distance_multiplier), int(bool(use_frustum)), int(bool(use_lod)), L.ptr(scratch), L.ptr(cut),
            L.ptr(cnt), L.stream()))
        n, overflow = (int(v) for v in cnt.cpu())
        if overflow:
            raise RuntimeError("hlgs: upper-tree cut: the order blob does not fit these nodes")
        return cut[:n]
    count = C.c_int(0)
    L.check(lib.hlgs_upper_tree_cut(N, L.ptr(nd), L.ptr(p), L.ptr(b), L.ptr(md), L.ptr(pl), L.ptr(cam),
                                    float(distance_multiplier), int(bool(use_frustum)), int(bool(use_lod)),
                                    L.ptr(scratch), L.ptr(cut), C.byref(count), L.stream()))
    return cut[:count.value]


def _rows(t):
    if not t.is_contiguous():
        raise RuntimeError("row storage must be contiguous")
    n = t.size(0)
    rb = t.element_size() * (t.numel() // n if n else 0)
    return rb


def gather_rows(storage, idx, out=None, device="cuda"):
    """out[i] = storage[idx[i]] (rows of the first dimension) on the GPU; storage on the device or pinned host."""
    lib = L.load()
    i = idx.to(device=device, dtype=torch.int64).contiguous()
    if out is None:
        out = torch.empty((i.numel(),) + tuple(storage.shape[1:]), dtype=storage.dtype, device=device)
    if storage.device.type == "cpu" and not storage.is_pinned():
        raise RuntimeError("host storage must be pinned (tensor.pin_memory()) for direct GPU access")
    L.check(lib.hlgs_gather_rows(i.numel(), _rows(storage), L.ptr(i), L.ptr(storage), L.ptr(out), L.stream()))
    return out


def scatter_rows(storage, idx, values):
    """storage[idx[i]] = values[i] on the GPU; storage on the device or pinned host."""
    lib = L.load()
    v = values.contiguous()
    i = idx.to(device=v.device, dtype=torch.int64).contiguous()
    if storage.device.type == "cpu" and not storage.is_pinned():
        raise RuntimeError("host storage must be pinned (tensor.pin_memory()) for direct GPU access")
    if v.dtype != storage.dtype or _rows(storage) != _rows(v):
        raise RuntimeError("values rows must match the storage rows")
    L.check(lib.hlgs_scatter_rows(i.numel(), _rows(storage), L.ptr(i), L.ptr(v), L.ptr(storage), L.stream()))


def spt_view_cut(upper_tree_nodes, upper_tree_xyz, bounds, min_distance_squared, view_proj, camera_position,
                 SPT_gaussian_indices, SPT_starts, SPT_max, SPT_min, skybox_points=0, distance_multiplier=1.0,
                 use_frustum=True, use_lod=False):
    """Body of GaussianModel.get_SPT_cut (gaussian_model.py:108-159) on the HIP path: the coarse cut of the upper
    tree (its LOD condition is disabled there, :124, hence use_lod=False), then the render indices
    [skybox range, get_spt_cut_cuda of the cut's SPT leaves, Gaussians of the cut's non-leaf nodes].
    Returns the reference's triple (render_indices, Gaussian ids of the SPT roots, SPT distances)."""
    import gaussian_hierarchy as GH
    planes = extract_frustum_planes(view_proj) if use_frustum else None
    coarse = upper_tree_cut(upper_tree_nodes, upper_tree_xyz, bounds, min_distance_squared, planes, camera_position,
                            distance_multiplier, use_frustum, use_lod).long()
    nodes = upper_tree_nodes
    leaf_mask = nodes[coarse, CHILD_COUNT] == 0
    leaf_nodes = coarse[leaf_mask]
    spt_leaf = nodes[leaf_nodes, FIRST_CHILD] >= 0
    SPT_indices = nodes[leaf_nodes][spt_leaf, FIRST_CHILD]
    SPT_node_indices = leaf_nodes[spt_leaf]
    cam = camera_position.reshape(-1)[:3].to(upper_tree_xyz.device)
    SPT_distances = (upper_tree_xyz[SPT_node_indices] - cam).pow(2).sum(1).sqrt()
    dev = upper_tree_xyz.device
    cut, _counts = GH.get_spt_cut_cuda(len(SPT_indices), SPT_gaussian_indices, SPT_starts, SPT_max, SPT_min,
                                       SPT_indices.to(torch.int32), SPT_distances)
    render = torch.cat([torch.arange(0, skybox_points, device=dev, dtype=torch.int32), cut,
                        nodes[coarse[~leaf_mask], MAX_SIDE].to(torch.int32)])
    return render, nodes[SPT_node_indices, MAX_SIDE], SPT_distances


def build_hierarchical_spt(nodes, xyz, scaling, root, SPT_Root_Volume, target_granularity, min_SPT_Size=100,
                           use_bounding_spheres=True):
    """SPTs and upper tree of a dynamic hierarchy (nodes (G,6) int32, xyz (G,3), scaling (G,3) unactivated
    log-scales).  Returns a dict of CPU tensors: SPT_starts, SPT_max, SPT_min, SPT_gaussian_indices,
    SPT_root_hierarchy_indices, upper_tree_nodes, upper_tree_xyz, upper_tree_scaling, min_distance_squared,
    bounding_sphere_radii (None without bounding spheres)."""
    lib = L.load()
    nd = nodes.detach().to("cpu", torch.int32).contiguous()
    p = xyz.detach().to("cpu", torch.float32).contiguous()
    sc = scaling.detach().to("cpu", torch.float32).contiguous()
    h = C.c_void_p()
    L.check(lib.hlgs_spt_build(nd.size(0), L.ptr(nd), L.ptr(p), L.ptr(sc), int(root), float(SPT_Root_Volume),
                               float(target_granularity), int(min_SPT_Size), int(bool(use_bounding_spheres)),
                               C.byref(h)))
    try:
        ns, ne, nu = C.c_int(), C.c_int(), C.c_int()
        L.check(lib.hlgs_spt_result_sizes(h, C.byref(ns), C.byref(ne), C.byref(nu)))
        i32 = lambda *s: torch.empty(s, dtype=torch.int32)  # noqa: E731
        f32 = lambda *s: torch.empty(s, dtype=torch.float32)  # noqa: E731
        out = dict(SPT_starts=i32(ns.value + 1), SPT_max=f32(ne.value), SPT_min=f32(ne.value),
                   SPT_gaussian_indices=i32(ne.value), SPT_root_hierarchy_indices=i32(ns.value),
                   upper_tree_nodes=i32(nu.value, 6), upper_tree_xyz=f32(nu.value, 3),
                   upper_tree_scaling=f32(nu.value, 3), min_distance_squared=f32(nu.value),
                   bounding_sphere_radii=f32(nu.value) if use_bounding_spheres else None)
        order = ("SPT_starts", "SPT_max", "SPT_min", "SPT_gaussian_indices", "SPT_root_hierarchy_indices",
                 "upper_tree_nodes", "upper_tree_xyz", "upper_tree_scaling", "min_distance_squared",
                 "bounding_sphere_radii")
        L.check(lib.hlgs_spt_result_copy(h, *[L.ptr(out[k]) if out[k] is not None else None for k in order]))
    finally:
        lib.hlgs_spt_result_free(h)
    return out
