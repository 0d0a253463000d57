"""SPT streaming step on the HIP path (csrc/stream.hip): the upper-tree coarse cut against the CPU restatement
(oracle/spt_ref.py), bit-exact (same nodes, same order), and the row gather / scatter of the cache against
plain indexing, with pinned host storage read and written directly by the GPU."""
import numpy as np
import pytest
import torch

from hlgs_core import synthetic as S
from oracle import spt_ref as SR

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _upper_tree(n=3000, seed=0):
    cam = S.make_camera(256, 192)
    h = S.make_dynamic_hierarchy(S.make_gaussians(n, 0, cam, seed=seed), seed=seed)
    nodes = h["nodes"].copy()
    nodes[:, 3] = np.where(nodes[:, 2] == 0, -1, nodes[:, 3])  # upper-tree convention: plain leaves have -1
    xyz = h["means3D"]
    bounds = (h["scales"].max(1) * 3.0).astype(np.float32)
    rng = np.random.default_rng(seed)
    md2 = (np.square(h["scales"].max(1) / 0.004) * rng.uniform(0.5, 2.0, len(nodes))).astype(np.float32)
    return nodes, xyz, bounds, md2


@pytest.mark.parametrize("seed,dmul,frustum,lod", [(0, 1.0, True, True), (1, 2.0, True, True), (2, 1.0, False, True),
                                                   (3, 1.0, True, False)])
def test_upper_tree_cut_matches_reference_walk(seed, dmul, frustum, lod):
    from hlgs_core import spt
    nodes, xyz, bounds, md2 = _upper_tree(3000 + 500 * seed, seed)
    R = np.eye(3)
    ang = 0.3 * seed
    R[0, 0], R[0, 2], R[2, 0], R[2, 2] = np.cos(ang), np.sin(ang), -np.sin(ang), np.cos(ang)
    cam = S.make_camera(320, 240, R=R, T=np.array([0.1 * seed, 0.0, 0.5]))
    planes = spt.extract_frustum_planes(cam["projmatrix"])
    t = lambda a: torch.tensor(a, device=DEV)  # noqa: E731
    got = spt.upper_tree_cut(t(nodes), t(xyz), t(bounds), t(md2), planes, cam["campos"], dmul, frustum, lod)
    want = SR.upper_tree_cut(nodes, xyz, bounds, md2, planes.numpy(), cam["campos"].numpy(), dmul, frustum, lod)
    assert 0 < len(want) < len(nodes)
    np.testing.assert_array_equal(got.cpu().numpy(), want)
    # the flat cut (k_cut_flat_eval + k_cut_flat_place) from the precomputed walk order: the same nodes in the same order
    order = spt.upper_tree_order(t(nodes))
    assert order is not None
    flat = spt.upper_tree_cut(t(nodes), t(xyz), t(bounds), t(md2), planes, cam["campos"], dmul, frustum, lod,
                              order=order)
    np.testing.assert_array_equal(flat.cpu().numpy(), want)


def test_flat_cut_refuses_another_trees_blob():
    """A walk-order blob built for another tree: its entry count and node ids do not belong to these
    nodes, so the flat cut reports it (count[1]) instead of placing a cut with holes or reading nodes past N."""
    from hlgs_core import spt
    nodes, xyz, bounds, md2 = _upper_tree(3000, 0)
    big, *_ = _upper_tree(3500, 1)
    cam = S.make_camera(320, 240, T=np.array([0.0, 0.0, 0.5]))
    planes = spt.extract_frustum_planes(cam["projmatrix"])
    t = lambda a: torch.tensor(a, device=DEV)  # noqa: E731
    for other in (big, nodes[: len(nodes) // 2 * 2 - 1]):
        order = spt.upper_tree_order(t(other))
        if order is None:
            continue
        assert int(order[3]) == len(other) != len(nodes)
        with pytest.raises(RuntimeError, match="order blob"):
            spt.upper_tree_cut(t(nodes), t(xyz), t(bounds), t(md2), planes, cam["campos"], 1.0, True, True,
                               order=order)
    # its own blob still cuts
    own = spt.upper_tree_order(t(nodes))
    want = SR.upper_tree_cut(nodes, xyz, bounds, md2, planes.numpy(), cam["campos"].numpy(), 1.0, True, True)
    got = spt.upper_tree_cut(t(nodes), t(xyz), t(bounds), t(md2), planes, cam["campos"], 1.0, True, True, order=own)
    np.testing.assert_array_equal(got.cpu().numpy(), want)


@pytest.mark.parametrize("n,frustum,lod", [(40000, False, False), (40000, True, True), (300000, False, False),
                                           (30000, False, False), (30000, True, True)])
def test_upper_tree_cut_wide_levels(n, frustum, lod):
    """Levels wider than the single-workgroup walk's 1,024 entries run as multi-workgroup launches (k_cut_level);
    300k leaves give nine such levels, one more than are queued, so the resume walk finishes the last one.  The
    30k-leaf trees (59,999 nodes) are within the flat cut's 65,535 entries: its thread runs span several levels."""
    from hlgs_core import spt
    nodes, xyz, bounds, md2 = _upper_tree(n, 7)
    cam = S.make_camera(320, 240, T=np.array([0.05, 0.0, 0.3]))
    planes = spt.extract_frustum_planes(cam["projmatrix"])
    t = lambda a: torch.tensor(a, device=DEV)  # noqa: E731
    got = spt.upper_tree_cut(t(nodes), t(xyz), t(bounds), t(md2), planes, cam["campos"], 1.0, frustum, lod)
    want = SR.upper_tree_cut(nodes, xyz, bounds, md2, planes.numpy(), cam["campos"].numpy(), 1.0, frustum, lod)
    assert len(want) > 2048
    np.testing.assert_array_equal(got.cpu().numpy(), want)
    order = spt.upper_tree_order(t(nodes))
    if len(nodes) > 65535:  # beyond the flat cut's entries: the level walk serves it
        assert order is None
        return
    flat = spt.upper_tree_cut(t(nodes), t(xyz), t(bounds), t(md2), planes, cam["campos"], 1.0, frustum, lod,
                              order=order)
    np.testing.assert_array_equal(flat.cpu().numpy(), want)


@pytest.mark.parametrize("width,dtype", [(3, torch.float32), (45, torch.float32), (4, torch.float32),
                                         (6, torch.int32), (1, torch.float32)])
def test_gather_scatter_rows_with_pinned_host_storage(width, dtype):
    from hlgs_core import spt
    rng = np.random.default_rng(width)
    P, n = 20000, 5000
    host = torch.tensor(rng.normal(size=(P, width)) * 100).to(dtype).pin_memory()
    idx = torch.tensor(rng.choice(P, n, replace=False), device=DEV)
    got = spt.gather_rows(host, idx)
    assert torch.equal(got.cpu(), host[idx.cpu()])
    vals = (got * 2 + 1).to(dtype)
    spt.scatter_rows(host, idx, vals)
    torch.cuda.synchronize()
    assert torch.equal(host[idx.cpu()], vals.cpu())
    dev_store = torch.zeros((P, width), dtype=dtype, device=DEV)
    spt.scatter_rows(dev_store, idx, vals)
    assert torch.equal(spt.gather_rows(dev_store, idx), vals)


def test_spt_view_cut_matches_restatement():
    """SPTs built in host code, then one view's get_SPT_cut body on the GPU (coarse cut + get_spt_cut_cuda +
    non-leaf upper-tree Gaussians) against the CPU restatements of both steps."""
    from hlgs_core import spt
    from oracle import oracle as O
    sky = 4
    cam0 = S.make_camera(256, 192)
    h = S.make_dynamic_hierarchy(S.make_gaussians(6000, 0, cam0, seed=8), skybox_points=sky, seed=8)
    nodes = torch.tensor(h["nodes"])
    nodes[:, 3] = torch.where(nodes[:, 2] == 2, nodes[:, 3], torch.zeros_like(nodes[:, 3]))
    b = spt.build_hierarchical_spt(nodes, torch.tensor(h["means3D"]), torch.log(torch.tensor(h["scales"])), sky, 3.0,
                                   0.02, 20)
    assert len(b["SPT_root_hierarchy_indices"]) > 5
    cam = S.make_camera(320, 240, T=np.array([0.05, 0.0, 0.3]))
    d = {k: (v.to(DEV) if v is not None else None) for k, v in b.items()}
    render, roots, dist = spt.spt_view_cut(d["upper_tree_nodes"], d["upper_tree_xyz"], d["bounding_sphere_radii"],
                                           d["min_distance_squared"], cam["projmatrix"], cam["campos"],
                                           d["SPT_gaussian_indices"], d["SPT_starts"], d["SPT_max"], d["SPT_min"],
                                           skybox_points=sky)
    un = b["upper_tree_nodes"].numpy()
    planes = spt.extract_frustum_planes(cam["projmatrix"]).numpy()
    coarse = SR.upper_tree_cut(un, b["upper_tree_xyz"].numpy(), b["bounding_sphere_radii"].numpy(),
                               b["min_distance_squared"].numpy(), planes, cam["campos"].numpy(), 1.0, True, False)
    leaf = un[coarse, 2] == 0
    lv = coarse[leaf]
    sptl = un[lv, 3] >= 0
    sidx = un[lv][sptl, 3]
    sdist = np.sqrt(((b["upper_tree_xyz"].numpy()[lv[sptl]] - cam["campos"].numpy()) ** 2).sum(1)).astype(np.float32)
    cut_o, _ = O.spt_cut(b["SPT_gaussian_indices"].numpy(), b["SPT_starts"].numpy(), b["SPT_max"].numpy(),
                         b["SPT_min"].numpy(), sidx, sdist, compat=True)
    want = np.concatenate([np.arange(sky), cut_o, un[coarse[~leaf], 5]]).astype(np.int32)
    assert len(want) > sky
    np.testing.assert_array_equal(render.cpu().numpy(), want)
    np.testing.assert_array_equal(roots.cpu().numpy(), un[lv[sptl], 5])
