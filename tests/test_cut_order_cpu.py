"""The flat coarse cut (round 5): the upper tree's walk order (hlgs_upper_tree_order, host code in
csrc/spt_build.cpp) and the placement k_cut_flat_eval / k_cut_flat_place apply to it, simulated on the CPU from the
blob word by word, against the reference walk restated in oracle/spt_ref.py (upper_tree_cut: the frontier of
scene/gaussian_model.py:364-404).  The GPU kernels are checked against the same oracle in tests/test_gpu_stream.py."""
import numpy as np
import pytest
import torch

from hlgs_core import spt
from hlgs_core import synthetic as S
from oracle import spt_ref as SR

HEADER = 80  # HLGS_CUT_ORDER_HEADER


def _upper_tree(n, seed):
    cam = S.make_camera(256, 192)
    h = S.make_dynamic_hierarchy(S.make_gaussians(n, 0, cam, seed=seed), seed=seed)
    nodes = h["nodes"].copy()
    nodes[:, 3] = np.where(nodes[:, 2] == 0, -1, nodes[:, 3])  # upper-tree convention: plain leaves have -1
    xyz = h["means3D"]
    bounds = (h["scales"].max(1) * 3.0).astype(np.float32)
    rng = np.random.default_rng(seed)
    md2 = (np.square(h["scales"].max(1) / 0.004) * rng.uniform(0.5, 2.0, len(nodes))).astype(np.float32)
    return nodes, xyz, bounds, md2


def _blob(nodes):
    b = spt.upper_tree_order(torch.tensor(nodes, dtype=torch.int32), device="cpu")
    return None if b is None else b.numpy()


def _flat_cut(blob, nodes, xyz, bounds, md2, planes, cam, dmul, frustum, lod):
    """k_cut_flat_eval + k_cut_flat_place restated over the blob."""
    M, nlev = int(blob[0]), int(blob[1])
    ls = blob[4:5 + nlev].astype(np.int64)
    fn = blob[HEADER:HEADER + M]
    pe = blob[HEADER + M:HEADER + 2 * M].astype(np.int64) & 0xFFFFFFFF
    pre, end = pe & 0xFFFF, pe >> 16
    off = HEADER + ((2 * M + 3) & ~3)
    pre16 = blob[off:off + (M + 1) // 2].view(np.uint16)[:M]
    np.testing.assert_array_equal(pre16, pre)
    st = np.empty(M, np.int64)
    for i, v in enumerate(fn):  # cut_node: 0 culled, 1 leaf, 2 condition false, 3 expand
        s = 3
        if frustum and not any(SR.frustum_visible(xyz[v], np.float32(bounds[v]), pl) for pl in planes):
            s = 0
        if s == 3 and nodes[v, 2] == 0:
            s = 1
        if s == 3 and lod and not SR.lod_expand(xyz[v], np.float32(md2[v]), cam, dmul):
            s = 2
        st[i] = s
    endv = np.zeros(M, np.int64)
    endv[pre] = np.where(st == 3, 0, end)
    excl = np.maximum.accumulate(np.concatenate([[0], endv[:-1]]))  # max scan over preorder
    covered = excl > np.arange(M)
    alive = ~covered[pre]
    leaf, stop = alive & (st == 1), alive & (st == 2)
    P1 = np.concatenate([[0], np.cumsum(leaf)])
    P2 = np.concatenate([[0], np.cumsum(stop)])
    lev = np.searchsorted(ls, np.arange(M), side="right") - 1  # level of each entry
    out = np.full(int(P1[-1] + P2[-1]), -1, np.int64)
    i = np.arange(M)
    out[P2[ls[lev[leaf]]] + P1[i[leaf]]] = fn[leaf]  # a leaf: stops before its level + leaves before it
    out[P1[ls[lev[stop] + 1]] + P2[i[stop]]] = fn[stop]  # a stop: leaves to its level's end + stops before it
    assert (out >= 0).all()
    return out.astype(np.int32)


@pytest.mark.parametrize("seed,dmul,frustum,lod", [(0, 1.0, True, True), (1, 2.0, True, True), (2, 1.0, False, True),
                                                   (3, 1.0, True, False), (4, 0.5, False, False),
                                                   (5, 1e9, True, True)])
def test_flat_cut_restatement_matches_reference_walk(seed, dmul, frustum, lod):
    nodes, xyz, bounds, md2 = _upper_tree(2000 + 500 * seed, seed)
    blob = _blob(nodes)
    assert blob is not None and blob[2] == 1 and blob[0] == len(nodes)  # every node of this tree is on the walk
    assert blob[3] == len(nodes)  # the node count it was built for (the kernels refuse another tree's blob)
    R = np.eye(3)
    ang = 0.3 * seed
    R[0, 0], R[0, 2], R[2, 0], R[2, 2] = np.cos(ang), np.sin(ang), -np.sin(ang), np.cos(ang)
    cam = S.make_camera(320, 240, R=R, T=np.array([0.1 * seed, 0.0, 0.5]))
    planes = spt.extract_frustum_planes(cam["projmatrix"]).numpy()
    want = SR.upper_tree_cut(nodes, xyz, bounds, md2, planes, cam["campos"].numpy(), dmul, frustum, lod)
    got = _flat_cut(blob, nodes, xyz, bounds, md2, planes.reshape(1, 4, 4), cam["campos"].numpy(), dmul, frustum, lod)
    assert len(want) > 0
    np.testing.assert_array_equal(got, want)


def test_order_blob_levels_and_preorder():
    nodes, *_ = _upper_tree(3000, 11)
    blob = _blob(nodes)
    M, nlev = int(blob[0]), int(blob[1])
    ls = blob[4:5 + nlev]
    assert ls[0] == 0 and ls[-1] == M and (np.diff(ls) > 0).all()
    fn = blob[HEADER:HEADER + M]
    assert fn[0] == 0 and sorted(fn.tolist()) == list(range(len(nodes)))
    pe = blob[HEADER + M:HEADER + 2 * M].astype(np.int64) & 0xFFFFFFFF
    pre, end = pe & 0xFFFF, pe >> 16
    assert sorted(pre.tolist()) == list(range(M)) and end[0] == M  # a bijection; the root spans everything
    assert (end > pre).all() and (end <= M).all()


def test_order_blob_limits_and_malformed_trees():
    # a chain deeper than 64 levels: the flat cut declines (None), the level walk handles it
    n = 70
    nodes = np.zeros((n, 6), np.int32)
    nodes[:, 4] = -1
    for i in range(n - 1):
        nodes[i, 2], nodes[i, 3] = 1, i + 1
    nodes[n - 1, 3] = -1
    assert _blob(nodes) is None
    assert _blob(_chain(60)) is not None
    # a node reachable twice is not a tree
    cyc = _chain(5)
    cyc[4, 2], cyc[4, 3] = 1, 1
    assert _blob(cyc) is None
    # out-of-range child index
    bad = _chain(5)
    bad[2, 3] = 99
    assert _blob(bad) is None
    # a single node (the root is a leaf)
    one = np.zeros((1, 6), np.int32)
    one[0, 3] = one[0, 4] = -1
    b = _blob(one)
    assert b is not None and b[0] == 1 and b[1] == 1


def _chain(n):
    nodes = np.zeros((n, 6), np.int32)
    nodes[:, 4] = -1
    for i in range(n - 1):
        nodes[i, 2], nodes[i, 3] = 1, i + 1
    nodes[n - 1, 3] = -1
    return nodes


def test_order_blob_entry_limit():
    # a complete binary tree of 2^17 - 1 nodes has more entries than the flat cut places (65,535)
    n = (1 << 17) - 1
    nodes = np.zeros((n, 6), np.int32)
    nodes[:, 3] = nodes[:, 4] = -1
    inner = np.arange(n // 2)
    nodes[inner, 2] = 2
    nodes[inner, 3] = 2 * inner + 1
    nodes[2 * inner + 1, 4] = 2 * inner + 2
    assert _blob(nodes) is None
    small = (1 << 15) - 1
    nodes = nodes[:small].copy()
    nodes[small // 2:, 2], nodes[small // 2:, 3] = 0, -1
    b = _blob(nodes)
    assert b is not None and b[0] == small and b[1] == 15
