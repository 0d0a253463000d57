"""Hierarchy files, static traversal and scene assembly (host code in libhlgs.so, no GPU needed).

The reference's loader/writer need Eigen (not vendored) and the reference ships no hierarchy files, so parity is
pinned on the byte layouts restated in oracle/hier_format.py: files written here must parse there and vice
versa, bit for bit, for every layout (.dhier at SH degrees 0-3, .hier full and binary16), and expand_to_target
must equal the recursive traversal.cpp restatement.
"""
import numpy as np
import pytest
import torch

from hlgs_core import synthetic as S
from oracle import hier_format as HF


def _tree(n=300, deg=3, seed=0):
    cam = S.make_camera(128, 96)
    return S.make_dynamic_hierarchy(S.make_gaussians(n, deg, cam, seed=seed), seed=seed)


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_dhier_round_trip_both_ways(tmp_path, deg):
    import gaussian_hierarchy as GH
    h = _tree(200, deg, seed=deg)
    G = h["means3D"].shape[0]
    log_scales = np.log(h["scales"])
    args = [torch.tensor(h["means3D"]), torch.tensor(h["shs"]), torch.tensor(h["opacities"]),
            torch.tensor(log_scales), torch.tensor(h["rotations"]), torch.tensor(h["nodes"])]
    ours = tmp_path / "ours.dhier"
    GH.write_dynamic_hierarchy(str(ours), *args, deg)
    r = HF.read_dhier(str(ours))
    assert r["sh_degree"] == deg
    np.testing.assert_array_equal(r["pos"], h["means3D"])
    np.testing.assert_array_equal(r["shs"], h["shs"].reshape(G, -1))
    np.testing.assert_array_equal(r["opac"].reshape(-1), h["opacities"].reshape(-1))
    np.testing.assert_array_equal(r["log_scales"], log_scales.astype(np.float32))
    np.testing.assert_array_equal(r["rot"], h["rotations"])
    np.testing.assert_array_equal(r["nodes"], h["nodes"])
    theirs = tmp_path / "theirs.dhier"
    HF.write_dhier(str(theirs), h["means3D"], h["shs"], h["opacities"], log_scales, h["rotations"], h["nodes"], deg,
                   n_header=12345)  # the loader ignores the stored node count
    pos, shs, alpha, sc, rot, nodes = GH.load_dynamic_hierarchy(str(theirs))
    assert shs.shape == (G, (deg + 1) ** 2, 3) and alpha.shape == (G, 1) and nodes.shape == (G, 6)
    assert nodes.dtype == torch.int32 and pos.device.type == "cpu"
    np.testing.assert_array_equal(pos.numpy(), h["means3D"])
    np.testing.assert_array_equal(shs.numpy(), h["shs"])
    np.testing.assert_array_equal(alpha.numpy(), h["opacities"])
    np.testing.assert_array_equal(sc.numpy(), log_scales.astype(np.float32))
    np.testing.assert_array_equal(rot.numpy(), h["rotations"])
    np.testing.assert_array_equal(nodes.numpy(), h["nodes"])


def test_dhier_writer_takes_the_first_coefficients_of_wider_rows(tmp_path):
    """write_dynamic_hierarchy writes (deg+1)^2 x 3 floats per Gaussian from the start of the contiguous shs
    (hierarchy_writer.cpp:133-150), so a 16-coefficient tensor saved at degree 1 keeps its first 12 floats of
    the flat buffer -- the reference's behaviour, reproduced."""
    import gaussian_hierarchy as GH
    h = _tree(50, 3, seed=4)
    G = h["means3D"].shape[0]
    p = tmp_path / "d1.dhier"
    GH.write_dynamic_hierarchy(str(p), torch.tensor(h["means3D"]), torch.tensor(h["shs"]),
                               torch.tensor(h["opacities"]), torch.tensor(h["scales"]), torch.tensor(h["rotations"]),
                               torch.tensor(h["nodes"]), 1)
    r = HF.read_dhier(str(p))
    np.testing.assert_array_equal(r["shs"].reshape(-1), h["shs"].reshape(-1)[: G * 12])


def _static_tree(rng, n_nodes=60, P=500):
    """Random static hierarchy in breadth-first order (children contiguous), Node = {depth (leaves 0), parent,
    start, count_leafs, count_merged, start_children, count_children} (types.h:82-91)."""
    nodes = np.zeros((n_nodes, 7), np.int32)
    nodes[0, 1] = -1
    frontier, nxt = [0], 1
    while frontier:
        new = []
        for v in frontier:
            k = int(rng.integers(0, 4)) if nxt < n_nodes else 0
            k = min(k, n_nodes - nxt)
            nodes[v, 5], nodes[v, 6] = nxt, k
            for c in range(k):
                nodes[nxt + c, 1] = v
                new.append(nxt + c)
            nxt += k
        frontier = new
    nodes = nodes[:nxt]
    for v in range(len(nodes) - 1, -1, -1):  # height above the deepest leaf
        kids = range(nodes[v, 5], nodes[v, 5] + nodes[v, 6])
        nodes[v, 0] = 0 if nodes[v, 6] == 0 else 1 + max(nodes[c, 0] for c in kids)
    nodes[:, 2] = rng.integers(0, P, len(nodes))
    nodes[:, 3] = rng.integers(0, 4, len(nodes))
    nodes[:, 4] = rng.integers(0, 3, len(nodes))
    return nodes


@pytest.mark.parametrize("compressed", [False, True])
def test_hier_round_trip_both_ways(tmp_path, compressed):
    import gaussian_hierarchy as GH
    rng = np.random.default_rng(3)
    P = 400
    nodes = _static_tree(rng, 80, P)
    N = nodes.shape[0]
    pos = rng.normal(0, 5, (P, 3)).astype(np.float32)
    rot = rng.normal(0, 1, (P, 4)).astype(np.float32)
    ls = rng.normal(-3, 1, (P, 3)).astype(np.float32)
    op = rng.uniform(0, 1, (P, 1)).astype(np.float32)
    shs = rng.normal(0, 0.3, (P, 16, 3)).astype(np.float32)
    boxes = rng.normal(0, 10, (N, 2, 4)).astype(np.float32)
    theirs = tmp_path / "theirs.hier"
    HF.write_hier(str(theirs), pos, shs, op, ls, rot, nodes, boxes, compressed=compressed)
    got = GH.load_hierarchy(str(theirs))
    want = HF.read_hier(str(theirs))
    assert want["half"] == compressed
    for g, k in zip(got, ("pos", "shs", "opac", "log_scales", "rot", "nodes", "boxes")):
        np.testing.assert_array_equal(g.numpy().reshape(want[k].shape), want[k])
    if not compressed:
        np.testing.assert_array_equal(got[1].numpy(), shs)
        np.testing.assert_array_equal(got[5].numpy(), nodes)
    # our writer (binary16, the reference's default) parses back to the same half-rounded values
    ours = tmp_path / "ours.hier"
    GH.write_hierarchy(str(ours), *[torch.tensor(a) for a in (pos, shs, op, ls, rot, nodes, boxes)])
    HF.write_hier(str(tmp_path / "ref_half.hier"), pos, shs, op, ls, rot, nodes, boxes, compressed=True)
    assert open(ours, "rb").read() == open(tmp_path / "ref_half.hier", "rb").read()


def test_binary16_conversion_is_round_to_nearest_even(tmp_path):
    """Edge values through the .hier half layout: ties, subnormals, overflow, signed zero, infinities."""
    import gaussian_hierarchy as GH
    rng = np.random.default_rng(9)
    special = np.array([0.0, -0.0, 1.0, 65504.0, 65519.99, 65520.0, -70000.0, 6.1e-5, 5.96e-8, 2.98e-8, 2.99e-8,
                        1e-9, 1.0 + 2 ** -11, 1.0 + 3 * 2 ** -11, 2049.0, 2051.0, np.inf, -np.inf], np.float32)
    vals = np.concatenate([special, rng.normal(0, 1, 4000).astype(np.float32) * 10.0 ** rng.integers(-8, 5, 4000)])
    P = (len(vals) + 47) // 48
    shs = np.zeros(P * 48, np.float32)
    shs[: len(vals)] = vals
    shs = shs.reshape(P, 16, 3)
    z = lambda *s: np.zeros(s, np.float32)  # noqa: E731
    nodes = np.zeros((1, 7), np.int32)
    nodes[0, 1] = -1
    p = tmp_path / "h.hier"
    GH.write_hierarchy(str(p), *[torch.tensor(a) for a in (z(P, 3), shs, z(P, 1), z(P, 3), z(P, 4), nodes,
                                                          z(1, 2, 4))])
    got = GH.load_hierarchy(str(p))[1].numpy().reshape(-1)[: len(vals)]
    with np.errstate(over="ignore"):  # 65520 and beyond round to infinity, as intended
        want = vals.astype(np.float16).astype(np.float32)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


def test_hier_writer_refuses_to_lose_information(tmp_path):
    import gaussian_hierarchy as GH
    nodes = np.zeros((2, 7), np.int32)
    nodes[1, 3] = 40000  # count_leafs > 32000 does not fit the HalfNode int16 (hierarchy_writer.cpp:90-92)
    z = lambda *s: torch.zeros(s)  # noqa: E731
    with pytest.raises(RuntimeError, match="Would lose information!"):
        GH.write_hierarchy(str(tmp_path / "x.hier"), z(1, 3), z(1, 16, 3), z(1, 1), z(1, 3), z(1, 4),
                           torch.tensor(nodes), z(2, 2, 4))
    with pytest.raises(RuntimeError, match="File not found!"):
        GH.load_dynamic_hierarchy(str(tmp_path / "missing.dhier"))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_expand_to_target_matches_recursive_traversal(seed):
    import gaussian_hierarchy as GH
    rng = np.random.default_rng(seed)
    nodes = _static_tree(rng, 200)
    for target in range(-1, int(nodes[:, 0].max()) + 2):
        got = GH.expand_to_target(torch.tensor(nodes), target)
        assert got.dtype == torch.int32
        np.testing.assert_array_equal(got.numpy(), HF.expand_to_target(nodes, target))


def test_scene_assembly_matches_create_from_hier():
    """Skybox prepend and index shifts of GaussianModel.create_from_hier (scene/gaussian_model.py:1050-1095)."""
    from hlgs_core import scene
    h = _tree(120, 3, seed=6)
    sky = S.make_dynamic_hierarchy(S.make_gaussians(120, 3, S.make_camera(128, 96), seed=6), skybox_points=7,
                                   seed=6)
    out = scene.assemble_hierarchy(torch.tensor(h["means3D"]), torch.tensor(h["shs"]), torch.tensor(h["opacities"]),
                                   torch.tensor(h["scales"]), torch.tensor(h["rotations"]), torch.tensor(h["nodes"]),
                                   sky=dict(xyz=torch.tensor(sky["means3D"][:7]),
                                            features_dc=torch.tensor(sky["shs"][:7, :1]),
                                            features_rest=torch.tensor(sky["shs"][:7, 1:4]),
                                            opacity_logits=torch.logit(torch.tensor(sky["opacities"][:7])),
                                            scales=torch.tensor(sky["scales"][:7]),
                                            rotations=torch.tensor(sky["rotations"][:7])),
                                   max_sh_degree=3)
    assert out["skybox_points"] == 7
    nodes_ref = sky["nodes"].copy()
    nodes_ref[:, -1] = 0  # create_from_hier zeroes the last column
    np.testing.assert_array_equal(out["nodes"].numpy(), nodes_ref)
    np.testing.assert_allclose(out["xyz"].numpy(), sky["means3D"])
    np.testing.assert_allclose(out["opacity"].numpy(), sky["opacities"], rtol=1e-6)
    G = h["means3D"].shape[0] + 7
    assert out["features_dc"].shape == (G, 1, 3) and out["features_rest"].shape == (G, 15, 3)
