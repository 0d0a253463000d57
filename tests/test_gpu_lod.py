"""HIP LOD kernels, SPT cut, render_post lerp and the in-kernel hierarchy rasterizer mode against the
oracle.  Integer outputs (selected nodes, parents, cut lists, per-tile lists) must be bit-exact; float
weights within 1e-6; lerp gradients within 1e-5 (float atomics change summation order only)."""
import numpy as np
import pytest
import torch

from hlgs_core import synthetic as S
from oracle import oracle as O
from helpers import assert_grad, binned, drops_empty, gpu_render, oracle_render, rel_err, settings_for, image_check

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _tree(n=600, sky=0, seed=0):
    cam = S.make_camera(128, 96)
    return S.make_dynamic_hierarchy(S.make_gaussians(n, 3, cam, seed=seed), skybox_points=sky, seed=seed), cam


@pytest.mark.parametrize("P,W,H,band", [(300, 200, 120, 64), (5000, 200, 120, 256), (12000, 200, 120, 512),
                                        (30000, 200, 120, 1024), (60000, 128, 128, 4096)])
def test_point_list_and_ranges_bit_exact(P, W, H, band):
    """Tile lists across every sort path: one-wave register sorts of 64..1024 keys and the block sort."""
    from diff_gaussian_rasterization import _C
    cam = S.make_camera(W, H)
    sc = S.make_gaussians(P, 1, cam, seed=11)
    sc["means3D"][::7, 2] = 9.0  # depth ties
    fr = O.forward(dict(sc), S.cam_numpy(cam), drop_empty=drops_empty(P))
    counts = fr.ranges[:, 1] - fr.ranges[:, 0]
    # each case's longest list lands in its sort path's band (block sort: 1025..4096)
    lo = 1024 if band == 4096 else band // 2
    assert counts.max() <= band and (band == 64 or counts.max() > lo), counts.max()
    t = lambda a: torch.tensor(a, device=DEV)  # noqa: E731
    e = torch.empty(0, device=DEV)
    out = _C.rasterize_gaussians(cam["bg"], e, e, e, e, t(sc["means3D"]), e, t(sc["opacities"]), t(sc["scales"]),
                                 t(sc["rotations"]), 1.0, e, cam["viewmatrix"], cam["projmatrix"], cam["tanfovx"],
                                 cam["tanfovy"], H, W, t(sc["shs"]), 1, cam["campos"], False, True, True)
    R = out[0]
    assert R == fr.R
    kept = binned(fr)
    pl = _C.inspect_point_list(out[4], kept).cpu().numpy().astype(np.uint32)
    rg = _C.inspect_ranges(out[5], W, H).cpu().numpy().astype(np.uint32)
    np.testing.assert_array_equal(rg, fr.ranges)
    np.testing.assert_array_equal(pl, fr.point_list[:kept])
    np.testing.assert_array_equal(out[7].cpu().numpy(), fr.seen)


@pytest.mark.parametrize("W,H", [(2048, 2048), (2064, 2048)])
def test_tile_grid_limits_lists_bit_exact(W, H):
    """The largest tile grid the LDS binning takes (128 x 128 = 16,384 tiles: 512 look-back blocks in the fused plan)
    and the next width up, which takes the generic path (device-atomic tile counts in the preprocess, one thread per
    Gaussian in the key scatter): ranges, point_list, n_contrib and seen against the oracle, with the zero-mask
    instances left out by both paths alike."""
    from diff_gaussian_rasterization import _C
    P = 150_000
    cam = S.make_camera(W, H)
    sc = S.make_gaussians(P, 1, cam, seed=23)
    fr = O.forward(dict(sc), S.cam_numpy(cam), drop_empty=drops_empty(P))
    t = lambda a: torch.tensor(a, device=DEV)  # noqa: E731
    e = torch.empty(0, device=DEV)
    out = _C.rasterize_gaussians(cam["bg"], e, e, e, e, t(sc["means3D"]), e, t(sc["opacities"]), t(sc["scales"]),
                                 t(sc["rotations"]), 1.0, e, cam["viewmatrix"], cam["projmatrix"], cam["tanfovx"],
                                 cam["tanfovy"], H, W, t(sc["shs"]), 1, cam["campos"], False, True, True)
    R = out[0]
    assert R == fr.R
    kept = binned(fr)
    np.testing.assert_array_equal(_C.inspect_ranges(out[5], W, H).cpu().numpy().astype(np.uint32), fr.ranges)
    np.testing.assert_array_equal(_C.inspect_point_list(out[4], kept, P).cpu().numpy().astype(np.uint32),
                                  fr.point_list[:kept])
    N = W * H
    n_contrib = _C._field(out[5], (4 * N + 255) // 256 * 256, N, torch.int32).cpu().numpy()
    np.testing.assert_array_equal(n_contrib, fr.n_contrib.astype(np.int32))
    np.testing.assert_array_equal(out[7].cpu().numpy(), fr.seen)
    mx, nbad, ok = image_check(out[1].cpu().numpy(), fr.color)
    assert ok, (mx, nbad)


def test_generic_binning_path_backward():
    """Forward and backward through the generic binning path (a tile grid above the LDS binning's 16,384 tiles), with
    the zero-mask instances dropped: the Gaussian backward skips their never-written record slots."""
    W, H, P = 2064, 2048, 60_000
    cam = S.make_camera(W, H)
    sc = S.make_gaussians(P, 3, cam, seed=29)
    g = S.upstream_grads(W, H, seed=4)
    gpu = gpu_render(sc, cam, grads=g)
    ref = oracle_render(sc, cam, grads=g, drop_empty=drops_empty(P))
    np.testing.assert_array_equal(gpu["radii"], ref["radii"])
    mx, nbad, ok = image_check(gpu["color"], ref["color"])
    assert ok, (mx, nbad)
    for k in ref:
        if k.startswith("d"):
            assert_grad(k, gpu[k][..., :ref[k].shape[-1]], ref[k])


@pytest.mark.parametrize("deg", [0, 3])
def test_decisions_bit_exact_for_elongated_splats(deg):
    """Strongly anisotropic splats (the float quadratic form cancels): the GPU keeps and skips exactly the
    oracle's pairs -- n_contrib, seen and point_list bit-exact, preprocess records bit-exact, image <= 1e-6."""
    from diff_gaussian_rasterization import _C
    W, H = 256, 192
    cam = S.make_camera(W, H)
    sc = S.make_gaussians(6000, deg, cam, seed=17)
    rng = np.random.default_rng(5)
    sc["scales"] = np.ascontiguousarray(sc["scales"] * np.exp(rng.uniform(-2.5, 2.5, sc["scales"].shape))
                                        .astype(np.float32))
    fr = O.forward(dict(sc), S.cam_numpy(cam), drop_empty=drops_empty(6000))
    t = lambda a: torch.tensor(a, device=DEV)  # noqa: E731
    e = torch.empty(0, device=DEV)
    out = _C.rasterize_gaussians(cam["bg"], e, e, e, e, t(sc["means3D"]), e, t(sc["opacities"]), t(sc["scales"]),
                                 t(sc["rotations"]), 1.0, e, cam["viewmatrix"], cam["projmatrix"], cam["tanfovx"],
                                 cam["tanfovy"], H, W, t(sc["shs"]), deg, cam["campos"], False, False, True)
    R = out[0]
    assert R == fr.R
    kept = binned(fr)
    np.testing.assert_array_equal(_C.inspect_point_list(out[4], kept).cpu().numpy().astype(np.uint32),
                                  fr.point_list[:kept])
    N = W * H
    n_contrib = _C._field(out[5], (4 * N + 255) // 256 * 256, N, torch.int32).cpu().numpy()
    np.testing.assert_array_equal(n_contrib, fr.n_contrib.astype(np.int32))
    np.testing.assert_array_equal(out[7].cpu().numpy(), fr.seen)
    rec = _C.inspect_splats(out[3], 6000).cpu().numpy()
    vis = out[2].cpu().numpy() > 0
    np.testing.assert_array_equal(rec[vis][:, 2:6], fr.conic_opacity[vis])
    assert np.abs(out[1].cpu().numpy() - fr.color).max() <= 1e-6


@pytest.mark.parametrize("sky", [0, 4])
def test_expand_to_size_dynamic_and_weights(sky):
    import gaussian_hierarchy as GH
    h, cam = _tree(800, sky=sky)
    nodes, pos, sc = h["nodes"], h["means3D"], h["scales"]
    N = nodes.shape[0]
    vp = np.array([0.05, 0.0, -0.1], np.float32)
    vd = np.array([0.0, 0.0, 1.0], np.float32)
    for target in (0.0008, 0.003, 0.01):
        ri = torch.zeros(N, dtype=torch.int32, device=DEV)
        pi = torch.zeros(N, dtype=torch.int32, device=DEV)
        ni = torch.zeros(N, dtype=torch.int32, device=DEV)
        n = GH.expand_to_size_dynamic(torch.tensor(nodes, device=DEV), torch.tensor(pos, device=DEV),
                                      torch.tensor(sc, device=DEV), target, torch.tensor(vp, device=DEV),
                                      torch.tensor(vd), ri, pi, ni)
        n_o, ri_o, pi_o, ni_o = O.expand_to_size_dynamic(nodes, pos, sc, target, vp, vd)
        assert n == n_o and n > 0
        np.testing.assert_array_equal(ri[:n].cpu().numpy(), ri_o[:n])
        np.testing.assert_array_equal(ni[:n].cpu().numpy(), ni_o[:n])
        np.testing.assert_array_equal(pi[:n].cpu().numpy(), pi_o[:n])
        ts = torch.zeros(N, device=DEV)
        kids = torch.zeros(N, dtype=torch.int32, device=DEV)
        GH.get_interpolation_weights_dynamic(ni[:n], target, torch.tensor(nodes, device=DEV),
                                             torch.tensor(pos, device=DEV), torch.tensor(sc, device=DEV),
                                             torch.tensor(vp), torch.tensor(vd), ts, kids)
        ts_o, kids_o = O.interp_weights_dynamic(ni_o[:n], target, nodes, pos, sc, vp)
        np.testing.assert_allclose(ts[:n].cpu().numpy(), ts_o, rtol=0, atol=1e-6)
        np.testing.assert_array_equal(kids[:n].cpu().numpy(), kids_o)


def test_expand_to_size_static():
    import gaussian_hierarchy as GH
    rng = np.random.default_rng(1)
    N = 500
    nodes = np.zeros((N, 7), np.int32)
    nodes[:, 1] = [-1] + [int(rng.integers(0, i)) for i in range(1, N)]
    nodes[:, 0] = rng.integers(0, 4, N)
    nodes[:, 2] = np.arange(N) * 2
    nodes[:, 3] = rng.integers(0, 3, N)
    nodes[:, 4] = rng.integers(0, 2, N)
    nodes[:, 6] = np.bincount(nodes[1:, 1], minlength=N)
    c = rng.uniform(-3, 3, (N, 3))
    e = rng.uniform(0.05, 1.0, (N, 3))
    boxes = np.zeros((N, 8), np.float32)
    boxes[:, :3], boxes[:, 4:7], boxes[:, 3] = c - e, c + e, e.max(1) * 2
    vp = np.array([0.3, 0.1, -0.2], np.float32)
    cap = int(nodes[:, 3].sum() + nodes[:, 4].sum()) + 1
    ri, pi, ni = (torch.zeros(cap, dtype=torch.int32, device=DEV) for _ in range(3))
    n = GH.expand_to_size(torch.tensor(nodes, device=DEV), torch.tensor(boxes, device=DEV), 0.3,
                          torch.tensor(vp, device=DEV), torch.zeros(3), ri, pi, ni)
    n_o, ri_o, pi_o, ni_o = O.expand_to_size(nodes, boxes, 0.3, vp)
    assert n == n_o
    for a, b in ((ri, ri_o), (pi, pi_o), (ni, ni_o)):
        np.testing.assert_array_equal(a[:n].cpu().numpy(), b[:n])
    ts = torch.zeros(N, device=DEV)
    kids = torch.zeros(N, dtype=torch.int32, device=DEV)
    idx = torch.arange(N, dtype=torch.int32, device=DEV)
    GH.get_interpolation_weights(idx, 0.3, torch.tensor(nodes, device=DEV), torch.tensor(boxes, device=DEV),
                                 torch.tensor(vp), torch.zeros(3), ts, kids)
    ts_o, kids_o = O.interp_weights(np.arange(N, dtype=np.int32), 0.3, nodes, boxes, vp)
    np.testing.assert_allclose(ts.cpu().numpy(), ts_o, atol=1e-6)
    np.testing.assert_array_equal(kids.cpu().numpy(), kids_o)


@pytest.mark.parametrize("compat", [True, False])
def test_spt_cut(compat):
    import gaussian_hierarchy as GH
    from test_oracle_lod import _random_spts
    for seed in range(4):
        gidx, starts, smax, smin, sidx, sdist = _random_spts(seed, S_count=300, sel=200)
        if seed == 0:
            gidx[0] = 0  # exercises the reference's DeviceSelect(x != 0) drop
        t = lambda a: torch.tensor(a, device=DEV)  # noqa: E731
        cut, cp = GH.get_spt_cut_cuda(len(sidx), t(gidx), t(starts), t(smax), t(smin), t(sidx), t(sdist), compat=compat)
        cut_o, cp_o = O.spt_cut(gidx, starts, smax, smin, sidx, sdist, compat=compat)
        np.testing.assert_array_equal(cut.cpu().numpy(), cut_o)
        np.testing.assert_array_equal(cp.cpu().numpy(), cp_o)


def test_lod_interpolation_forward_backward():
    import gaussian_hierarchy as GH
    h, cam = _tree(1000, sky=6)
    N = h["nodes"].shape[0]
    vp = np.zeros(3, np.float32)
    n, ri, pi, ni = O.expand_to_size_dynamic(h["nodes"], h["means3D"], h["scales"], 0.002, vp,
                                             np.array([0, 0, 1], np.float32))
    ts, _ = O.interp_weights_dynamic(ni[:n], 0.002, h["nodes"], h["means3D"], h["scales"], vp)
    pi = pi.copy()
    pi[n:] = 0
    Sk = 6
    leaf = lambda a: torch.tensor(a, device=DEV, requires_grad=True)  # noqa: E731
    m, s, r, o, sh = leaf(h["means3D"]), leaf(h["scales"]), leaf(h["rotations"]), leaf(h["opacities"]), leaf(h["shs"])
    outs = GH.interpolate_lod(m, s, r, o, sh, torch.tensor(ri[:n], device=DEV), torch.tensor(pi, device=DEV),
                              torch.tensor(np.pad(ts, (0, N - n)), device=DEV), Sk)
    ref = O.lod_interp_forward(Sk, ri[:n], pi[:n], ts, h["means3D"], h["scales"], h["rotations"], h["opacities"],
                               h["shs"])
    for got, key in zip(outs, ("means", "scales", "rots", "opac", "shs")):
        np.testing.assert_allclose(got.detach().cpu().numpy().reshape(ref[key].shape), ref[key], rtol=1e-6, atol=1e-6)
    rng = np.random.default_rng(0)
    gs = [rng.normal(size=tuple(x.shape)).astype(np.float32) for x in outs]
    sum((x * torch.tensor(g, device=DEV)).sum() for x, g in zip(outs, gs)).backward()
    d = O.lod_interp_backward(Sk, ri[:n], pi[:n], ts, h["rotations"], N,
                              dict(means=gs[0], scales=gs[1], rots=gs[2], opac=gs[3], shs=gs[4]))
    for leaf_t, key in zip((m, s, r, o, sh), ("means", "scales", "rots", "opac", "shs")):
        np.testing.assert_allclose(leaf_t.grad.cpu().numpy().reshape(d[key].shape), d[key], rtol=1e-5, atol=1e-5)
    # the gather backward is bitwise deterministic and writes every row (no pre-zeroed buffers)
    first = [t.grad.clone() for t in (m, s, r, o, sh)]
    for t in (m, s, r, o, sh):
        t.grad = None
    outs = GH.interpolate_lod(m, s, r, o, sh, torch.tensor(ri[:n], device=DEV), torch.tensor(pi, device=DEV),
                              torch.tensor(np.pad(ts, (0, N - n)), device=DEV), Sk)
    sum((x * torch.tensor(g, device=DEV)).sum() for x, g in zip(outs, gs)).backward()
    for a, t in zip(first, (m, s, r, o, sh)):
        assert torch.equal(a, t.grad)


def test_in_kernel_hierarchy_mode_matches_oracle():
    """render_indices / parent_indices / interpolation_weights / num_node_kids non-empty: the reference's
    in-kernel lerp and kids-alpha path (forward.cu:268-349,522-558; backward.cu:626-718,458-494)."""
    from diff_gaussian_rasterization import GaussianRasterizer
    h, _ = _tree(1500)
    cam = S.make_camera(128, 96)
    N = h["nodes"].shape[0]
    vp = cam["campos"].numpy()
    n, ri, pi, ni = O.expand_to_size_dynamic(h["nodes"], h["means3D"], h["scales"], 0.004, vp,
                                             np.array([0, 0, 1], np.float32))
    ts, kids = O.interp_weights_dynamic(ni[:n], 0.004, h["nodes"], h["means3D"], h["scales"], vp)
    roots = h["nodes"][ri[:n], 1] < 0
    pidx = np.where(roots, -1, pi[:n]).astype(np.int32)
    scene = dict(means3D=h["means3D"], opacities=h["opacities"], shs=h["shs"], scales=h["scales"],
                 rotations=h["rotations"], sh_degree=3, indices=ri[:n], parent_indices=pidx, ts=ts, kids=kids)
    fr = O.forward(scene, S.cam_numpy(cam))
    g, gd = S.upstream_grads(128, 96)
    gr = O.backward(fr, scene, g, gd)
    t = lambda a, rg=False: torch.tensor(a, device=DEV, requires_grad=rg)  # noqa: E731
    hier = dict(render_indices=t(ri[:n]), parent_indices=t(pidx), interpolation_weights=t(ts), num_node_kids=t(kids))
    rast = GaussianRasterizer(settings_for(cam, 3, DEV, hierarchy=hier))
    m, o, sh, s, r = t(h["means3D"], True), t(h["opacities"], True), t(h["shs"], True), t(h["scales"], True), \
        t(h["rotations"], True)
    m2 = torch.zeros_like(m, requires_grad=True)
    color, radii, invd = rast(means3D=m, means2D=m2, opacities=o, shs=sh, scales=s, rotations=r)
    np.testing.assert_array_equal(radii.cpu().numpy(), fr.radii)
    mx, nbad, ok = image_check(color.detach().cpu().numpy(), fr.color)
    assert ok, (mx, nbad)
    ((color * t(g)).sum() + (invd * t(gd)).sum()).backward()
    for name, leaf_t in (("dmean3D", m), ("dopacity", o), ("dscale", s), ("drot", r), ("dsh", sh), ("dmean2D", m2)):
        assert_grad(name, leaf_t.grad.cpu().numpy(), gr[name])


@pytest.mark.parametrize("deg", [3, 1])
def test_interpolation_weights_without_render_indices(deg):
    """interpolation_weights / num_node_kids given with an empty render_indices: the preprocess's common kernel takes
    its separately instantiated interpolation path (the alpha threshold's bisection, the lerped alpha and the kids
    exponent in both blends), against the oracle with the same ts / kids."""
    from diff_gaussian_rasterization import GaussianRasterizer
    cam = S.make_camera(160, 112)
    sc = S.make_gaussians(3000, deg, cam, seed=5)
    rng = np.random.default_rng(11)
    P = sc["means3D"].shape[0]
    ts = rng.uniform(0.05, 1.0, P).astype(np.float32)
    kids = rng.integers(1, 9, P).astype(np.int32)
    scene = dict(sc, ts=ts, kids=kids)
    fr = O.forward(scene, S.cam_numpy(cam))
    g, gd = S.upstream_grads(160, 112)
    gr = O.backward(fr, scene, g, gd)
    t = lambda a, rg=False: torch.tensor(a, device=DEV, requires_grad=rg)  # noqa: E731
    hier = dict(interpolation_weights=t(ts), num_node_kids=t(kids))
    rast = GaussianRasterizer(settings_for(cam, deg, DEV, hierarchy=hier))
    m, o, sh, s, r = (t(sc[k], True) for k in ("means3D", "opacities", "shs", "scales", "rotations"))
    m2 = torch.zeros_like(m, requires_grad=True)
    color, radii, invd = rast(means3D=m, means2D=m2, opacities=o, shs=sh, scales=s, rotations=r)
    np.testing.assert_array_equal(radii.cpu().numpy(), fr.radii)
    mx, nbad, ok = image_check(color.detach().cpu().numpy(), fr.color)
    assert ok, (mx, nbad)
    ((color * t(g)).sum() + (invd * t(gd)).sum()).backward()
    for name, leaf_t in (("dmean3D", m), ("dopacity", o), ("dscale", s), ("drot", r), ("dsh", sh), ("dmean2D", m2)):
        assert_grad(name, leaf_t.grad.cpu().numpy(), gr[name])


def test_morton_codes_bit_exact():
    """get_morton_indices (morton.cu:9-42) against the float32 numpy restatement, plus sort_morton's
    permutation (gaussian_model.py:570-589) keeping the root first."""
    import gaussian_hierarchy as GH
    from hlgs_core import scene
    from oracle import hier_format as HF
    rng = np.random.default_rng(12)
    xyz = rng.normal(0, 20, (50000, 3)).astype(np.float32)
    mn, mx = xyz.min(0), xyz.max(0)
    codes = torch.zeros(len(xyz), dtype=torch.int64, device=DEV)
    GH.get_morton_indices(torch.tensor(xyz, device=DEV), torch.tensor(mn, device=DEV), torch.tensor(mx, device=DEV),
                          codes)
    np.testing.assert_array_equal(codes.cpu().numpy(), HF.morton_codes(xyz, mn, mx))
    idx = scene.morton_order(torch.tensor(xyz, device=DEV), skybox_points=5).cpu().numpy()
    assert idx[0] == 5 and sorted(idx.tolist()) == list(range(5, 50000))


@pytest.mark.parametrize("deg", [3, 1])
def test_lod_interpolation_backward_wide_buckets(deg):
    """Parents shared by many selected rows (buckets far longer than a binary tree's), nodes that are both a child
    and a parent, a skybox prefix: the gather backward against the oracle restatement of the lerp's autograd."""
    import gaussian_hierarchy as GH
    rng = np.random.default_rng(7)
    N, n, Sk, M = 5000, 1500, 5, (deg + 1) ** 2
    ri = rng.choice(np.arange(Sk, N), n, replace=False).astype(np.int32)
    pi = rng.choice(np.arange(Sk, 40), n).astype(np.int32)          # ~40 rows per parent
    pi[::7] = ri[(np.arange(len(pi[::7])) * 3) % n]                  # parents that are selected children too
    ts = rng.uniform(0, 1, n).astype(np.float32)
    h = dict(means3D=rng.normal(size=(N, 3)), scales=rng.uniform(0.01, 1, (N, 3)), rotations=rng.normal(size=(N, 4)),
             opacities=rng.uniform(0, 1, (N, 1)), shs=rng.normal(size=(N, M, 3)))
    h = {k: v.astype(np.float32) for k, v in h.items()}
    leaf = lambda a: torch.tensor(a, device=DEV, requires_grad=True)  # noqa: E731
    m, s, r, o, sh = leaf(h["means3D"]), leaf(h["scales"]), leaf(h["rotations"]), leaf(h["opacities"]), leaf(h["shs"])
    pfull = np.zeros(N, np.int32)
    pfull[:n] = pi
    outs = GH.interpolate_lod(m, s, r, o, sh, torch.tensor(ri, device=DEV), torch.tensor(pfull, device=DEV),
                              torch.tensor(np.pad(ts, (0, N - n)), device=DEV), Sk)
    gs = [rng.normal(size=tuple(x.shape)).astype(np.float32) for x in outs]
    sum((x * torch.tensor(g, device=DEV)).sum() for x, g in zip(outs, gs)).backward()
    d = O.lod_interp_backward(Sk, ri, pi, ts, h["rotations"], N,
                              dict(means=gs[0], scales=gs[1], rots=gs[2], opac=gs[3], shs=gs[4]))
    for leaf_t, key in zip((m, s, r, o, sh), ("means", "scales", "rots", "opac", "shs")):
        np.testing.assert_allclose(leaf_t.grad.cpu().numpy().reshape(d[key].shape), d[key], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("i", [0, 1, 2])
def test_lod_interpolation_matches_reference_render_post(i):
    """interpolate_lod (forward and its gather backward) against render_post's lerp block executed from the
    reference itself, and autograd through it (tests/golden/golden_lerp.npz, make_golden.py lerp_fixture)."""
    import os
    import gaussian_hierarchy as GH
    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_lerp.npz"))
    sky = int(z[f"skybox_points_{i}"])
    leaves = [torch.tensor(z[f"{k}_{i}"], device=DEV, requires_grad=True)
              for k in ("xyz", "scaling", "rotation", "opacity", "features")]
    G = leaves[0].shape[0]
    n = z[f"render_indices_{i}"].shape[0]
    pad = lambda a, dt: torch.tensor(np.concatenate([a, np.zeros(G - n, a.dtype)]), device=DEV, dtype=dt)  # noqa
    outs = GH.interpolate_lod(*leaves, torch.tensor(z[f"render_indices_{i}"], device=DEV),
                              pad(z[f"parent_indices_{i}"], torch.int32), pad(z[f"weights_{i}"], torch.float32), sky)
    keys = ("means", "scales", "rots", "opac", "shs")
    for o, k in zip(outs, keys):
        want = z[f"out_{k}_{i}"]
        np.testing.assert_allclose(o.detach().cpu().numpy().reshape(want.shape), want, rtol=1e-6, atol=1e-7,
                                   err_msg=k)
    sum((o * torch.tensor(z[f"up_{k}_{i}"], device=DEV).reshape(o.shape)).sum() for o, k in zip(outs, keys)).backward()
    for leaf, k in zip(leaves, keys):
        want = z[f"grad_{k}_{i}"]
        np.testing.assert_allclose(leaf.grad.cpu().numpy().reshape(want.shape), want, rtol=1e-5, atol=1e-6,
                                   err_msg=k)
