"""alt_gaussian_rasterization (the alt rasterizer of submodules/alt-rasterizer, default in train_post.py) on
the HIP path against the oracle's alt restatement, on identical seeded inputs.

Forward: per-pixel L-inf <= 1e-4; radii, per-tile lists (after exact tile culling), num_rendered (counting the
culled instances, as the reference does) and n_contrib bit-exact.  Backward: max|gpu - oracle| / max|oracle|
<= 1e-3 per gradient tensor.  SparseGaussianAdam / adamUpdate against a float32 numpy restatement of
adam.cu:9-36 (rel 1e-6, untouched rows bit-exact).
"""
import numpy as np
import pytest
import torch

from hlgs_core import synthetic as S
from helpers import assert_grad, drops_empty, image_check, rel_err
from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
FWD_TOL = 1e-4
GRAD_TOL = 1e-3


def _alt_scene(P, deg, W, H, seed=0, bg=(0.0, 0.0, 0.0), aa=True):
    cam = S.make_camera(W, H, bg=bg)
    sc = S.make_gaussians(P, deg, cam, seed=seed)
    sc["dc"] = np.ascontiguousarray(sc["shs"][:, :1])
    sc["shs"] = np.ascontiguousarray(sc["shs"][:, 1:])
    sc["alt"] = True
    sc["antialiasing"] = aa
    return sc, cam


def _settings(cam, deg, aa, debug=False):
    from alt_gaussian_rasterization import GaussianRasterizationSettings
    return GaussianRasterizationSettings(
        image_height=cam["H"], image_width=cam["W"], tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"],
        bg=cam["bg"].to(DEV), scale_modifier=1.0, viewmatrix=cam["viewmatrix"].to(DEV),
        projmatrix=cam["projmatrix"].to(DEV), sh_degree=deg, campos=cam["campos"].to(DEV), prefiltered=False,
        debug=debug, antialiasing=aa)


def _gpu(sc, cam, grads, use_colors=False):
    from alt_gaussian_rasterization import GaussianRasterizer
    t = lambda a: torch.tensor(np.ascontiguousarray(a), device=DEV, requires_grad=True)  # noqa: E731
    means3D = t(sc["means3D"])
    means2D = torch.zeros_like(means3D, requires_grad=True)
    opac, scales, rots = t(sc["opacities"]), t(sc["scales"]), t(sc["rotations"])
    kw = dict(colors_precomp=t(sc["colors_precomp"])) if use_colors else dict(dc=t(sc["dc"]), shs=t(sc["shs"]))
    rast = GaussianRasterizer(_settings(cam, sc["sh_degree"], sc["antialiasing"]))
    color, radii, invd = rast(means3D=means3D, means2D=means2D, opacities=opac, scales=scales, rotations=rots, **kw)
    out = dict(color=color.detach().cpu().numpy(), radii=radii.cpu().numpy(), invdepth=invd.detach().cpu().numpy())
    if grads is not None:
        g, gd = grads
        loss = (color * torch.tensor(g, device=DEV)).sum() + (invd * torch.tensor(gd, device=DEV)).sum()
        loss.backward()
        out.update(dmean3D=means3D.grad.cpu().numpy(), dmean2D=means2D.grad.cpu().numpy(),
                   dopacity=opac.grad.cpu().numpy(), dscale=scales.grad.cpu().numpy(), drot=rots.grad.cpu().numpy())
        for k, v in kw.items():
            out["d" + k] = v.grad.cpu().numpy()
    return out


def _oracle(sc, cam, grads, use_colors=False):
    s = dict(sc)
    if use_colors:
        s.pop("dc"), s.pop("shs")
    else:
        s.pop("colors_precomp", None)
    fr = O.forward(s, S.cam_numpy(cam))
    out = dict(color=fr.color, radii=fr.radii, invdepth=fr.invdepth, frame=fr)
    if grads is not None:
        gr = O.backward(fr, s, *grads)
        out.update(dmean3D=gr["dmean3D"], dmean2D=gr["dmean2D"], dopacity=gr["dopacity"], dscale=gr["dscale"],
                   drot=gr["drot"])
        if use_colors:
            out["dcolors_precomp"] = gr["dcolor"]
        else:
            out["ddc"], out["dshs"] = gr["ddc"], gr["dsh"]
    return out


def _compare(sc, cam, use_colors=False):
    g = S.upstream_grads(cam["W"], cam["H"], seed=1)
    gpu = _gpu(sc, cam, g, use_colors)
    ref = _oracle(sc, cam, g, use_colors)
    np.testing.assert_array_equal(gpu["radii"], ref["radii"])
    for k in ("color", "invdepth"):
        mx, nbad, ok = image_check(gpu[k], ref[k], FWD_TOL)
        assert ok, f"{k} L-inf {mx} ({nbad} pixels over {FWD_TOL})"
    for k in ref:
        if k.startswith("d"):
            assert_grad(k, gpu[k][..., :ref[k].shape[-1]], ref[k])
    return gpu, ref


@pytest.mark.parametrize("P,deg,W,H,aa", [(300, 0, 64, 64, True), (2000, 3, 128, 96, True), (1500, 1, 100, 75, False),
                                          (4000, 2, 256, 256, True), (3000, 3, 200, 120, False)])
def test_alt_forward_backward_parity(P, deg, W, H, aa):
    sc, cam = _alt_scene(P, deg, W, H, seed=P, aa=aa)
    _compare(sc, cam)


def test_alt_random_background_and_opaque_clamp():
    """Non-zero bg (the alt backward counts the bg term twice) and splats at the 0.99 clamp (no zeroing rule)."""
    sc, cam = _alt_scene(1200, 3, 96, 64, seed=4, bg=(0.3, 0.6, 0.9))
    sc["opacities"][::5] = 0.9995
    _compare(sc, cam)


def test_alt_colors_precomp_path():
    sc, cam = _alt_scene(800, 0, 80, 64, seed=8)
    sc["colors_precomp"] = np.random.default_rng(3).uniform(0, 1, (800, 3)).astype(np.float32)
    _compare(sc, cam, use_colors=True)


@pytest.mark.parametrize("P,W,H,stretch", [(2500, 160, 128, 1.0), (40000, 128, 128, 1.0), (3000, 320, 256, 30.0)])
def test_alt_tile_culling_lists_bit_exact(P, W, H, stretch):
    """Binned instances after the exact per-tile culling, their depth order, num_rendered (culled instances
    included) and per-pixel contributor counts equal the oracle's.  stretch: every third splat made a long thin
    rotated ellipse spanning many tiles, where the binning walk's per-row candidate columns (alt_row_cols) cut
    most of the rect and must never drop a tile the per-tile test keeps."""
    from alt_gaussian_rasterization import _C
    from diff_gaussian_rasterization import _C as HC
    sc, cam = _alt_scene(P, 1, W, H, seed=21)
    sc["means3D"][::9, 2] = 6.0  # depth ties
    if stretch > 1.0:
        sc["scales"][::3, 0] *= stretch
        sc["opacities"][::3] = 0.9
    fr = O.forward(dict(sc), S.cam_numpy(cam), drop_empty=drops_empty(sc["means3D"].shape[0]))
    t = lambda a: torch.tensor(a, device=DEV)  # noqa: E731
    e = torch.empty(0, device=DEV)
    out = _C.rasterize_gaussians(cam["bg"], t(sc["means3D"]), e, t(sc["opacities"]), t(sc["scales"]),
                                 t(sc["rotations"]), 1.0, e, cam["viewmatrix"], cam["projmatrix"], cam["tanfovx"],
                                 cam["tanfovy"], H, W, t(sc["dc"]), t(sc["shs"]), 1, cam["campos"], False, True, False)
    num_rendered, _, color, invd, radii, geom, binning, img, _ = out
    assert num_rendered == fr.R
    rg = HC.inspect_ranges(img, W, H).cpu().numpy().astype(np.uint32)
    np.testing.assert_array_equal(rg, fr.ranges)
    kept = int((fr.ranges[:, 1] - fr.ranges[:, 0]).sum())
    assert kept < fr.R
    np.testing.assert_array_equal(HC.inspect_point_list(binning, kept).cpu().numpy().astype(np.uint32),
                                  fr.point_list[:kept])
    N = W * H
    n_contrib = HC._field(img, (4 * N + 255) // 256 * 256, N, torch.int32).cpu().numpy()
    np.testing.assert_array_equal(n_contrib, fr.n_contrib.astype(np.int32))
    assert np.abs(color.cpu().numpy() - fr.color).max() <= 1e-4


def test_alt_empty_and_all_culled():
    from alt_gaussian_rasterization import _C
    sc, cam = _alt_scene(200, 1, 48, 32, seed=2, bg=(0.25, 0.5, 0.75))
    sc["means3D"][:, 2] = -5.0  # all behind the camera: nothing binned, the alt rasterizer renders bg
    g = S.upstream_grads(48, 32, seed=1)
    gpu, ref = _compare(sc, cam)
    np.testing.assert_allclose(gpu["color"], np.broadcast_to(np.float32([0.25, 0.5, 0.75])[:, None, None],
                                                            (3, 32, 48)))
    assert all(np.all(gpu[k] == 0) for k in gpu if k.startswith("d"))
    e = torch.empty(0, device=DEV)
    out = _C.rasterize_gaussians(cam["bg"], torch.empty((0, 3), device=DEV), e, e, e, e, 1.0, e, cam["viewmatrix"],
                                 cam["projmatrix"], cam["tanfovx"], cam["tanfovy"], 32, 48, e, e, 0, cam["campos"],
                                 False, True, False)
    assert out[0] == 0 and torch.all(out[2] == 0) and out[3].shape == (1, 32, 48)
    del g


def test_alt_degree0_without_rest_gives_dc_no_gradient():
    """sh of shape (P, 0, 3): the reference's SH backward is skipped (backward.cu:443, shs == nullptr), so dc
    gets exactly zero gradient while the forward still colours with it."""
    sc, cam = _alt_scene(600, 0, 64, 48, seed=5)
    sc["shs"] = np.zeros((600, 0, 3), np.float32)
    g = S.upstream_grads(64, 48, seed=1)
    gpu = _gpu(sc, cam, g)
    ref = _oracle(sc, cam, g)
    mx, _, ok = image_check(gpu["color"], ref["color"], FWD_TOL)
    assert ok, mx
    assert np.all(gpu["ddc"] == 0) and np.all(ref["ddc"] == 0)
    assert_grad("dmean3D", gpu["dmean3D"], ref["dmean3D"])


def test_alt_backward_is_deterministic():
    sc, cam = _alt_scene(3000, 3, 128, 128, seed=9, bg=(0.1, 0.2, 0.3))
    g = S.upstream_grads(128, 128, seed=1)
    a, b = _gpu(sc, cam, g), _gpu(sc, cam, g)
    for k in a:
        if k.startswith("d"):
            np.testing.assert_array_equal(a[k], b[k])


def _adam_ref(p, g, m, v, vis, lr, b1, b2, eps, M):
    p, m, v = p.copy(), m.copy(), v.copy()
    on = np.repeat(vis, M)[: p.size]
    f = np.float32
    m2 = f(b1) * m + f(1 - f(b1)) * g
    v2 = f(b2) * v + f(1 - f(b2)) * g * g
    p2 = p + (f(-lr) * m2) / (np.sqrt(v2) + f(eps))
    return np.where(on, p2, p), np.where(on, m2, m), np.where(on, v2, v)


@pytest.mark.parametrize("N,M", [(1000, 3), (777, 1), (513, 45), (4096, 4)])
def test_adam_update_matches_reference(N, M):
    from alt_gaussian_rasterization import _C
    rng = np.random.default_rng(N + M)
    p, g = rng.normal(size=N * M).astype(np.float32), rng.normal(size=N * M).astype(np.float32)
    m, v = rng.normal(size=N * M).astype(np.float32) * 0.1, rng.uniform(0, 1, N * M).astype(np.float32)
    vis = rng.uniform(size=N) < 0.6
    tp, tg, tm, tv = (torch.tensor(x, device=DEV) for x in (p, g, m, v))
    _C.adamUpdate(tp, tg, tm, tv, torch.tensor(vis, device=DEV), 1e-3, 0.9, 0.999, 1e-15, N, M)
    rp, rm, rv = _adam_ref(p, g, m, v, vis, 1e-3, 0.9, 0.999, 1e-15, M)
    off = ~np.repeat(vis, M)
    for got, want, old in ((tp, rp, p), (tm, rm, m), (tv, rv, v)):
        got = got.cpu().numpy()
        np.testing.assert_array_equal(got[off], old[off])  # invisible rows untouched
        np.testing.assert_allclose(got, want, rtol=2e-6, atol=1e-7)


def test_sparse_gaussian_adam_step():
    from alt_gaussian_rasterization import SparseGaussianAdam
    N = 300
    x = torch.nn.Parameter(torch.randn(N, 16, 3, device=DEV))
    opt = SparseGaussianAdam([{"params": [x], "lr": 0.01, "name": "f_rest"}], lr=0.0, eps=1e-15)
    x.grad = torch.randn_like(x)
    vis = torch.rand(N, device=DEV) < 0.5
    before = x.detach().clone()
    opt.step(vis, N)
    moved = (x.detach() != before).reshape(N, -1).any(1)
    assert torch.equal(moved, vis)
    st = opt.state[x]
    np.testing.assert_allclose(st["exp_avg"][vis].cpu().numpy(), (0.1 * x.grad[vis]).cpu().numpy(), rtol=1e-6)


@pytest.mark.parametrize("aa", [True, False])
def test_alt_wide_splats_balanced_binning(aa):
    """A few splats whose rects cover most of a 512x384 frame (hundreds of tiles): the binning spreads their
    instances over the block and the record sums go through the wave-wide path (> 32 slots)."""
    sc, cam = _alt_scene(3000, 1, 512, 384, seed=31, aa=aa)
    sc["scales"][:6] *= 40.0
    sc["opacities"][:6] = np.float32(0.3)
    _compare(sc, cam)


@pytest.mark.parametrize("aa,op", [(True, (0.01, 0.08)), (False, (0.2, 0.9))])
def test_alt_backward_chunks_from_sampled_state(aa, op):
    """Dense, faint scenes (tile lists of ~600-1300 entries): the chunked blend backward of the alt variant
    (doubled background term) against the oracle's single back-to-front pass."""
    sc, cam = _alt_scene(8000, 2, 64, 64, seed=17, bg=(0.2, 0.5, 0.7), aa=aa)
    sc["opacities"] = np.random.default_rng(17).uniform(op[0], op[1], (8000, 1)).astype(np.float32)
    gpu, ref = _compare(sc, cam)
    assert np.diff(ref["frame"].ranges.astype(np.int64), axis=1).max() > 2 * 128
