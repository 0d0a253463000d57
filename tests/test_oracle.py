"""Pin the oracle (CPU restatement) before trusting it as the GPU checker.

* SH->RGB against golden vectors produced by the reference's own utils/sh_utils.eval_sh
  (tests/golden/make_golden.py).
* Camera matrices against golden vectors from the reference's utils/graphics_utils.
* Forward image and every gradient against an independent float64 torch-autograd restatement of the
  reference forward (preprocessCUDA + renderCUDA semantics, vectorised per tile).  The reference's
  analytic backward (backward.cu) must equal autograd of its forward wherever the forward is smooth.
"""
import os

import numpy as np
import pytest
import torch

from hlgs_core import synthetic as S
from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_sh_colors_match_reference_eval_sh(deg):
    z = np.load(os.path.join(GOLD, "golden_sh.npz"))
    rgb, clamped = O.sh_colors(z[f"shs_{deg}"], z[f"means_{deg}"], z[f"campos_{deg}"], deg)
    np.testing.assert_allclose(rgb, z[f"rgb_{deg}"], rtol=2e-6, atol=2e-6)
    assert np.all((clamped != 0) == (z[f"rgb_{deg}"] == 0).any(1) | (clamped != 0))


def test_camera_matches_reference_graphics_utils():
    z = np.load(os.path.join(GOLD, "golden_camera.npz"))
    for i in range(4):
        W, H = [int(v) for v in z[f"WH_{i}"]]
        cam = S.make_camera(W, H, R=z[f"R_{i}"], T=z[f"T_{i}"])
        np.testing.assert_array_equal(cam["viewmatrix"].numpy(), z[f"view_{i}"])
        np.testing.assert_array_equal(cam["projmatrix"].numpy(), z[f"proj_{i}"])
        np.testing.assert_allclose(cam["campos"].numpy(), z[f"campos_{i}"], rtol=0, atol=1e-6)


REALCAM_TAGS = dict(native=dict(), hd=dict(W=1920, H=1080), pp=dict(primx=0.47, primy=0.53))


@pytest.mark.parametrize("tag", list(REALCAM_TAGS))
def test_real_cameras_match_reference_graphics_utils(tag):
    """The reference's own cameras (cameras.json: rotated, fx != fy, ragged sizes) through S.real_camera against the
    matrices utils/graphics_utils builds for them (scene/cameras.py:102-107), bit for bit."""
    z = np.load(os.path.join(GOLD, "golden_realcam.npz"))
    cams = S.load_real_cameras()
    assert len(cams) == int(z["count"]) >= 8
    for i, e in enumerate(cams):
        cam = S.real_camera(e, **REALCAM_TAGS[tag])
        assert [cam["W"], cam["H"]] == list(z[f"WH_{tag}_{i}"])
        np.testing.assert_array_equal(cam["viewmatrix"].numpy(), z[f"view_{tag}_{i}"])
        np.testing.assert_array_equal(cam["projmatrix"].numpy(), z[f"proj_{tag}_{i}"])
        np.testing.assert_allclose(cam["campos"].numpy(), z[f"campos_{tag}_{i}"], rtol=1e-6, atol=0)
        np.testing.assert_allclose([cam["tanfovx"], cam["tanfovy"]], z[f"tanfov_{tag}_{i}"], rtol=1e-15)
    assert len({(e["width"], e["height"]) for e in cams}) >= 4 and all(e["fx"] != e["fy"] for e in cams)


def real_camera_small(i, W, H, bg=(0.0, 0.0, 0.0), **kw):
    """Real camera i of the fixture, kept at its own FoV and rendered at W x H (small enough for float64 autograd)."""
    return S.real_camera(S.load_real_cameras()[i], W=W, H=H, bg=bg, **kw)


# ------------------------------------------------------------------------------------------------------
# float64 autograd restatement
# ------------------------------------------------------------------------------------------------------
C0 = 0.28209479177387814
C1 = 0.4886025119029199
C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
      1.445305721320277, -0.5900435899266435]


def _sh_rgb(deg, sh, d):
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    r = C0 * sh[:, 0]
    if deg > 0:
        r = r - C1 * y * sh[:, 1] + C1 * z * sh[:, 2] - C1 * x * sh[:, 3]
    if deg > 1:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        r = (r + C2[0] * xy * sh[:, 4] + C2[1] * yz * sh[:, 5] + C2[2] * (2 * zz - xx - yy) * sh[:, 6]
             + C2[3] * xz * sh[:, 7] + C2[4] * (xx - yy) * sh[:, 8])
    if deg > 2:
        r = (r + C3[0] * y * (3 * xx - yy) * sh[:, 9] + C3[1] * xy * z * sh[:, 10]
             + C3[2] * y * (4 * zz - xx - yy) * sh[:, 11] + C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12]
             + C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + C3[5] * z * (xx - yy) * sh[:, 14]
             + C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return torch.clamp_min(r + 0.5, 0.0)


class _AAScale(torch.autograd.Function):
    """h = sqrt(max(2.5e-5, det(cov)/det(cov + 0.3 I))) with the reference's backward
    (backward.cu:212-246).  Quirk: that backward evaluates d(ratio)/d(cov), derived for the undilated
    covariance, at the *dilated* entries (c_xx, c_yy already include +0.3), so it is not the exact
    derivative of its own forward.  Every other term of this restatement is plain autograd."""

    @staticmethod
    def forward(ctx, a, b, c):
        w = 0.3
        ratio = (a * c - b * b) / ((a + w) * (c + w) - b * b)
        h = torch.sqrt(torch.clamp_min(ratio, 2.5e-5))
        ctx.save_for_backward(a, b, c, ratio, h)
        return h

    @staticmethod
    def backward(ctx, g):
        a, b, c, ratio, h = ctx.saved_tensors
        w = 0.3
        d_inside = torch.where(ratio <= 2.5e-5, torch.zeros_like(g), g / (2 * h))
        x, y, z = a + w, c + w, b  # dilated, as the reference uses them
        den = d_inside / (w * w + w * (x + y) + x * y - z * z) ** 2
        return w * (w * y + y * y + z * z) * den, -2.0 * w * z * (w + x + y) * den, w * (w * x + x * x + z * z) * den


class _ClampST(torch.autograd.Function):
    """min(alpha, 0.99) whose gradient passes straight through: the alt rasterizer's backward has no
    o * G > 0.99 => dL/dalpha = 0 rule (alt-rasterizer/cuda_rasterizer/backward.cu:596-624)."""

    @staticmethod
    def forward(ctx, a):
        return torch.clamp(a, max=0.99)

    @staticmethod
    def backward(ctx, g):
        return g


def torch_render(sc, cam, fr, deg, alt=False, aa=True):
    """Differentiable float64 forward with the reference's semantics; the per-tile sorted lists come from
    the oracle frame (the sort itself has no gradient).  alt=True: the alt rasterizer's forward (AA scaling
    only when `aa`) with its backward's two departures from autograd modelled explicitly -- the clamp
    gradient passes through, and the T_final * bg term enters dL/dalpha twice (backward.cu:608, 619)."""
    dt = torch.float64
    leaf = lambda a: torch.tensor(np.asarray(a, np.float64), dtype=dt, requires_grad=True)  # noqa: E731
    P = sc["means3D"].shape[0]
    means, scales, rots = leaf(sc["means3D"]), leaf(sc["scales"]), leaf(sc["rotations"])
    opac, shs = leaf(sc["opacities"]), leaf(sc["shs"])
    if alt:  # dc + rest as separate leaves, concatenated for the SH polynomial
        dc_l = leaf(sc["dc"])
        shs = leaf(sc["shs"])
        sh_all = torch.cat([dc_l, shs], 1)
    else:
        sh_all = shs
    W, H = cam["W"], cam["H"]
    view = torch.tensor(cam["viewmatrix"].numpy().reshape(4, 4), dtype=dt)
    proj = torch.tensor(cam["projmatrix"].numpy().reshape(4, 4), dtype=dt)
    campos = torch.tensor(cam["campos"].numpy(), dtype=dt)
    fx = W / (2 * cam["tanfovx"])
    fy = H / (2 * cam["tanfovy"])
    ph = torch.cat([means, torch.ones(P, 1, dtype=dt)], 1)
    tview = ph @ view
    hom = ph @ proj
    ndc = hom[:, :2] / (hom[:, 3:4] + 1e-7)
    ndc.retain_grad()
    pix = ((ndc + 1) * torch.tensor([W, H], dtype=dt) - 1) * 0.5
    # cov3D = R diag(s^2) R^T with the reference's (unnormalised) quaternion polynomial
    r, x, y, z = rots[:, 0], rots[:, 1], rots[:, 2], rots[:, 3]
    Rs = torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], -1),
        torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], -1),
        torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1)], -2)
    Sig = Rs @ torch.diag_embed(scales ** 2) @ Rs.transpose(1, 2)
    A = view[:3, :3].T  # linear part of the view transform acting on column vectors
    tz = tview[:, 2]
    limx, limy = 1.3 * cam["tanfovx"], 1.3 * cam["tanfovy"]
    tx = torch.clamp(tview[:, 0] / tz, -limx, limx) * tz
    ty = torch.clamp(tview[:, 1] / tz, -limy, limy) * tz
    zero = torch.zeros_like(tz)
    J = torch.stack([torch.stack([fx / tz, zero, -fx * tx / (tz * tz)], -1),
                     torch.stack([zero, fy / tz, -fy * ty / (tz * tz)], -1)], -2)
    JA = J @ A
    cov2 = JA @ Sig @ JA.transpose(1, 2)
    a, b, c = cov2[:, 0, 0], cov2[:, 0, 1], cov2[:, 1, 1]
    hs = _AAScale.apply(a, b, c) if aa else torch.ones_like(a)
    a, c = a + 0.3, c + 0.3
    det = a * c - b * b
    conic = torch.stack([c / det, -b / det, a / det], -1)
    o2 = opac[:, 0] * hs
    d = means - campos
    rgb = _sh_rgb(deg, sh_all, d / d.norm(dim=1, keepdim=True))
    invz = 1.0 / tz
    bg = torch.tensor(cam["bg"].numpy(), dtype=dt)
    gx = (W + 15) // 16
    color = torch.zeros(3, H, W, dtype=dt)
    inv = torch.zeros(1, H, W, dtype=dt)
    for t, (s, e) in enumerate(fr.ranges.astype(np.int64)):
        tx0, ty0 = (t % gx) * 16, (t // gx) * 16
        xs = torch.arange(tx0, min(tx0 + 16, W), dtype=dt)
        ys = torch.arange(ty0, min(ty0 + 16, H), dtype=dt)
        py, px = torch.meshgrid(ys, xs, indexing="ij")
        px, py = px.reshape(-1, 1), py.reshape(-1, 1)
        if e > s:
            ids = torch.tensor(fr.point_list[s:e].astype(np.int64))
            dx = pix[ids, 0][None] - px
            dy = pix[ids, 1][None] - py
            cn = conic[ids]
            power = -0.5 * (cn[None, :, 0] * dx * dx + cn[None, :, 2] * dy * dy) - cn[None, :, 1] * dx * dy
            raw = o2[ids][None] * torch.exp(power)
            alpha = _ClampST.apply(raw) if alt else torch.clamp(raw, max=0.99)
            keep = (power <= 0) & (alpha >= 1.0 / 255.0)
            alpha = torch.where(keep, alpha, torch.zeros_like(alpha))
            one_m = 1 - alpha
            Tb = torch.cumprod(torch.cat([torch.ones_like(one_m[:, :1]), one_m[:, :-1]], 1), 1)
            stop = keep & (Tb * one_m < 1e-4)
            dead = torch.cumsum(stop.to(torch.int64), 1) > 0  # the stopping splat and everything behind it
            alpha = torch.where(dead, torch.zeros_like(alpha), alpha)
            Tb = torch.cumprod(torch.cat([torch.ones_like(alpha[:, :1]), (1 - alpha)[:, :-1]], 1), 1)
            w = alpha * Tb
            Tf = Tb[:, -1] * (1 - alpha[:, -1])
            col = w @ rgb[ids] + Tf[:, None] * bg[None]
            if alt:
                col = col + (Tf - Tf.detach())[:, None] * bg[None]
            dep = w @ invz[ids]
        else:
            col = bg[None].expand(px.shape[0], 3)
            dep = torch.zeros(px.shape[0], dtype=dt)
        hh, ww = len(ys), len(xs)
        color[:, ty0:ty0 + hh, tx0:tx0 + ww] = col.T.reshape(3, hh, ww)
        inv[0, ty0:ty0 + hh, tx0:tx0 + ww] = dep.reshape(hh, ww)
    out = dict(color=color, invdepth=inv, means=means, scales=scales, rots=rots, opac=opac, shs=shs, ndc=ndc)
    if alt:
        out["dc"] = dc_l
    return out


def _fwd_tol_far(cam, sc):
    """Forward tolerance of the float32 oracle against float64 for a camera far from the world origin.  The real
    cameras sit up to ~133 units from it, so the float32 view transform p_view = R p + t cancels terms of that size
    down to depths of 2-30: its rounding moves a splat centre by ~eps * |t| * f / z pixels (~2e-3 px here), which the
    float64 restatement of the same float32 inputs does not have.  The bound scales 1e-5 by |t| / min depth (>= 1):
    a wrong view matrix or a swapped focal length moves pixels by O(1), far above it."""
    t = float(np.abs(cam["viewmatrix"].numpy()[3, :3]).max())
    zmin = float((np.c_[sc["means3D"], np.ones(len(sc["means3D"]))] @ cam["viewmatrix"].numpy().astype(np.float64))[:, 2].min())
    return 1e-5 * max(1.0, t / max(zmin, 1e-3))


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-12)


@pytest.mark.parametrize("P,deg,W,H,bg,realcam", [(250, 3, 64, 48, (0.0, 0.0, 0.0), None),
                                                  (300, 1, 48, 40, (0.2, 0.5, 0.8), None),
                                                  (150, 0, 40, 40, (0.1, 0.1, 0.1), None),
                                                  (250, 3, 60, 44, (0.3, 0.2, 0.1), 0),
                                                  (300, 2, 52, 36, (0.0, 0.0, 0.0), 5),
                                                  (250, 1, 47, 41, (0.6, 0.3, 0.2), 9)])
def test_oracle_matches_float64_autograd(P, deg, W, H, bg, realcam):
    """realcam: one of the reference's own cameras (rotated view matrix, fx != fy; camera 9 with an off-centre
    principal point), so T = W J of computeCov2D (forward.cu:141-176) and the mean-gradient chain through the view
    matrix (backward.cu:285-312, 433-447) are exercised with a non-identity W."""
    if realcam is None:
        cam = S.make_camera(W, H, bg=bg)
    else:
        cam = real_camera_small(realcam, W, H, bg=bg, **(dict(primx=0.47, primy=0.53) if realcam == 9 else {}))
    sc = S.make_gaussians(P, deg, cam, seed=P)
    fr = O.forward(sc, S.cam_numpy(cam))
    g, gd = S.upstream_grads(W, H)
    gr = O.backward(fr, sc, g, gd)
    tr = torch_render(sc, cam, fr, deg)
    tol = 1e-5 if realcam is None else _fwd_tol_far(cam, sc)
    assert _rel(fr.color, tr["color"].detach().numpy()) < tol
    assert _rel(fr.invdepth, tr["invdepth"].detach().numpy()) < tol
    loss = (tr["color"] * torch.tensor(g, dtype=torch.float64)).sum() + \
        (tr["invdepth"] * torch.tensor(gd, dtype=torch.float64)).sum()
    loss.backward()
    vis = fr.radii > 0
    checks = [("dmean3D", tr["means"].grad), ("dscale", tr["scales"].grad), ("drot", tr["rots"].grad),
              ("dopacity", tr["opac"].grad), ("dsh", tr["shs"].grad)]
    for name, ref in checks:
        e = _rel(gr[name][vis], ref.numpy()[vis])
        assert e < 2e-3, f"{name}: oracle vs autograd rel err {e}"
    e = _rel(gr["dmean2D"][vis, :2], tr["ndc"].grad.numpy()[vis])
    assert e < 2e-3, f"dmean2D: {e}"
    # invisible Gaussians receive exactly zero
    for name in ("dmean3D", "dscale", "drot", "dopacity", "dsh"):
        assert np.all(gr[name][~vis] == 0)


def test_oracle_zero_instances_and_empty():
    cam = S.make_camera(32, 32, bg=(0.5, 0.5, 0.5))
    sc = S.make_gaussians(50, 0, cam, seed=1)
    sc["means3D"][:, 2] = -3.0
    fr = O.forward(sc, S.cam_numpy(cam))
    assert fr.R == 0 and np.all(fr.color == 0)  # App. A-7: 0, not bg
    gr = O.backward(fr, sc, *S.upstream_grads(32, 32))
    assert all(np.all(v == 0) for v in gr.values() if v is not None)


def test_oracle_point_list_is_stable_tile_depth_order():
    cam = S.make_camera(64, 64)
    sc = S.make_gaussians(500, 0, cam, seed=2)
    sc["means3D"][::2, 2] = 7.0  # many exact depth ties
    fr = O.forward(sc, S.cam_numpy(cam))
    for s, e in fr.ranges:
        ids = fr.point_list[s:e]
        keys = [(fr.depths[i], i) for i in ids]
        assert keys == sorted(keys)


def alt_scene(sc, antialiasing=True):
    """The same Gaussians in the alt rasterizer's layout: dc (P,1,3) + the remaining coefficients."""
    out = dict(sc)
    out["dc"] = np.ascontiguousarray(sc["shs"][:, :1])
    out["shs"] = np.ascontiguousarray(sc["shs"][:, 1:])
    out["alt"] = True
    out["antialiasing"] = antialiasing
    return out


@pytest.mark.parametrize("P,deg,W,H,bg,aa,realcam", [(250, 3, 64, 48, (0.0, 0.0, 0.0), True, None),
                                                     (300, 2, 48, 40, (0.2, 0.5, 0.8), False, None),
                                                     (200, 1, 40, 40, (0.3, 0.1, 0.6), True, None),
                                                     (250, 3, 60, 44, (0.2, 0.4, 0.6), True, 3),
                                                     (250, 1, 45, 39, (0.0, 0.0, 0.0), False, 7)])
def test_alt_oracle_matches_float64_autograd(P, deg, W, H, bg, aa, realcam):
    """alt-rasterizer restatement (dc/rest split, optional AA, per-tile culling, its own backward); realcam as in
    test_oracle_matches_float64_autograd."""
    cam = S.make_camera(W, H, bg=bg) if realcam is None else real_camera_small(realcam, W, H, bg=bg)
    sc = alt_scene(S.make_gaussians(P, deg, cam, seed=P + 7), aa)
    sc["opacities"][: P // 10] = 0.999  # some splats reach the 0.99 clamp
    fr = O.forward(sc, S.cam_numpy(cam))
    assert fr.invdepth.shape == (1, H, W)
    g, gd = S.upstream_grads(W, H)
    gr = O.backward(fr, sc, g, gd)
    tr = torch_render(sc, cam, fr, deg, alt=True, aa=aa)
    tol = 1e-5 if realcam is None else _fwd_tol_far(cam, sc)
    assert _rel(fr.color, tr["color"].detach().numpy()) < tol
    assert _rel(fr.invdepth, tr["invdepth"].detach().numpy()) < tol
    loss = (tr["color"] * torch.tensor(g, dtype=torch.float64)).sum() + \
        (tr["invdepth"] * torch.tensor(gd, dtype=torch.float64)).sum()
    loss.backward()
    vis = fr.radii > 0
    checks = [("dmean3D", tr["means"].grad), ("dscale", tr["scales"].grad), ("drot", tr["rots"].grad),
              ("dopacity", tr["opac"].grad), ("dsh", tr["shs"].grad), ("ddc", tr["dc"].grad)]
    for name, ref in checks:
        e = _rel(gr[name][vis], ref.numpy()[vis])
        assert e < 2e-3, f"{name}: alt oracle vs autograd rel err {e}"
    e = _rel(gr["dmean2D"][vis, :2], tr["ndc"].grad.numpy()[vis])
    assert e < 2e-3, f"dmean2D: {e}"


def test_alt_oracle_culls_tiles_and_renders_bg_when_empty():
    cam = S.make_camera(64, 64, bg=(0.5, 0.25, 0.75))
    sc = alt_scene(S.make_gaussians(400, 1, cam, seed=3))
    fr = O.forward(sc, S.cam_numpy(cam))
    kept = int((fr.ranges[:, 1] - fr.ranges[:, 0]).sum())
    assert 0 < kept < fr.R  # some rect tiles are culled; num_rendered still counts them (sentinels)
    assert np.all(fr.point_list[kept:] == 0xFFFFFFFF)
    # every Gaussian/tile pair culled away contributes nothing: no pixel of that tile reaches alpha >= 1/255
    sc["means3D"][:, 2] = -3.0  # everything behind the camera: R == 0, the alt rasterizer still renders bg
    fr = O.forward(sc, S.cam_numpy(cam))
    assert fr.R == 0
    np.testing.assert_array_equal(fr.color, np.broadcast_to(np.float32([0.5, 0.25, 0.75])[:, None, None], (3, 64, 64)))


@pytest.mark.parametrize("P,deg,W,H,alt,elong", [(3000, 3, 160, 112, False, 0.0), (2500, 1, 128, 96, True, 0.0),
                                                 (3000, 2, 144, 96, False, 2.5)])
def test_drop_empty_changes_lists_not_images(P, deg, W, H, alt, elong):
    """drop_empty (the HIP binning with packed entries and HLGS_DROP_EMPTY) bins no instance whose footprint quadrant
    mask is 0.  The mask test is conservative (tools/cull_check.py), so such an instance reaches no pixel of its tile:
    the image, inverse depth, transmittance and every gradient stay bit-identical, the lists get shorter, num_rendered
    (record slots) stays, and every pixel's last contributor is the same Gaussian."""
    cam = S.make_camera(W, H, bg=(0.1, 0.2, 0.3))
    sc = S.make_gaussians(P, deg, cam, seed=P + deg)
    if elong:  # strongly anisotropic splats: the band test's widest cases
        rng = np.random.default_rng(7)
        sc["scales"] = np.ascontiguousarray(sc["scales"] * np.exp(rng.uniform(-elong, elong, sc["scales"].shape))
                                            .astype(np.float32))
    if alt:
        sc = alt_scene(sc)
    g = S.upstream_grads(W, H, seed=2)
    a = O.forward(dict(sc), S.cam_numpy(cam))
    b = O.forward(dict(sc), S.cam_numpy(cam), drop_empty=True)
    ka = int((a.ranges[:, 1].astype(np.int64) - a.ranges[:, 0]).sum())
    kb = int((b.ranges[:, 1].astype(np.int64) - b.ranges[:, 0]).sum())
    # the alt rasterizer's exact per-tile culling already removes nearly every such instance
    assert a.R == b.R and (kb <= ka if alt else kb < 0.95 * ka), (a.R, ka, kb)
    for k in ("color", "invdepth", "final_T", "radii", "seen"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)
    ga, gb = O.backward(a, dict(sc), *g), O.backward(b, dict(sc), *g)
    for k in ga:
        if ga[k] is not None:
            np.testing.assert_array_equal(ga[k], gb[k], err_msg=k)
    gx = (W + 15) // 16
    pix = np.arange(W * H)
    tile = (pix // W // 16) * gx + (pix % W) // 16
    live = (a.n_contrib > 0) & (b.n_contrib > 0)
    assert np.array_equal(a.n_contrib > 0, b.n_contrib > 0)
    la = a.point_list[a.ranges[tile[live], 0] + a.n_contrib[live] - 1]
    lb = b.point_list[b.ranges[tile[live], 0] + b.n_contrib[live] - 1]
    np.testing.assert_array_equal(la, lb)


# ------------------------------------------------------------------------------------------------------
# Reference-run fixtures for the Python pieces of the path (tests/golden/make_golden.py)

@pytest.mark.parametrize("i", [0, 1, 2])
def test_cov3d_matches_reference_build_covariance(i):
    """K1's computeCov3D (forward.cu:181-215) in the oracle against the reference's own Python covariance
    (build_scaling_rotation + strip_symmetric, scene/gaussian_model.py:678-682) on the normalised quaternions
    get_rotation hands the rasterizer (the kernel does not normalise, gaussian_model.py:691)."""
    z = np.load(os.path.join(GOLD, "golden_cov3d.npz"))
    s, r, mod = z[f"scales_{i}"], z[f"rotations_{i}"], float(z[f"modifier_{i}"])
    P = s.shape[0]
    rn = (r / np.linalg.norm(r.astype(np.float64), axis=1, keepdims=True)).astype(np.float32)
    cam = S.cam_numpy(S.make_camera(64, 64))
    sc = dict(means3D=np.tile(np.array([[0.0, 0.0, 5.0]], np.float32), (P, 1)), scales=s, rotations=rn,
              opacities=np.full((P, 1), 0.5, np.float32), colors_precomp=np.zeros((P, 3), np.float32),
              scale_modifier=mod)
    fr = O.forward(sc, cam)
    want = z[f"cov3D_{i}"].astype(np.float64)
    scale = np.abs(want).max(1, keepdims=True)  # per-Gaussian: the entries are products of scales
    np.testing.assert_allclose(fr.cov3D / scale, want / scale, rtol=0, atol=2e-6)


@pytest.mark.parametrize("i", [0, 1, 2])
def test_lod_lerp_matches_reference_render_post(i):
    """The oracle's lerp and its backward against render_post's interpolation block run from the reference
    (gaussian_renderer/__init__.py:304-339) and torch autograd through it."""
    z = np.load(os.path.join(GOLD, "golden_lerp.npz"))
    sky = int(z[f"skybox_points_{i}"])
    ri, pi, w = z[f"render_indices_{i}"], z[f"parent_indices_{i}"], z[f"weights_{i}"]
    leaves = [z[f"{k}_{i}"] for k in ("xyz", "scaling", "rotation", "opacity", "features")]
    keys = ("means", "scales", "rots", "opac", "shs")
    out = O.lod_interp_forward(sky, ri, pi, w, *leaves)
    for k in keys:
        want = z[f"out_{k}_{i}"]
        np.testing.assert_allclose(out[k].reshape(want.shape), want, rtol=1e-6, atol=1e-7, err_msg=k)
    d = O.lod_interp_backward(sky, ri, pi, w, leaves[2], leaves[0].shape[0], {k: z[f"up_{k}_{i}"] for k in keys})
    for k in keys:
        want = z[f"grad_{k}_{i}"]
        np.testing.assert_allclose(d[k].reshape(want.shape), want, rtol=1e-5, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("alt", [False, True])
def test_openmp_oracle_is_bitwise_serial(alt):
    """The OpenMP build (per-tile parallel blend and blend backward, per-Gaussian parallel preprocess and backward)
    computes exactly what the serial build does -- every image, list and gradient bit -- because the blend backward sums
    per (tile, Gaussian) record and adds the records in tile order (tile_records).  So the OpenMP build can stand in for
    the serial oracle on full-size frames (tests/test_gpu_scale.py, configs[3] at 4M Gaussians)."""
    from hlgs_core import synthetic as S
    W, H = 320, 240
    cam = S.cam_numpy(S.make_camera(W, H, bg=(0.2, 0.1, 0.3)))
    sc = S.make_gaussians(30000, 3, cam, seed=41)
    if alt:
        sc = dict(sc, alt=True, antialiasing=True, dc=sc["shs"][:, :1].copy(), shs=sc["shs"][:, 1:].copy())
    g, gd = S.upstream_grads(W, H, seed=5)
    outs = []
    for omp in (False, True):
        fr = O.forward(sc, cam, do_depth=True, omp=omp, drop_empty=True)
        gr = O.backward(fr, sc, g, gd)
        outs.append((fr, gr))
    (f0, g0), (f1, g1) = outs
    for k in ("color", "invdepth", "final_T", "n_contrib", "ranges", "radii", "means2D", "conic_opacity"):
        np.testing.assert_array_equal(getattr(f0, k), getattr(f1, k), err_msg=k)
    np.testing.assert_array_equal(f0.point_list[:f0.R], f1.point_list[:f1.R])
    for k, v in g0.items():
        if v is not None:
            np.testing.assert_array_equal(v.view(np.uint32), g1[k].view(np.uint32), err_msg=k)
    assert O.num_threads(True) > 1  # the comparison means something only with several threads
