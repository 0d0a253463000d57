"""GPU against the oracle under the reference's own cameras.

/root/reference/cameras.json holds 1,499 real cameras: six physical cameras with ragged images (1021-1028 x
686-690, so the last tile column and row are partial), arbitrary rotations, and fx != fy.  Twelve of them, spread
over the file, are committed with the matrices the reference's own utils/graphics_utils builds for them
(tests/golden/golden_realcam.npz; S.real_camera reproduces those bit for bit, tests/test_oracle.py).  With a
rotated view matrix:
  - computeCov2D's T = W J (forward.cu:141-176) is no longer J, so a transposed view matrix would show;
  - the mean gradient through the view matrix (backward.cu:285-312 via computeCov2DCUDA, :433-447 via the
    projection) mixes all three world axes;
  - focal_x != focal_y (rasterizer_impl.cu:246-247), so a swapped focal length would show.
Each seeded synthetic scene is placed in front of its camera by the camera-to-world transform (S.make_gaussians).
The cameras sit up to ~133 units from the world origin, as in the reference's dataset.

Criteria are the ones of every other parity test: radii, point_list, ranges, n_contrib, seen and the per-Gaussian
splat records (means2D, conic, opacity, colour, 1/depth) bit-exact; per-pixel L-inf <= 1e-4 with no exception;
every gradient within 1e-3 per tensor and element-wise (tests/helpers.py)."""
import numpy as np
import pytest
import torch

from hlgs_core import synthetic as S
from helpers import assert_grad, binned, drops_empty, gpu_render, image_check, oracle_render
from oracle import oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"
FWD_TOL = 1e-4
CAMS = S.load_real_cameras()


def _bg(i):
    return tuple(float(v) for v in np.random.default_rng(50 + i).uniform(0, 1, 3))


def _cam(i, **kw):
    return S.real_camera(CAMS[i], **kw)


def _check_frame(gpu, ref):
    np.testing.assert_array_equal(gpu["radii"], ref["radii"])
    for k in ("color", "invdepth"):
        mx, nbad, ok = image_check(gpu[k], ref[k], FWD_TOL)
        assert ok, f"{k}: L-inf {mx}, {nbad} pixels over {FWD_TOL}"
    for k in ref:
        if k.startswith("d"):
            assert_grad(k, gpu[k][..., :ref[k].shape[-1]], ref[k])


def _check_lists_and_records(sc, cam, deg):
    """The forward's integer outputs and the per-Gaussian splat records against the oracle frame, bit for bit."""
    from diff_gaussian_rasterization import _C
    W, H = cam["W"], cam["H"]
    fr = O.forward(dict(sc), S.cam_numpy(cam), drop_empty=drops_empty(sc["means3D"].shape[0]))
    t = lambda a: torch.tensor(a, device=DEV)  # noqa: E731
    e = torch.empty(0, device=DEV)
    out = _C.rasterize_gaussians(cam["bg"], e, e, e, e, t(sc["means3D"]), e, t(sc["opacities"]), t(sc["scales"]),
                                 t(sc["rotations"]), 1.0, e, cam["viewmatrix"], cam["projmatrix"], cam["tanfovx"],
                                 cam["tanfovy"], H, W, t(sc["shs"]), deg, cam["campos"], False, False, True)
    R = out[0]
    P = sc["means3D"].shape[0]
    assert R == fr.R and R > 0
    np.testing.assert_array_equal(_C.inspect_ranges(out[5], W, H).cpu().numpy().astype(np.uint32), fr.ranges)
    kept = binned(fr)
    np.testing.assert_array_equal(_C.inspect_point_list(out[4], kept, P).cpu().numpy().astype(np.uint32),
                                  fr.point_list[:kept])
    N = W * H
    n_contrib = _C._field(out[5], (4 * N + 255) // 256 * 256, N, torch.int32).cpu().numpy()
    np.testing.assert_array_equal(n_contrib, fr.n_contrib.astype(np.int32))
    np.testing.assert_array_equal(out[7].cpu().numpy(), fr.seen)
    rec = _C.inspect_splats(out[3], P).cpu().numpy()
    vis = out[2].cpu().numpy() > 0
    np.testing.assert_array_equal(rec[vis][:, 0:2], fr.means2D[vis])
    np.testing.assert_array_equal(rec[vis][:, 2:6], fr.conic_opacity[vis])
    np.testing.assert_array_equal(rec[vis][:, 6:9], fr.rgb[vis])
    np.testing.assert_array_equal(rec[vis][:, 9], (np.float32(1.0) / fr.depths[vis]).astype(np.float32))
    return fr


# (camera, SH degree, Gaussians, principal point): all 12 cameras at their native (ragged) sizes; cameras 2 and 9
# also with an off-centre principal point (the projection matrix's shear column, graphics_utils.py:51-77)
CASES = [(i, 3 if i % 2 == 0 else 0, 30_000, None) for i in range(12)] + \
        [(2, 3, 30_000, (0.47, 0.53)), (9, 1, 30_000, (0.53, 0.46))]


@pytest.mark.parametrize("i,deg,P,pp", CASES, ids=[f"cam{c[0]}-deg{c[1]}" + ("-pp" if c[3] else "") for c in CASES])
def test_realcam_forward_backward_parity(i, deg, P, pp):
    kw = dict(primx=pp[0], primy=pp[1]) if pp else {}
    cam = _cam(i, bg=_bg(i), **kw)
    assert cam["fx"] != cam["fy"] and not np.allclose(cam["R"], np.eye(3))
    sc = S.make_gaussians(P, deg, cam, seed=1000 + i)
    g = S.upstream_grads(cam["W"], cam["H"], seed=2 + i)
    _check_frame(gpu_render(sc, cam, grads=g), oracle_render(sc, cam, grads=g))


@pytest.mark.parametrize("i,deg", [(1, 3), (6, 0), (11, 2)])
def test_realcam_lists_and_records_bit_exact(i, deg):
    cam = _cam(i)
    sc = S.make_gaussians(20_000, deg, cam, seed=2000 + i)
    # elongated splats too: the cancelling quadratic form under a rotated W
    sc["scales"][::4] = (sc["scales"][::4] * np.float32([6.0, 0.3, 1.0])).astype(np.float32)
    _check_lists_and_records(sc, cam, deg)


def _alt_gpu(sc, cam, grads, aa):
    from alt_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    t = lambda a: torch.tensor(np.ascontiguousarray(a), device=DEV, requires_grad=True)  # noqa: E731
    means3D = t(sc["means3D"])
    means2D = torch.zeros_like(means3D, requires_grad=True)
    opac, scales, rots, dc, shs = t(sc["opacities"]), t(sc["scales"]), t(sc["rotations"]), t(sc["dc"]), t(sc["shs"])
    s = GaussianRasterizationSettings(image_height=cam["H"], image_width=cam["W"], tanfovx=cam["tanfovx"],
                                      tanfovy=cam["tanfovy"], bg=cam["bg"].to(DEV), scale_modifier=1.0,
                                      viewmatrix=cam["viewmatrix"].to(DEV), projmatrix=cam["projmatrix"].to(DEV),
                                      sh_degree=sc["sh_degree"], campos=cam["campos"].to(DEV), prefiltered=False,
                                      debug=False, antialiasing=aa)
    color, radii, invd = GaussianRasterizer(s)(means3D=means3D, means2D=means2D, opacities=opac, scales=scales,
                                               rotations=rots, dc=dc, shs=shs)
    g, gd = grads
    ((color * torch.tensor(g, device=DEV)).sum() + (invd * torch.tensor(gd, device=DEV)).sum()).backward()
    return dict(color=color.detach().cpu().numpy(), invdepth=invd.detach().cpu().numpy(), radii=radii.cpu().numpy(),
                dmean3D=means3D.grad.cpu().numpy(), dmean2D=means2D.grad.cpu().numpy(),
                dopacity=opac.grad.cpu().numpy(), dscale=scales.grad.cpu().numpy(), drot=rots.grad.cpu().numpy(),
                ddc=dc.grad.cpu().numpy(), dshs=shs.grad.cpu().numpy())


@pytest.mark.parametrize("i,deg,aa", [(0, 3, True), (4, 3, False), (7, 0, True), (10, 1, False)])
def test_realcam_alt_rasterizer_parity(i, deg, aa):
    """alt_gaussian_rasterization (train_post.py's rasterizer: eigen-radius rects with exact per-tile culling, dc/rest
    SH, antialiasing) under the same cameras against the oracle's alt restatement."""
    cam = _cam(i, bg=_bg(i))
    sc = S.make_gaussians(30_000, deg, cam, seed=3000 + i)
    sc["dc"] = np.ascontiguousarray(sc["shs"][:, :1])
    sc["shs"] = np.ascontiguousarray(sc["shs"][:, 1:])
    sc.update(alt=True, antialiasing=aa)
    g = S.upstream_grads(cam["W"], cam["H"], seed=3 + i)
    gpu = _alt_gpu(sc, cam, g, aa)
    fr = O.forward(dict(sc), S.cam_numpy(cam))
    gr = O.backward(fr, dict(sc), *g)
    ref = dict(color=fr.color, invdepth=fr.invdepth, radii=fr.radii, dmean3D=gr["dmean3D"], dmean2D=gr["dmean2D"],
               dopacity=gr["dopacity"], dscale=gr["dscale"], drot=gr["drot"], ddc=gr["ddc"], dshs=gr["dsh"])
    if deg == 0:  # no rest coefficients: the alt SH backward is skipped (A-19)
        ref.pop("ddc"), ref.pop("dshs"), gpu.pop("ddc"), gpu.pop("dshs")
    _check_frame(gpu, ref)


def test_realcam_1080p_configs1_frame():
    """configs[1]'s workload (1M Gaussians, SH degree 3, 1920x1080, inverse depth) seen through one of the
    reference's cameras, kept at its own FoV (so fx / fy = 1.07, non-square pixels), against the serial oracle."""
    cam = _cam(5, W=1920, H=1080)
    sc = S.make_gaussians(1_000_000, 3, cam, seed=0)
    g = S.upstream_grads(1920, 1080, seed=1)
    _check_frame(gpu_render(sc, cam, grads=g), oracle_render(sc, cam, grads=g))
