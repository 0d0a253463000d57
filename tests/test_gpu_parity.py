"""HIP path (libhlgs.so via the public API) against the oracle on identical seeded inputs.

Forward: per-pixel L-inf <= 1e-4 (BASELINE.json north_star), radii / tiles bit-exact.
Backward: max|gpu - oracle| / max|oracle| <= 1e-3 per gradient tensor (north_star "1e-3 rel").
"""
import numpy as np
import pytest
import torch

from hlgs_core import synthetic as S
from helpers import assert_grad, drops_empty, gpu_render, image_check, oracle_render, rel_err

pytestmark = pytest.mark.gpu

FWD_TOL = 1e-4
GRAD_TOL = 1e-3


def _scene(P, deg, W, H, seed=0, bg=(0.0, 0.0, 0.0), **kw):
    cam = S.make_camera(W, H, bg=bg)
    sc = S.make_gaussians(P, deg, cam, seed=seed, **kw)
    return sc, cam


def _compare(sc, cam, do_depth=True, use_colors=False, use_cov=False, grads=True):
    g = S.upstream_grads(cam["W"], cam["H"], seed=1, depth=do_depth) if grads else None
    gpu = gpu_render(sc, cam, do_depth=do_depth, grads=g, use_colors=use_colors, use_cov=use_cov)
    ref = oracle_render(sc, cam, do_depth=do_depth, grads=g, use_colors=use_colors, use_cov=use_cov,
                        drop_empty=drops_empty(sc["means3D"].shape[0]))
    np.testing.assert_array_equal(gpu["radii"], ref["radii"])
    mx, nbad, ok = image_check(gpu["color"], ref["color"], FWD_TOL)
    assert ok, f"color L-inf {mx} ({nbad} pixels over {FWD_TOL})"
    if do_depth:
        mx, nbad, ok = image_check(gpu["invdepth"], ref["invdepth"], FWD_TOL)
        assert ok, f"invdepth L-inf {mx} ({nbad} pixels)"
    else:
        assert gpu["invdepth"].shape[0] == 0
    if grads:
        for k in ref:
            if k.startswith("d"):
                assert_grad(k, gpu[k][..., :ref[k].shape[-1]], ref[k])
    return gpu, ref


# (10000, 0, 256, 256) is BASELINE configs[0] (10k Gaussians, SH degree 0, one 256x256 camera) on the GPU path
@pytest.mark.parametrize("P,deg,W,H", [(300, 0, 64, 64), (2000, 3, 128, 96), (1500, 1, 100, 75), (4000, 2, 256, 256),
                                       (10000, 0, 256, 256)])
def test_forward_backward_parity(P, deg, W, H):
    sc, cam = _scene(P, deg, W, H, seed=P)
    _compare(sc, cam)


def test_random_background_no_depth():
    sc, cam = _scene(1000, 3, 96, 64, bg=(0.3, 0.6, 0.9))
    _compare(sc, cam, do_depth=False)


def test_colors_precomp_path():
    sc, cam = _scene(800, 0, 80, 64)
    sc["colors_precomp"] = np.random.default_rng(3).uniform(0, 1, (800, 3)).astype(np.float32)
    _compare(sc, cam, use_colors=True)


def test_cov3d_precomp_path():
    sc, cam = _scene(800, 1, 80, 64)
    from oracle import oracle as O
    # build cov3D the way the oracle's preprocess does (scale_modifier 1)
    fr = O.forward(dict(means3D=sc["means3D"], opacities=sc["opacities"], shs=sc["shs"], sh_degree=1,
                        scales=sc["scales"], rotations=sc["rotations"]), S.cam_numpy(cam))
    sc["cov3D_precomp"] = fr.cov3D.copy()
    _compare(sc, cam, use_cov=True)


def test_empty_and_all_culled():
    sc, cam = _scene(200, 0, 64, 64)
    behind = dict(sc)
    behind["means3D"] = sc["means3D"].copy()
    behind["means3D"][:, 2] = -5.0  # everything behind the camera: R == 0, output 0 (not bg)
    cam_bg = S.make_camera(64, 64, bg=(0.5, 0.5, 0.5))
    gpu = gpu_render(behind, cam_bg, grads=S.upstream_grads(64, 64))
    assert np.all(gpu["color"] == 0) and np.all(gpu["radii"] == 0)
    assert np.all(gpu["dmean3D"] == 0)
    empty = {k: (v[:0] if isinstance(v, np.ndarray) else v) for k, v in sc.items()}
    gpu = gpu_render(empty, cam_bg, grads=None)
    assert gpu["color"].shape == (3, 64, 64) and np.all(gpu["color"] == 0)


def test_near_plane_straddle_and_opaque():
    sc, cam = _scene(1500, 2, 64, 64, zmin=0.15, zmax=0.6, opacity_std=4.0)
    _compare(sc, cam)


def test_depth_ties_keep_index_order():
    sc, cam = _scene(400, 0, 64, 64)
    sc["means3D"][:, 2] = 5.0  # identical depths: ties resolved by ascending Gaussian index
    gpu, ref = _compare(sc, cam)


def test_long_tile_lists_use_merge_path():
    # > 4096 instances in the tiles around the centre exercise the LDS-sort + merge-pass binning
    cam = S.make_camera(64, 64)
    sc = S.make_gaussians(9000, 0, cam, seed=5, zmin=10.0, zmax=12.0, xy_spread=0.05, sigma_px=(1.0, 2.0))
    _compare(sc, cam)


@pytest.mark.parametrize("P", [1400, 2600, 4700, 12500])
def test_long_tile_sort_lengths(P):
    """Clustered splats whose centre tiles hold ~1,025-2,048, ~2,049-4,096 and > 4,096 entries (runs of 4,096 plus a
    ragged last run): the block sort's three-substage LDS passes (bitonic_group), its wave-local passes, and the merge
    passes of the longest lists."""
    cam = S.make_camera(64, 64)
    sc = S.make_gaussians(P, 0, cam, seed=P, zmin=10.0, zmax=12.0, xy_spread=0.05, sigma_px=(1.0, 2.0))
    _compare(sc, cam)


def test_backward_is_deterministic():
    sc, cam = _scene(3000, 3, 128, 128, seed=9)
    g = S.upstream_grads(128, 128)
    a = gpu_render(sc, cam, grads=g)
    b = gpu_render(sc, cam, grads=g)
    for k in ("dmean3D", "dmean2D", "dopacity", "d_shs", "d_scales", "d_rotations"):
        np.testing.assert_array_equal(a[k], b[k])


def test_sh_rows_with_unusual_coefficient_count():
    """shs rows of 6 coefficients at degree 1 (not a square count): the generic SH paths."""
    sc, cam = _scene(1800, 2, 96, 80, seed=33)
    sc["shs"] = np.ascontiguousarray(sc["shs"][:, :6])
    sc["sh_degree"] = 1
    _compare(sc, cam)


def test_binning_capacity_fallback_matches():
    """One-call forward with a too-small cached binning buffer (second call path), an exact one and an
    oversized one all give the same frame and the same backward."""
    from diff_gaussian_rasterization import _C
    sc, cam = _scene(2500, 2, 160, 120, seed=21)
    g = S.upstream_grads(160, 120)
    dev = torch.device("cuda", torch.cuda.current_device())
    runs = []
    for hint in (1, 0, 1 << 26):
        _C._binning_hint[dev] = hint
        runs.append(gpu_render(sc, cam, grads=g))
    _C._binning_hint.pop(dev, None)
    for r in runs[1:]:
        for k in ("color", "invdepth", "radii", "dmean3D", "dopacity", "d_shs"):
            np.testing.assert_array_equal(runs[0][k], r[k])


def test_loss_through_one_output_only():
    """A loss on invdepth alone (color gradient None) or on color alone (invdepth gradient None) gives the
    same gradients as passing explicit zero upstream gradients."""
    sc, cam = _scene(1500, 1, 96, 64, seed=41)
    g, gd = S.upstream_grads(96, 64, seed=2)
    zero_g, zero_gd = np.zeros_like(g), np.zeros_like(gd)
    only_depth = gpu_render(sc, cam, grads=(None, gd))
    ref_depth = gpu_render(sc, cam, grads=(zero_g, gd))
    only_color = gpu_render(sc, cam, grads=(g, None))
    ref_color = gpu_render(sc, cam, grads=(g, zero_gd))
    for k in ("dmean3D", "dmean2D", "dopacity", "d_shs", "d_scales", "d_rotations"):
        np.testing.assert_array_equal(only_depth[k], ref_depth[k])
        np.testing.assert_array_equal(only_color[k], ref_color[k])


def test_mark_visible_and_relocation():
    from diff_gaussian_rasterization import GaussianRasterizer, compute_relocation
    from oracle import oracle as O
    from helpers import settings_for
    sc, cam = _scene(1000, 0, 64, 64, zmin=0.05, zmax=5.0)
    sc["means3D"][::3, 2] *= -1.0  # a third of the points behind the camera
    rast = GaussianRasterizer(settings_for(cam, 0, "cuda"))
    vis = rast.markVisible(torch.tensor(sc["means3D"], device="cuda")).cpu().numpy()
    np.testing.assert_array_equal(vis, O.mark_visible(sc["means3D"], cam["viewmatrix"].numpy(), cam["projmatrix"].numpy()))
    rng = np.random.default_rng(0)
    n_max = 51
    binoms = np.zeros((n_max, n_max), np.float32)
    from math import comb
    for n in range(n_max):
        for k in range(n + 1):
            binoms[n, k] = comb(n, k)
    op = rng.uniform(0.01, 0.99, 500).astype(np.float32)
    scl = rng.uniform(0.01, 1, (500, 3)).astype(np.float32)
    N = rng.integers(1, 8, 500).astype(np.int32)
    o_g, s_g = compute_relocation(torch.tensor(op, device="cuda"), torch.tensor(scl, device="cuda"),
                                  torch.tensor(N, device="cuda"), torch.tensor(binoms, device="cuda"), n_max)
    o_r, s_r = O.compute_relocation(op, scl, N, binoms, n_max)
    np.testing.assert_allclose(o_g.cpu().numpy(), o_r, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(s_g.cpu().numpy(), s_r, rtol=1e-4, atol=1e-6)


def test_wide_splats_balanced_binning():
    """As test_alt_wide_splats_balanced_binning, for the hierarchy rasterizer (every rect tile is binned)."""
    sc, cam = _scene(3000, 2, 512, 384, seed=33)
    sc["scales"][:6] *= 40.0
    sc["opacities"][:6] = np.float32(0.3)
    _compare(sc, cam)


def _transparent_dense(P, deg, W, H, seed, opacity=(0.01, 0.08)):
    """Many faint splats over a small image: tile lists of several hundred entries with every pixel still live
    hundreds of splats deep, so the backward's chunks (bwd_chunk_len) start from the forward's sampled state."""
    sc, cam = _scene(P, deg, W, H, seed=seed)
    rng = np.random.default_rng(seed)
    sc["opacities"] = rng.uniform(opacity[0], opacity[1], (P, 1)).astype(np.float32)
    return sc, cam


@pytest.mark.parametrize("P,deg,W,H,depth,op", [(6000, 3, 96, 64, True, (0.01, 0.08)), (9000, 1, 80, 80, False, (0.01, 0.08)),
                                                (3000, 0, 48, 32, True, (0.01, 0.08)), (8000, 2, 64, 64, True, (0.2, 0.9))])
def test_backward_chunks_from_sampled_state(P, deg, W, H, depth, op):
    """Chunked backward (one wave per (tile, chunk)) against the oracle's single back-to-front pass; the last case
    has pixels that stop (T < 1e-4) inside a chunk."""
    sc, cam = _transparent_dense(P, deg, W, H, seed=P, opacity=op)
    gpu, ref = _compare(sc, cam, do_depth=depth)
    # the frame really has multi-chunk tiles whose pixels are live at the chunk boundaries
    counts = np.diff(ref["frame"].ranges.astype(np.int64), axis=1).ravel()
    assert counts.max() > 2 * 192, counts.max()  # three chunks of at least kBwdChunk = 192 entries
    nc = ref["frame"].n_contrib
    assert nc.max() > 256, nc.max()
    if op[1] > 0.5:  # pixels stop (T would drop below 1e-4) inside the middle chunk
        assert 448 < np.median(nc) < 896 and nc.max() < counts.max()


@pytest.mark.parametrize("case", ["dense", "long_lists"])
def test_unpacked_tile_list_entries(case):
    """The plain-index tile lists that frames of 2^28 or more Gaussians use (hlgs_set_entry_packing(0) forces them
    here): the blends then test each splat's footprint themselves, with the same result."""
    from hlgs_core import _lib as L
    if case == "dense":
        sc, cam = _scene(4000, 3, 128, 96, seed=77)
    else:  # > 1,024 entries per tile around the centre: block LDS sort and merge passes
        cam = S.make_camera(64, 64)
        sc = S.make_gaussians(6000, 1, cam, seed=78, zmin=10.0, zmax=12.0, xy_spread=0.05, sigma_px=(1.0, 2.0))
    lib = L.load()
    lib.hlgs_set_entry_packing(0)
    try:
        assert lib.hlgs_point_list_entry_shift(1000) == 0
        _compare(sc, cam)
    finally:
        lib.hlgs_set_entry_packing(1)
    assert lib.hlgs_point_list_entry_shift(1000) == 4


def clamp_boundary_scene(step):
    """One splat on the optical axis of an odd-sized image: it projects exactly onto pixel centre (32, 32), so there
    dx = dy = 0, G = exp2(0) = 1 and the backward's test alpha o' G equals the record opacity o' = o h (h: the
    anti-aliasing compensation, forward.cu).  o is searched so that o' is exactly the float `step` ulps from 0.99f.
    The splat is wide (h ~ 0.996), so o < 1 and every float near 0.99f is some o h."""
    from oracle import oracle as O
    cam = S.make_camera(65, 65)
    target = np.float32(0.99)
    for _ in range(abs(step)):
        target = np.nextafter(target, np.float32(2.0 if step > 0 else 0.0))
    sc = dict(means3D=np.array([[0.0, 0.0, 4.0]], np.float32), scales=np.full((1, 3), 0.6, np.float32),
              rotations=np.array([[1.0, 0.0, 0.0, 0.0]], np.float32), opacities=np.array([[0.5]], np.float32),
              shs=np.full((1, 1, 3), 0.3, np.float32), sh_degree=0)
    h = O.forward(sc, S.cam_numpy(cam)).conic_opacity[0, 3] / np.float32(0.5)
    o = np.float32(target / h)
    for _ in range(64):
        sc["opacities"][0, 0] = o
        got = O.forward(sc, S.cam_numpy(cam)).conic_opacity[0, 3]
        if got == target:
            return sc, cam, target
        o = np.nextafter(o, np.float32(2.0 if got < target else 0.0))
    raise AssertionError("no opacity gives the target record opacity")


@pytest.mark.parametrize("step", [-1, 0, 1, 2])
def test_alpha_clamp_threshold_exact(step):
    """The backward zeroes dL/dalpha where o G > 0.99f (backward.cu:619, 693), decided exactly at the float boundary
    (ADVICE r03): the centre pixel's test alpha is prev(0.99f), 0.99f, next(0.99f) or next(next(0.99f))
    (clamp_boundary_scene); its dL/dalpha is kept for the first two and zeroed for the others, as the oracle does."""
    sc, cam, target = clamp_boundary_scene(step)
    gpu, ref = _compare(sc, cam)
    fr = ref["frame"]
    assert fr.means2D[0].tolist() == [32.0, 32.0] and fr.conic_opacity[0, 3] == target


def test_packing_switch_between_forward_and_backward():
    """The backward decodes the tile lists as the forward wrote them (the frame's packing decision travels in the image
    buffer, Img::misc[kMiscPack]), so turning hlgs_set_entry_packing off between a forward and its backward changes
    nothing."""
    from diff_gaussian_rasterization import GaussianRasterizer
    from helpers import settings_for
    from hlgs_core import _lib as L
    sc, cam = _scene(3000, 2, 128, 96, seed=91)
    g, gd = S.upstream_grads(128, 96, seed=3)
    ref = gpu_render(sc, cam, grads=(g, gd))
    t = lambda a: torch.tensor(np.ascontiguousarray(a), device="cuda", requires_grad=True)  # noqa: E731
    m, s_, r, o, sh = (t(sc[k]) for k in ("means3D", "scales", "rotations", "opacities", "shs"))
    m2 = torch.zeros_like(m, requires_grad=True)
    color, _, inv = GaussianRasterizer(settings_for(cam, 2, "cuda"))(means3D=m, means2D=m2, opacities=o, shs=sh,
                                                                      scales=s_, rotations=r)
    lib = L.load()
    lib.hlgs_set_entry_packing(0)
    try:
        torch.autograd.backward([color, inv], [torch.tensor(g, device="cuda"), torch.tensor(gd, device="cuda")])
    finally:
        lib.hlgs_set_entry_packing(1)
    for k, v in (("dmean3D", m), ("dopacity", o), ("d_shs", sh), ("d_scales", s_), ("d_rotations", r)):
        np.testing.assert_array_equal(v.grad.cpu().numpy(), ref[k], err_msg=k)
