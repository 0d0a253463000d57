"""The binning plan's failure path and the reference-layout binning option, against the oracle.

- The fused plan (k_tile_offsets_plan) bounds every look-back poll.  hlgs_set_plan_polls(0) makes every block that has
  to wait time out at once: the frame must then be re-planned with the two-launch plan (k_tile_offsets + k_plan) and
  match the oracle exactly -- ranges, point_list, n_contrib, image and gradients -- instead of failing or rendering
  wrong lists (a middle block's timeout is reported through misc[kMiscFail]).
- hlgs_set_drop_empty(0) bins every instance of the reference's binning (rasterizer_impl.cu:70-115), zero-mask ones
  included, so point_list and n_contrib are bit-exact with the oracle's reference layout (drop_empty=False).
"""
import numpy as np
import pytest
import torch

from hlgs_core import _lib as L
from hlgs_core import synthetic as S
from oracle import oracle as O
from helpers import assert_grad, binned, drops_empty, gpu_render, image_check, oracle_render

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _raster(sc, cam, deg):
    from diff_gaussian_rasterization import _C
    W, H = cam["W"], cam["H"]
    t = lambda a: torch.tensor(a, device=DEV)  # noqa: E731
    e = torch.empty(0, device=DEV)
    return _C, _C.rasterize_gaussians(cam["bg"], e, e, e, e, t(sc["means3D"]), e, t(sc["opacities"]), t(sc["scales"]),
                                      t(sc["rotations"]), 1.0, e, cam["viewmatrix"], cam["projmatrix"],
                                      cam["tanfovx"], cam["tanfovy"], H, W, t(sc["shs"]), deg, cam["campos"], False,
                                      True, True)


def _lists_match(sc, cam, deg, drop):
    P = sc["means3D"].shape[0]
    W, H = cam["W"], cam["H"]
    fr = O.forward(dict(sc), S.cam_numpy(cam), drop_empty=drop)
    _C, out = _raster(sc, cam, deg)
    assert out[0] == fr.R
    kept = binned(fr)
    np.testing.assert_array_equal(_C.inspect_ranges(out[5], W, H).cpu().numpy().astype(np.uint32), fr.ranges)
    np.testing.assert_array_equal(_C.inspect_point_list(out[4], kept, P).cpu().numpy().astype(np.uint32),
                                  fr.point_list[:kept])
    N = W * H
    n_contrib = _C._field(out[5], (4 * N + 255) // 256 * 256, N, torch.int32).cpu().numpy()
    np.testing.assert_array_equal(n_contrib, fr.n_contrib.astype(np.int32))
    mx, nbad, ok = image_check(out[1].cpu().numpy(), fr.color)
    assert ok, (mx, nbad)
    return fr


@pytest.mark.parametrize("P,W,H", [(60000, 1024, 768), (8000, 320, 200)])
def test_plan_lookback_timeout_replans(P, W, H):
    lib = L.load()
    cam = S.make_camera(W, H)
    sc = S.make_gaussians(P, 2, cam, seed=31)
    try:
        lib.hlgs_set_plan_polls(0)  # every waiting block of the fused plan times out at once
        _lists_match(sc, cam, 2, drops_empty(P))
        g = S.upstream_grads(W, H, seed=2)
        gpu = gpu_render(sc, cam, grads=g)
        ref = oracle_render(sc, cam, grads=g, drop_empty=drops_empty(P))
        mx, nbad, ok = image_check(gpu["color"], ref["color"])
        assert ok, (mx, nbad)
        for k in ref:
            if k.startswith("d"):
                assert_grad(k, gpu[k][..., :ref[k].shape[-1]], ref[k])
    finally:
        lib.hlgs_set_plan_polls(1 << 20)
    # and the next frame, with the default bound, takes the fused plan again
    _lists_match(sc, cam, 2, drops_empty(P))


@pytest.mark.parametrize("P,W,H", [(20000, 256, 192), (3000, 96, 80)])
def test_drop_empty_off_gives_reference_lists(P, W, H):
    lib = L.load()
    cam = S.make_camera(W, H)
    sc = S.make_gaussians(P, 1, cam, seed=17)
    try:
        lib.hlgs_set_drop_empty(0)
        assert lib.hlgs_point_list_drops_empty(P) == 0
        fr_ref = _lists_match(sc, cam, 1, False)
        g = S.upstream_grads(W, H, seed=4)
        gpu = gpu_render(sc, cam, grads=g)
        ref = oracle_render(sc, cam, grads=g, drop_empty=False)
        for k in ref:
            if k.startswith("d"):
                assert_grad(k, gpu[k][..., :ref[k].shape[-1]], ref[k])
    finally:
        lib.hlgs_set_drop_empty(1)
    assert lib.hlgs_point_list_drops_empty(P) == 1
    fr_drop = _lists_match(sc, cam, 1, True)
    assert binned(fr_drop) < binned(fr_ref)  # the default leaves the zero-mask instances out


def test_switch_flipped_during_frames_is_per_frame():
    """The binning switches are read once per frame (FrameOpts): a thread flips drop_empty while
    this one renders.  Every frame's hlgs_frame_info.drops_empty must equal the drop word its own plan kernel wrote
    (Img::misc[4]) and its binned count must be the oracle's for that setting -- never a mix of the two."""
    import ctypes as C
    import threading
    from diff_gaussian_rasterization import _C
    lib = L.load()
    P, W, H = 20000, 256, 192
    cam = S.make_camera(W, H)
    sc = S.make_gaussians(P, 1, cam, seed=17)
    want = {d: binned(O.forward(dict(sc), S.cam_numpy(cam), drop_empty=d)) for d in (False, True)}
    assert want[True] < want[False]
    t = lambda a: torch.tensor(a, device=DEV)  # noqa: E731
    e = torch.empty(0, device=DEV)
    a, keep, P_, _, _ = _C._raster_args(cam["bg"], e, e, e, e, t(sc["means3D"]), e, t(sc["opacities"]),
                                        t(sc["scales"]), t(sc["rotations"]), 1.0, e, cam["viewmatrix"],
                                        cam["projmatrix"], cam["tanfovx"], cam["tanfovy"], H, W, t(sc["shs"]), 1,
                                        cam["campos"], False, False)
    u8 = dict(dtype=torch.uint8, device=DEV)
    geom = torch.empty((lib.hlgs_geom_buffer_size(P),), **u8)
    img = torch.empty((lib.hlgs_image_buffer_size(W, H),), **u8)
    binning = torch.empty((lib.hlgs_binning_buffer_size(2 * want[False]),), **u8)
    radii = torch.empty((P,), dtype=torch.int32, device=DEV)
    color = torch.empty((3, H, W), device=DEV)
    stop = threading.Event()

    def flip():
        on = 0
        while not stop.is_set():
            lib.hlgs_set_drop_empty(on)
            on ^= 1
    th = threading.Thread(target=flip)
    th.start()
    seen_flags = set()
    try:
        for _ in range(60):
            info = L.FrameInfo()
            L.check(lib.hlgs_rasterize_forward(C.byref(a), L.ptr(geom), L.ptr(img), L.ptr(radii), L.ptr(binning),
                                               binning.numel(), C.byref(info), L.ptr(color), None, None, L.stream()))
            assert info.rendered == 1
            misc = _C._field(img, lib.hlgs_image_misc_offset(W, H), 16, torch.int32).cpu().numpy()
            assert info.entry_shift == 4 and misc[3] == 1
            assert misc[4] == info.drops_empty, (misc[4], info.drops_empty)
            assert info.num_binned == want[bool(info.drops_empty)], (info.num_binned, info.drops_empty)
            seen_flags.add(info.drops_empty)
    finally:
        stop.set()
        th.join()
        lib.hlgs_set_drop_empty(1)
    del keep
    assert lib.hlgs_point_list_drops_empty(P) == 1
