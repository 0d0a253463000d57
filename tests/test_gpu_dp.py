"""View-DP gradient exchange on the GPU path: the rasterizer backward writes parameter gradients straight into the
exchange's flat buffer (hlgs_core.dp.direct_grad), autograd adopts them as .grad, and the values are bitwise the
ones the backward produces into fresh tensors."""
import numpy as np
import pytest
import torch

from helpers import settings_for
from hlgs_core import synthetic as S


@pytest.mark.gpu
def test_backward_writes_into_exchange_buffer():
    from diff_gaussian_rasterization import GaussianRasterizer
    from hlgs_core.dp import FlatGradExchange
    cam = S.make_camera(160, 96)
    sc = S.make_gaussians(4000, 3, cam, seed=3)
    g, gd = S.upstream_grads(160, 96, seed=4)
    t = lambda a: torch.tensor(np.ascontiguousarray(a), device="cuda", requires_grad=True)  # noqa: E731
    params = [t(sc["means3D"]), t(sc["scales"]), t(sc["rotations"]), t(sc["opacities"]), t(sc["shs"])]
    rast = GaussianRasterizer(settings_for(cam, 3, "cuda", do_depth=True))
    gc, gi = torch.tensor(g, device="cuda"), torch.tensor(gd, device="cuda")

    def run():
        for p in params:
            p.grad = None
        m, s, r, o, sh = params
        color, _, inv = rast(means3D=m, means2D=torch.zeros_like(m, requires_grad=True), opacities=o, shs=sh,
                             scales=s, rotations=r)
        torch.autograd.backward([color, inv], [gc, gi])
        torch.cuda.synchronize()
        return [p.grad for p in params]

    fresh = [x.clone() for x in run()]
    ex = FlatGradExchange(params)
    try:
        direct = run()
        lo, hi = ex.flat.data_ptr(), ex.flat.data_ptr() + 4 * ex.flat.numel()
        assert all(lo <= d.data_ptr() < hi for d in direct), "gradients were copied, not written in place"
        for a, b in zip(fresh, direct):
            assert torch.equal(a, b)
        # with .grad already set the backward must not write into the buffer it accumulates into
        m, s, r, o, sh = params
        color, _, inv = rast(means3D=m, means2D=torch.zeros_like(m, requires_grad=True), opacities=o, shs=sh,
                             scales=s, rotations=r)
        torch.autograd.backward([color, inv], [gc, gi])
        torch.cuda.synchronize()
        for a, p in zip(fresh, params):
            torch.testing.assert_close(p.grad, 2 * a, rtol=1e-6, atol=1e-6)
    finally:
        ex.close()


@pytest.mark.gpu
@pytest.mark.parametrize("alt", [False, True])
def test_split_backward_on_late_stream_matches(alt):
    """With an overlapping exchange the SH backward runs on the exchange's late stream
    (hlgs_rasterize_backward_split); after join() -- or allreduce() -- every gradient is bitwise the in-order
    backward's, read on the current stream with no device-wide synchronisation."""
    from hlgs_core.dp import FlatGradExchange
    cam = S.make_camera(160, 96)
    sc = S.make_gaussians(6000, 3, cam, seed=5)
    g, gd = S.upstream_grads(160, 96, seed=6)
    t = lambda a: torch.tensor(np.ascontiguousarray(a), device="cuda", requires_grad=True)  # noqa: E731
    gc, gi = torch.tensor(g, device="cuda"), torch.tensor(gd, device="cuda")
    if alt:
        from alt_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
        params = [t(sc["means3D"]), t(sc["scales"]), t(sc["rotations"]), t(sc["opacities"]), t(sc["shs"][:, :1]),
                  t(sc["shs"][:, 1:])]
        rast = GaussianRasterizer(GaussianRasterizationSettings(
            image_height=96, image_width=160, tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"],
            bg=torch.zeros(3, device="cuda"), scale_modifier=1.0, viewmatrix=cam["viewmatrix"].cuda(),
            projmatrix=cam["projmatrix"].cuda(), sh_degree=3, campos=cam["campos"].cuda(), prefiltered=False,
            debug=False, antialiasing=True))
    else:
        from diff_gaussian_rasterization import GaussianRasterizer
        params = [t(sc["means3D"]), t(sc["scales"]), t(sc["rotations"]), t(sc["opacities"]), t(sc["shs"])]
        rast = GaussianRasterizer(settings_for(cam, 3, "cuda", do_depth=True))

    def backward():
        for p in params:
            p.grad = None
        if alt:
            m, s, r, o, dc, sh = params
            color, _, inv = rast(means3D=m, means2D=torch.zeros_like(m, requires_grad=True), opacities=o, dc=dc,
                                 shs=sh, scales=s, rotations=r)
        else:
            m, s, r, o, sh = params
            color, _, inv = rast(means3D=m, means2D=torch.zeros_like(m, requires_grad=True), opacities=o, shs=sh,
                                 scales=s, rotations=r)
        torch.autograd.backward([color, inv], [gc, gi])

    backward()
    ref = [p.grad.clone() for p in params]
    ex = FlatGradExchange(params, overlap=True)
    try:
        for _ in range(3):
            backward()
            assert ex.pending is not None, "the SH backward did not run on the late stream"
            ex.join()  # no torch.cuda.synchronize(): ordering comes from the event alone
            got = [p.grad.clone() for p in params]
            ex.release()
            for a, b in zip(ref, got):
                assert torch.equal(a, b)
    finally:
        ex.close()


@pytest.mark.gpu
def test_overlap_two_renders_of_the_same_leaves_in_one_backward():
    """overlap=True with two rasterizer calls on the same leaves in one autograd pass: the second backward finds the
    parameter's view claimed, joins the late stream before autograd sums its gradient with the view, and the summed
    gradients are bitwise those of the in-order backward."""
    from diff_gaussian_rasterization import GaussianRasterizer
    from hlgs_core.dp import FlatGradExchange
    cam = S.make_camera(160, 96)
    sc = S.make_gaussians(6000, 3, cam, seed=7)
    g, gd = S.upstream_grads(160, 96, seed=8)
    t = lambda a: torch.tensor(np.ascontiguousarray(a), device="cuda", requires_grad=True)  # noqa: E731
    gc, gi = torch.tensor(g, device="cuda"), torch.tensor(gd, device="cuda")
    params = [t(sc["means3D"]), t(sc["scales"]), t(sc["rotations"]), t(sc["opacities"]), t(sc["shs"])]
    rast = GaussianRasterizer(settings_for(cam, 3, "cuda", do_depth=True))

    def backward():
        for p in params:
            p.grad = None
        m, s_, r, o, sh = params
        outs, grads = [], []
        for k in range(2):
            color, _, inv = rast(means3D=m, means2D=torch.zeros_like(m, requires_grad=True), opacities=o, shs=sh,
                                 scales=s_, rotations=r)
            outs += [color, inv]
            grads += [gc * (k + 1), gi]
        torch.autograd.backward(outs, grads)

    backward()
    ref = [p.grad.clone() for p in params]
    ex = FlatGradExchange(params, overlap=True)
    try:
        for _ in range(3):
            backward()
            ex.join()
            got = [p.grad.clone() for p in params]
            ex.release()
            for a, b in zip(ref, got):
                assert torch.equal(a, b)
    finally:
        ex.close()


@pytest.mark.gpu
@pytest.mark.parametrize("alt,overlap", [(False, False), (True, False), (False, True), (True, True)])
def test_colour_factored_sh_exchange(alt, overlap):
    """Colour-factored exchange (FlatGradExchange(colour_factor=...)): the backward hands the exchange dL/dRGB instead of
    the SH gradient and the exchange rebuilds it (hlgs_sh_grad_from_colour).  One view: every gradient bitwise the plain
    backward's.  Two views' rows rebuilt together: the average of the two views' SH (and dc) gradients.  overlap=True:
    the exchange joins any late SH-backward work before it reads this rank's colour row."""
    import ctypes as C
    from hlgs_core import _lib as L
    from hlgs_core.dp import FlatGradExchange
    W, H = 160, 96
    cams = [S.make_camera(W, H), S.make_camera(W, H, T=np.array([0.3, -0.1, 0.2]))]
    sc = S.make_gaussians(6000, 3, cams[0], seed=7)
    g, gd = S.upstream_grads(W, H, seed=8)
    t = lambda a: torch.tensor(np.ascontiguousarray(a), device="cuda", requires_grad=True)  # noqa: E731
    gc, gi = torch.tensor(g, device="cuda"), torch.tensor(gd, device="cuda")
    if alt:
        from alt_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
        params = [t(sc["means3D"]), t(sc["scales"]), t(sc["rotations"]), t(sc["opacities"]), t(sc["shs"][:, :1]),
                  t(sc["shs"][:, 1:])]

        def rast(cam):
            return GaussianRasterizer(GaussianRasterizationSettings(
                image_height=H, image_width=W, tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"],
                bg=torch.zeros(3, device="cuda"), scale_modifier=1.0, viewmatrix=cam["viewmatrix"].cuda(),
                projmatrix=cam["projmatrix"].cuda(), sh_degree=3, campos=cam["campos"].cuda(), prefiltered=False,
                debug=False, antialiasing=True))
        factor = dict(means=params[0], sh=params[5], dc=params[4])
    else:
        from diff_gaussian_rasterization import GaussianRasterizer
        params = [t(sc["means3D"]), t(sc["scales"]), t(sc["rotations"]), t(sc["opacities"]), t(sc["shs"])]

        def rast(cam):
            return GaussianRasterizer(settings_for(cam, 3, "cuda", do_depth=True))
        factor = dict(means=params[0], sh=params[4])

    def backward(cam):
        for p in params:
            p.grad = None
        if alt:
            m, s, r, o, dc, sh = params
            color, _, inv = rast(cam)(means3D=m, means2D=torch.zeros_like(m, requires_grad=True), opacities=o, dc=dc,
                                      shs=sh, scales=s, rotations=r)
        else:
            m, s, r, o, sh = params
            color, _, inv = rast(cam)(means3D=m, means2D=torch.zeros_like(m, requires_grad=True), opacities=o, shs=sh,
                                      scales=s, rotations=r)
        torch.autograd.backward([color, inv], [gc, gi])

    plain = []
    for cam in cams:
        backward(cam)
        plain.append([p.grad.clone() for p in params])
    ex = FlatGradExchange(params, colour_factor=factor, overlap=overlap)
    rows = []
    try:
        for cam, ref in zip(cams, plain):
            backward(cam)
            assert ex.cf.written, "the backward did not take the colour-factored path"
            ex.allreduce()  # one rank: the rebuild from this view's row alone (joins the late stream first)
            rows.append(ex.cf.mine.clone())
            for a, p in zip(ref, params):
                assert torch.equal(a, p.grad)
    finally:
        ex.close()
    # two views rebuilt together, averaged, against the mean of the two views' plain gradients
    P = params[0].shape[0]
    rows = torch.stack(rows).contiguous()
    sh_p = params[5] if alt else params[4]
    dsh = torch.empty_like(sh_p)
    ddc = torch.empty_like(params[4]) if alt else None
    lib = L.load()
    L.check(lib.hlgs_sh_grad_from_colour(P, 2, 3, sh_p.shape[1], L.VARIANT_ALT if alt else L.VARIANT_HIERARCHY,
                                         L.ptr(params[0].detach()), rows.data_ptr(), rows.data_ptr() + 16,
                                         rows.shape[1], 0.5, L.ptr(dsh), L.ptr(ddc) if alt else None, L.stream()))
    i_sh = 5 if alt else 4
    torch.testing.assert_close(dsh, 0.5 * (plain[0][i_sh] + plain[1][i_sh]), rtol=1e-6, atol=1e-7)
    if alt:
        torch.testing.assert_close(ddc, 0.5 * (plain[0][4] + plain[1][4]), rtol=1e-6, atol=1e-7)
