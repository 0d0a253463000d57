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
