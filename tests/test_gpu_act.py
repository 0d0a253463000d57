"""The fused parameter activations (hlgs_core.activations.activate, csrc/act.hip) against torch's own sigmoid / exp /
normalize (scene/gaussian_model.py:44-56), forward and backward, including a zero rotation (normalize's eps) and
saturated opacities."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("n", [1, 1000, 300_001])
def test_activate_matches_torch(n):
    from hlgs_core.activations import activate
    g = torch.Generator().manual_seed(n)
    op = (torch.randn(n, 1, generator=g) * 4).to(DEV)
    sc = (torch.randn(n, 3, generator=g) * 2 - 4).to(DEV)
    rot = torch.randn(n, 4, generator=g).to(DEV)
    op[0] = 40.0   # sigmoid saturates
    rot[0] = 0.0   # normalize's eps branch
    if n > 2:
        op[1] = -40.0
        rot[1] = torch.tensor([1e-20, 0.0, 0.0, 0.0])
    ins = [t.clone().requires_grad_(True) for t in (op, sc, rot)]
    ref_in = [t.clone().requires_grad_(True) for t in (op, sc, rot)]
    got = activate(*ins)
    ref = (torch.sigmoid(ref_in[0]), torch.exp(ref_in[1]), torch.nn.functional.normalize(ref_in[2]))
    for a, b in zip(got, ref):
        assert a.shape == b.shape
        np.testing.assert_allclose(a.detach().cpu().numpy(), b.detach().cpu().numpy(), rtol=2e-6, atol=1e-30)
    ups = [torch.randn(t.shape, generator=g).to(DEV) for t in ref]
    torch.autograd.backward(got, ups)
    torch.autograd.backward(ref, ups)
    for a, b, name in zip(ins, ref_in, ("opacity", "scaling", "rotation")):
        ga, gb = a.grad.cpu().numpy(), b.grad.cpu().numpy()
        scale = np.abs(gb).max() + 1e-30
        assert np.abs(ga - gb).max() <= 1e-5 * scale, (name, np.abs(ga - gb).max(), scale)
        bad = np.abs(ga - gb) > 1e-4 * np.abs(gb) + 1e-6 * scale
        assert not bad.any(), (name, int(bad.sum()))


def test_activate_partial_gradients():
    """Only the opacity reaches the loss: the other two gradients stay None upstream and are skipped."""
    from hlgs_core.activations import activate
    op = torch.randn(500, 1, device=DEV, requires_grad=True)
    sc = torch.randn(500, 3, device=DEV, requires_grad=True)
    rot = torch.randn(500, 4, device=DEV, requires_grad=True)
    o, s, r = activate(op, sc, rot)
    o.sum().backward()
    y = torch.sigmoid(op.detach())
    np.testing.assert_allclose(op.grad.cpu().numpy(), (y * (1 - y)).cpu().numpy(), rtol=1e-6, atol=1e-12)
    assert sc.grad is None and rot.grad is None
