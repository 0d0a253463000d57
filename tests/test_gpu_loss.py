"""HIP loss kernels (csrc/loss.hip through hlgs_core.loss / fused_ssim) against the reference's own loss_utils
outputs (tests/golden/golden_loss.npz) and, at training size, against the float64 restatement
oracle/loss_ref.py.  Losses within 1e-5 relative, gradients within 1e-4 of the gradient's max magnitude."""
import os

import numpy as np
import pytest
import torch

from oracle import loss_ref as LR

pytestmark = pytest.mark.gpu
DEV = "cuda"
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_loss.npz")


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.mark.parametrize("i", [0, 1, 2])
def test_losses_match_reference_golden(i):
    from hlgs_core import loss
    z = np.load(GOLD)
    g = lambda k: torch.tensor(z[f"{k}_{i}"], device=DEV)  # noqa: E731
    img = g("img").requires_grad_(True)
    s = loss.ssim(img, g("gt"))
    s.backward()
    assert abs(float(s.detach()) - float(z[f"ssim_{i}"])) <= 1e-5 * abs(float(z[f"ssim_{i}"]))
    assert _rel(img.grad.cpu().numpy(), z[f"g_ssim_{i}"]) <= 1e-4
    img = g("img").requires_grad_(True)
    inv = g("inv").requires_grad_(True)
    tot, Ll1, Ls, Ld = loss.photometric_loss(img, g("gt"), float(z[f"lam_{i}"]), inv, g("mono"), g("mask"),
                                             float(z[f"dw_{i}"]))
    tot.backward()
    assert abs(float(tot.detach()) - float(z[f"loss_{i}"])) <= 1e-5 * abs(float(z[f"loss_{i}"]))
    assert abs(float(Ll1.detach()) - float(z[f"l1_{i}"])) <= 1e-5 * abs(float(z[f"l1_{i}"]))
    assert abs(float(Ld.detach()) - float(z[f"depth_l1_{i}"])) <= 1e-5 * abs(float(z[f"depth_l1_{i}"]))
    assert _rel(img.grad.cpu().numpy(), z[f"g_img_{i}"]) <= 1e-4
    assert _rel(inv.grad.cpu().numpy(), z[f"g_inv_{i}"]) <= 1e-6


@pytest.mark.parametrize("shape,padding", [((1, 3, 1080, 1920), "same"), ((1, 3, 1080, 1920), "valid"),
                                           ((2, 3, 77, 131), "same"), ((3, 45, 29), "valid"),
                                           ((1, 2, 7, 9), "same"), ((1, 1, 33, 233), "valid")])
def test_fused_ssim_matches_restatement(shape, padding):
    from fused_ssim import fused_ssim
    rng = np.random.default_rng(sum(shape))
    a = rng.uniform(0, 1, shape).astype(np.float32)
    b = np.clip(a + rng.normal(0, 0.1, shape), 0, 1).astype(np.float32)
    x = torch.tensor(a, device=DEV, requires_grad=True)
    s = fused_ssim(x, torch.tensor(b, device=DEV), padding=padding)
    s.backward()
    xr = torch.tensor(a, dtype=torch.float64, requires_grad=True)
    sr = LR.ssim(xr, torch.tensor(b), valid=padding == "valid")
    sr.backward()
    assert abs(float(s) - float(sr)) <= 1e-5 * abs(float(sr))
    assert _rel(x.grad.cpu().numpy(), xr.grad.numpy()) <= 1e-4


def test_fused_ssim_is_deterministic_and_train_false_has_no_grad():
    from fused_ssim import fused_ssim
    a = torch.rand(1, 3, 300, 200, device=DEV)
    b = torch.rand(1, 3, 300, 200, device=DEV)
    vals, grads = [], []
    for _ in range(2):
        x = a.clone().requires_grad_(True)
        s = fused_ssim(x, b)
        s.backward()
        vals.append(float(s))
        grads.append(x.grad.cpu().numpy())
    assert vals[0] == vals[1]
    np.testing.assert_array_equal(grads[0], grads[1])
    x = a.clone().requires_grad_(True)
    s = fused_ssim(x, b, train=False)
    assert abs(float(s) - vals[0]) <= 1e-6
    with pytest.raises(RuntimeError, match="train=False"):
        s.backward()


@pytest.mark.parametrize("depth", [False, True])
def test_photometric_clamp_image_equals_clamp_then_loss(depth):
    """photometric_loss(img, ..., clamp_image=True) is photometric_loss(img.clamp(0, 1), ...) bit for bit -- the loss
    and the gradient reaching img, including pixels outside [0, 1] (gradient 0 there, torch's clamp backward)."""
    from hlgs_core.loss import photometric_loss
    g = torch.Generator().manual_seed(7)
    img = (torch.rand(3, 70, 90, generator=g) * 1.6 - 0.3).to("cuda")  # ~35% of the values outside [0, 1]
    gt = torch.rand(3, 70, 90, generator=g).to("cuda")
    inv = torch.rand(1, 70, 90, generator=g).to("cuda").requires_grad_(True) if depth else None
    mono = torch.rand(1, 70, 90, generator=g).to("cuda") if depth else None
    a = img.clone().requires_grad_(True)
    b = img.clone().requires_grad_(True)
    kw = dict(invdepth=inv, mono_invdepth=mono, depth_weight=0.5) if depth else {}
    la = photometric_loss(a, gt, 0.2, clamp_image=True, **kw)[0]
    lb = photometric_loss(b.clamp(0, 1), gt, 0.2, **kw)[0]
    assert float(la) == float(lb)
    la.backward()
    lb.backward()
    assert torch.equal(a.grad, b.grad)
    assert (a.grad[(img < 0) | (img > 1)] == 0).all()
