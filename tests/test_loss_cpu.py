"""Pin the loss restatement (oracle/loss_ref.py) to the reference's own utils/loss_utils outputs
(tests/golden/golden_loss.npz) before it checks the HIP loss kernels (tests/test_gpu_loss.py)."""
import os

import numpy as np
import pytest
import torch

from oracle import loss_ref as LR

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_loss.npz")


@pytest.mark.parametrize("i", [0, 1, 2])
def test_loss_restatement_matches_reference_loss_utils(i):
    z = np.load(GOLD)
    g = lambda k: torch.tensor(z[f"{k}_{i}"])  # noqa: E731
    img = g("img").double().requires_grad_(True)
    s = LR.ssim(img, g("gt"))
    assert abs(float(s.detach()) - float(z[f"ssim_{i}"])) < 2e-6
    (gs,) = torch.autograd.grad(s, img)
    np.testing.assert_allclose(gs.numpy(), z[f"g_ssim_{i}"], rtol=1e-3, atol=1e-9)
    img = g("img").double().requires_grad_(True)
    inv = g("inv").double().requires_grad_(True)
    tot = LR.photometric(img, g("gt"), float(z[f"lam_{i}"]), inv, g("mono"), g("mask"), float(z[f"dw_{i}"]))
    assert abs(float(tot.detach()) - float(z[f"loss_{i}"])) < 2e-6
    gi, gv = torch.autograd.grad(tot, (img, inv))
    np.testing.assert_allclose(gi.numpy(), z[f"g_img_{i}"], rtol=1e-3, atol=1e-9)
    np.testing.assert_allclose(gv.numpy(), z[f"g_inv_{i}"], rtol=1e-5, atol=1e-12)


def test_loss_api_signatures():
    import inspect

    import fused_ssim
    from hlgs_core import loss
    sig = lambda f: list(inspect.signature(f).parameters)  # noqa: E731
    assert sig(fused_ssim.fused_ssim) == ["img1", "img2", "padding", "train"]
    assert sig(loss.ssim) == ["img1", "img2", "window_size", "size_average"]
    assert sig(loss.l1_loss) == ["network_output", "gt"]
