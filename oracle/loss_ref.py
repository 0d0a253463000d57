"""CPU restatement of the training-step losses (float64 torch on the CPU).

TEST INFRASTRUCTURE ONLY (tests/ import it as the checker of csrc/loss.hip; the product path never does).
Restates utils/loss_utils.py:17-63 (l1_loss, gaussian/create_window, _ssim with zero padding 5), the fused_ssim
padding="valid" crop (map[..., 5:-5, 5:-5]) and the depth term of train_single.py:111-118.  Pinned against
tests/golden/golden_loss.npz, which the reference's own loss_utils produced (tests/golden/make_golden.py).
"""
import math

import torch
import torch.nn.functional as F


def window(dtype=torch.float64):
    g = torch.tensor([math.exp(-(x - 5) ** 2 / float(2 * 1.5 ** 2)) for x in range(11)], dtype=torch.float32)
    g = (g / g.sum()).to(dtype)
    return (g[:, None] @ g[None, :])[None, None]


def ssim_map(img1, img2):
    """(C, H, W) or (B, C, H, W) -> SSIM map of the same shape (loss_utils.py:44-63)."""
    x, y = img1.double(), img2.double()
    squeeze = x.dim() == 3
    if squeeze:
        x, y = x[None], y[None]
    C = x.shape[1]
    w = window().expand(C, 1, 11, 11).contiguous()
    conv = lambda t: F.conv2d(t, w, padding=5, groups=C)  # noqa: E731
    mu1, mu2 = conv(x), conv(y)
    s11 = conv(x * x) - mu1 ** 2
    s22 = conv(y * y) - mu2 ** 2
    s12 = conv(x * y) - mu1 * mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    m = ((2 * mu1 * mu2 + C1) * (2 * s12 + C2)) / ((mu1 ** 2 + mu2 ** 2 + C1) * (s11 + s22 + C2))
    return m[0] if squeeze else m


def ssim(img1, img2, valid=False):
    m = ssim_map(img1, img2)
    return m[..., 5:-5, 5:-5].mean() if valid else m.mean()


def photometric(image, gt, lam, inv=None, mono=None, mask=None, dw=0.0):
    loss = (1.0 - lam) * torch.abs(image.double() - gt.double()).mean() + lam * (1.0 - ssim(image, gt))
    if inv is not None and dw > 0:
        m = mask.double() if mask is not None else 1.0
        loss = loss + dw * torch.abs((inv.double() - mono.double()) * m).mean()
    return loss
