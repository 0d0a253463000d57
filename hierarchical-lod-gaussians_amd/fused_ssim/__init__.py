"""Drop-in for the `fused_ssim` package train_post.py imports (train_post.py:29, 559; hierarchy_viewer.py:29) but the
reference does not vendor: fused_ssim(img1, img2, padding="same", train=True) -> mean SSIM (11x11 Gaussian window,
sigma 1.5, C1 = 0.01^2, C2 = 0.03^2), differentiable w.r.t. img1, computed by the HIP kernels of
hlgs_core.loss (csrc/loss.hip)."""
from hlgs_core.loss import fused_ssim

__all__ = ["fused_ssim"]
