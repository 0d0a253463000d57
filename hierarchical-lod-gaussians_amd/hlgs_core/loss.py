"""Photometric losses of the training step on the HIP path (libhlgs.so, csrc/loss.hip).

  l1_loss(network_output, gt)                 utils/loss_utils.py:17-18
  ssim(img1, img2, window_size=11, size_average=True)   utils/loss_utils.py:32-63 (11x11 window only)
  fused_ssim(img1, img2, padding="same", train=True)    the un-vendored fused_ssim package (train_post.py:29, 559)
  photometric_loss(image, gt, lambda_dssim, ...)        the whole loss of train_single.py:106-121 in two kernels:
      (1 - lambda_dssim) * L1 + lambda_dssim * (1 - SSIM) [+ depth_weight * mean |(invdepth - mono) * mask|]

Gradients flow to the rendered image (and the rendered inverse depth), not to the ground truth, as in the
reference's training graph.  Every backward coefficient stays on the device (no host synchronisation).
"""
import ctypes as C

import torch

from hlgs_core import _lib as L


def _planes(t):
    """(..., H, W) float tensor -> (contiguous float32 tensor, planes, H, W)."""
    if t.dim() < 2:
        raise RuntimeError("expected an image tensor (..., H, W)")
    t = t.contiguous().float()
    H, W = t.shape[-2], t.shape[-1]
    return t, t.numel() // (H * W), H, W


def _ssim_forward(img1, img2, valid, train, clamp1=False):
    lib = L.load()
    x, Cn, H, W = _planes(img1)
    y, Cy, Hy, Wy = _planes(img2.detach())
    if (Cn, H, W) != (Cy, Hy, Wy):
        raise RuntimeError("img1 and img2 must have the same shape")
    L.require_gpu(x, y)
    out = torch.empty(2, dtype=torch.float32, device=x.device)
    maps = torch.empty((Cn, 3, H, W), dtype=torch.float32, device=x.device) if train else None
    scratch = torch.empty(lib.hlgs_ssim_scratch_size(Cn, H, W), dtype=torch.uint8, device=x.device)
    flags = (1 if valid else 0) | (2 if clamp1 else 0)  # HLGS_SSIM_VALID, HLGS_SSIM_CLAMP1
    L.check(lib.hlgs_ssim_forward_ex(Cn, H, W, L.ptr(x), L.ptr(y), flags, L.ptr(maps), L.ptr(scratch), L.ptr(out),
                                     L.stream()))
    return out, x, y, maps, (Cn, H, W)


def _ssim_backward(x, y, maps, shape, coef, clamp1=False):
    lib = L.load()
    Cn, H, W = shape
    grad = torch.empty_like(x)
    L.check(lib.hlgs_ssim_backward_ex(Cn, H, W, L.ptr(x), L.ptr(y), 2 if clamp1 else 0, L.ptr(maps),
                                      L.ptr(coef.contiguous()), L.ptr(grad), L.stream()))
    return grad


class _SSIM(torch.autograd.Function):
    """mean SSIM map (and mean |img1 - img2| as a by-product, non-differentiable here)."""

    @staticmethod
    def forward(ctx, img1, img2, valid, train):
        out, x, y, maps, shape = _ssim_forward(img1, img2, valid, train)
        ctx.save_for_backward(x, y, maps if maps is not None else torch.empty(0, device=x.device))
        ctx.shape, ctx.train, ctx.in_shape = shape, train, img1.shape
        Cn, H, W = shape
        ctx.n_map = Cn * (H - 10) * (W - 10) if valid else Cn * H * W
        return out[0]

    @staticmethod
    def backward(ctx, g):
        if not ctx.train:
            raise RuntimeError("fused_ssim was called with train=False: no gradient maps were kept")
        x, y, maps = ctx.saved_tensors
        coef = torch.stack([g.float() / ctx.n_map, torch.zeros_like(g, dtype=torch.float32)])
        grad = _ssim_backward(x, y, maps, ctx.shape, coef).reshape(ctx.in_shape)
        return grad, None, None, None


def fused_ssim(img1, img2, padding="same", train=True):
    """Mean SSIM of img1 against img2 ((B, C, H, W) or (C, H, W)); gradient w.r.t. img1 only."""
    assert padding in ["same", "valid"]
    return _SSIM.apply(img1, img2, padding == "valid", bool(train))


def ssim(img1, img2, window_size=11, size_average=True):
    """utils/loss_utils.ssim with the 11x11 window (the only size the reference uses)."""
    if window_size != 11:
        raise NotImplementedError("the HIP SSIM kernel implements the reference's 11x11 window")
    if not size_average:
        raise NotImplementedError("size_average=False (per-image SSIM) is not used by the training scripts")
    return fused_ssim(img1, img2, "same", torch.is_grad_enabled() and img1.requires_grad)


def l1_loss(network_output, gt):
    return torch.abs((network_output - gt)).mean()


class _Photometric(torch.autograd.Function):
    @staticmethod
    def forward(ctx, image, gt, invdepth, mono, mask, lambda_dssim, depth_weight, clamp_image):
        train = image.requires_grad or (invdepth is not None and invdepth.requires_grad)
        out, x, y, maps, shape = _ssim_forward(image, gt, False, train, clamp_image)
        ctx.clamp_image = clamp_image
        Ll1, ssim_v = out[1], out[0]
        loss = (1.0 - lambda_dssim) * Ll1 + lambda_dssim * (1.0 - ssim_v)
        Ld = torch.zeros((), dtype=torch.float32, device=x.device)
        dep = None
        if invdepth is not None and depth_weight > 0:
            lib = L.load()
            inv = invdepth.contiguous().float()
            mo = mono.contiguous().float()
            mk = mask.contiguous().float() if mask is not None else None
            n = inv.numel()
            if mo.numel() != n or (mk is not None and mk.numel() != n):
                raise RuntimeError("invdepth, mono_invdepth and depth_mask must have the same size")
            scratch = torch.empty(lib.hlgs_depth_l1_scratch_size(n), dtype=torch.uint8, device=x.device)
            o = torch.empty(1, dtype=torch.float32, device=x.device)
            L.check(lib.hlgs_depth_l1_forward(n, L.ptr(inv), L.ptr(mo), L.ptr(mk), L.ptr(scratch), L.ptr(o),
                                              L.stream()))
            Ld = o[0]
            loss = loss + depth_weight * Ld
            dep = (inv, mo, mk)
        ctx.save_for_backward(x, y, maps if maps is not None else torch.empty(0, device=x.device))
        ctx.dep = dep
        ctx.args = (shape, lambda_dssim, depth_weight, image.shape, None if invdepth is None else invdepth.shape)
        ctx.mark_non_differentiable(Ll1, ssim_v, Ld)
        return loss, Ll1, ssim_v, Ld

    @staticmethod
    def backward(ctx, g, _g1, _g2, _g3):
        x, y, maps = ctx.saved_tensors
        shape, lam, dw, ishape, dshape = ctx.args
        Cn, H, W = shape
        n = Cn * H * W
        g = g.float()
        coef = torch.stack([g * (-lam / n), g * ((1.0 - lam) / n)])
        d_img = _ssim_backward(x, y, maps, shape, coef, ctx.clamp_image).reshape(ishape)
        d_inv = None
        if ctx.dep is not None:
            lib = L.load()
            inv, mo, mk = ctx.dep
            d_inv = torch.empty_like(inv)
            c = (g * (dw / inv.numel())).reshape(1)
            L.check(lib.hlgs_depth_l1_backward(inv.numel(), L.ptr(inv), L.ptr(mo), L.ptr(mk), L.ptr(c), L.ptr(d_inv),
                                               L.stream()))
            d_inv = d_inv.reshape(dshape)
        return d_img, None, d_inv, None, None, None, None, None


def photometric_loss(image, gt, lambda_dssim, invdepth=None, mono_invdepth=None, depth_mask=None, depth_weight=0.0,
                     clamp_image=False):
    """-> (loss, Ll1, SSIM, Ll1depth_pure): the training loss of train_single.py:106-118 (and, without the depth
    term, train_post.py:558-559) with L1, SSIM and the depth L1 computed by two fused HIP passes; `loss` is
    differentiable w.r.t. image and invdepth.  clamp_image=True is photometric_loss(image.clamp(0, 1), ...) -- the
    renderers' rendered_image.clamp(0, 1) (gaussian_renderer/__init__.py:142, 612) -- folded into the same passes."""
    return _Photometric.apply(image, gt, invdepth, mono_invdepth, depth_mask, float(lambda_dssim), float(depth_weight),
                              bool(clamp_image))
