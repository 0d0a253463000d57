"""Drop-in `alt_gaussian_rasterization` for MI355X.

Public surface of submodules/alt-rasterizer/alt_gaussian_rasterization/__init__.py: `rasterize_gaussians`
(:21-44), the autograd function (:46-157), `GaussianRasterizationSettings` (13 fields, same order,
:159-172), `GaussianRasterizer` (:174-242) and `SparseGaussianAdam` (:244-271).  The rasterizer is the
default one of train_post.py (:102, 510-523) and train_coarse.py (:103).  Forward returns
(color (3,H,W), radii (P,), invdepth (1,H,W)); backward returns the gradients in input order.
"""
from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "SparseGaussianAdam", "_C"]


def cpu_deep_copy_tuple(input_tuple):
    return tuple(item.cpu().clone() if isinstance(item, torch.Tensor) else item for item in input_tuple)


def rasterize_gaussians(means3D, means2D, dc, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, dc, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings)


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, dc, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings):
        rs = raster_settings
        args = (rs.bg, means3D, colors_precomp, opacities, scales, rotations, rs.scale_modifier, cov3Ds_precomp,
                rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width, dc, sh,
                rs.sh_degree, rs.campos, rs.prefiltered, rs.antialiasing, rs.debug)
        if rs.debug:  # __init__.py:87-95: keep a CPU snapshot of the arguments for post-mortem debugging
            cpu_args = cpu_deep_copy_tuple(args)
            try:
                out = _C.rasterize_gaussians(*args)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_fw.dump")
                print("\nAn error occured in forward. Please forward snapshot_fw.dump for debugging.")
                raise ex
        else:
            out = _C.rasterize_gaussians(*args)
        num_rendered, num_buckets, color, invdepths, radii, geom_buf, binning_buf, img_buf, sample_buf = out
        ctx.raster_settings = rs
        ctx.num_rendered = num_rendered
        ctx.num_buckets = num_buckets
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, dc, sh, opacities,
                              geom_buf, binning_buf, img_buf, sample_buf)
        return color, radii, invdepths

    @staticmethod
    def backward(ctx, grad_out_color, _, grad_out_depth):
        rs = ctx.raster_settings
        (colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, dc, sh, opacities, geom_buf, binning_buf,
         img_buf, sample_buf) = ctx.saved_tensors
        args = (rs.bg, means3D, radii, colors_precomp, opacities, scales, rotations, rs.scale_modifier,
                cov3Ds_precomp, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, grad_out_color, dc, sh,
                grad_out_depth, rs.sh_degree, rs.campos, geom_buf, ctx.num_rendered, binning_buf, img_buf,
                ctx.num_buckets, sample_buf, rs.antialiasing, rs.debug)
        need_cov3D = cov3Ds_precomp.numel() > 0  # otherwise no gradient for it, and its rows are not written
        if rs.debug:
            cpu_args = cpu_deep_copy_tuple(args)
            try:
                grads = _C.rasterize_gaussians_backward(*args, need_cov3D=need_cov3D)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_bw.dump")
                print("\nAn error occured in backward. Writing snapshot_bw.dump for debugging.\n")
                raise ex
        else:
            grads = _C.rasterize_gaussians_backward(*args, need_cov3D=need_cov3D)
        (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_dc, grad_sh,
         grad_scales, grad_rotations) = grads
        return (grad_means3D, grad_means2D, grad_dc, grad_sh, grad_colors_precomp, grad_opacities, grad_scales,
                grad_rotations, grad_cov3Ds_precomp if need_cov3D else None, None)


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool
    antialiasing: bool


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        """Boolean frustum (z > 0.2) mask per position."""
        with torch.no_grad():
            rs = self.raster_settings
            return _C.mark_visible(positions, rs.viewmatrix, rs.projmatrix)

    def forward(self, means3D, means2D, opacities, dc=None, shs=None, colors_precomp=None, scales=None,
                rotations=None, cov3D_precomp=None):
        rs = self.raster_settings
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')
        empty = lambda t: t if t is not None else torch.empty(0, dtype=torch.float32, device=means3D.device)  # noqa: E731
        return rasterize_gaussians(means3D, means2D, empty(dc), empty(shs), empty(colors_precomp), opacities,
                                   empty(scales), empty(rotations), empty(cov3D_precomp), rs)


class SparseGaussianAdam(torch.optim.Adam):
    """Adam that updates only the rows of visible Gaussians (__init__.py:244-271): one parameter tensor per
    group, N Gaussians, M = numel / N values per Gaussian; no bias correction (adam.cu:9-36)."""

    def __init__(self, params, lr, eps):
        super().__init__(params=params, lr=lr, eps=eps)

    @torch.no_grad()
    def step(self, visibility, N):
        for group in self.param_groups:
            lr = group["lr"]
            eps = group["eps"]
            assert len(group["params"]) == 1, "more than one tensor in group"
            param = group["params"][0]
            if param.grad is None:
                continue
            state = self.state[param]
            if len(state) == 0:
                state['step'] = torch.tensor(0.0, dtype=torch.float32)
                state['exp_avg'] = torch.zeros_like(param, memory_format=torch.preserve_format)
                state['exp_avg_sq'] = torch.zeros_like(param, memory_format=torch.preserve_format)
            exp_avg = state["exp_avg"]
            exp_avg_sq = state["exp_avg_sq"]
            M = param.numel() // N
            _C.adamUpdate(param, param.grad, exp_avg, exp_avg_sq, visibility, lr, 0.9, 0.999, eps, N, M)
