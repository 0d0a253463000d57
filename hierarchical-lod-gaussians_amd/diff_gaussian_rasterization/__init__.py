"""Drop-in `diff_gaussian_rasterization` for MI355X.

Public surface of submodules/hierarchy-rasterizer/diff_gaussian_rasterization/__init__.py:
`GaussianRasterizationSettings` (17 fields, same order, :145-162), `GaussianRasterizer` (:165-214),
`rasterize_gaussians` (:17-38) and `compute_relocation` (:216-218).  The autograd function keeps the
reference's contract -- forward returns (color (3,H,W), radii (P,), invdepth (1|0,H,W)); backward
returns gradients in input order -- and unpacks all eight values `_C.rasterize_gaussians` returns
(the reference unpacks seven).
"""
from typing import NamedTuple

import torch
import torch.nn as nn

from . import _C

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "compute_relocation", "_C"]


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
    render_indices: torch.Tensor
    parent_indices: torch.Tensor
    interpolation_weights: torch.Tensor
    num_node_kids: torch.Tensor
    do_depth: bool


def _hierarchy(rs):
    return rs.render_indices, rs.parent_indices, rs.interpolation_weights, rs.num_node_kids


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp, raster_settings):
        rs = raster_settings
        out = _C.rasterize_gaussians(rs.bg, *_hierarchy(rs), means3D, colors_precomp, opacities, scales, rotations,
                                     rs.scale_modifier, cov3Ds_precomp, rs.viewmatrix, rs.projmatrix, rs.tanfovx,
                                     rs.tanfovy, rs.image_height, rs.image_width, sh, rs.sh_degree, rs.campos,
                                     rs.prefiltered, rs.debug, rs.do_depth, need_seen=False)
        # `seen` is not part of the public return (color, radii, invdepth): the reference's wrapper never hands it on
        # (and cannot unpack it), so this path skips computing it
        num_rendered, color, radii, geom_buf, binning_buf, img_buf, invdepth, _seen = out
        ctx.raster_settings = rs
        ctx.num_rendered = num_rendered
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, opacities,
                              geom_buf, binning_buf, img_buf)
        ctx.mark_non_differentiable(radii)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for radii (or an unused output)
        return color, radii, invdepth

    @staticmethod
    def backward(ctx, grad_color, _grad_radii, grad_invdepth):
        rs = ctx.raster_settings
        (colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, opacities, geom_buf, binning_buf,
         img_buf) = ctx.saved_tensors
        if grad_color is None:  # only the inverse depth reached the loss
            grad_color = torch.zeros((3, rs.image_height, rs.image_width), dtype=torch.float32, device=means3D.device)
        d_means2D, d_colors, d_opac, d_means3D, d_cov3D, d_sh, d_scales, d_rots = _C.rasterize_gaussians_backward(
            rs.bg, *_hierarchy(rs), means3D, radii, colors_precomp, opacities, scales, rotations, rs.scale_modifier,
            cov3Ds_precomp, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, grad_color, grad_invdepth, sh,
            rs.sh_degree, rs.campos, geom_buf, ctx.num_rendered, binning_buf, img_buf, rs.debug,
            need_cov3D=cov3Ds_precomp.numel() > 0)
        # same order as the forward inputs; raster_settings gets None (and an empty cov3Ds_precomp no gradient: the
        # library then skips the 24 B per Gaussian of dL/dcov3D rows nothing would read)
        return (d_means3D, d_means2D, d_sh, d_colors, d_opac, d_scales, d_rots,
                d_cov3D if cov3Ds_precomp.numel() > 0 else None, None)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings)


def _empty_like_missing(t, ref):
    return t if t is not None else torch.empty(0, dtype=torch.float32, device=ref.device)


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        """Boolean frustum (z > 0.2) mask per position."""
        with torch.no_grad():
            rs = self.raster_settings
            return _C.mark_visible(positions, rs.viewmatrix, rs.projmatrix)

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        have_sh, have_col = shs is not None, colors_precomp is not None
        if have_sh == have_col:
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        have_sr = scales is not None or rotations is not None
        if (cov3D_precomp is None and (scales is None or rotations is None)) or (have_sr and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')
        fill = lambda t: _empty_like_missing(t, means3D)  # noqa: E731  (the reference passes torch.Tensor([]))
        return rasterize_gaussians(means3D, means2D, fill(shs), fill(colors_precomp), opacities, fill(scales),
                                   fill(rotations), fill(cov3D_precomp), self.raster_settings)


def compute_relocation(opacity_old, scale_old, N, binoms, n_max):
    return _C.compute_relocation(opacity_old, scale_old, N.int(), binoms, n_max)
