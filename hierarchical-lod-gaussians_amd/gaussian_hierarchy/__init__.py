"""Drop-in `gaussian_hierarchy` for MI355X: every function of `gaussian_hierarchy._C`
(submodules/gaussianhierarchy/ext.cpp:15-27: file I/O, traversal, runtime LOD cuts, Morton codes) plus
`interpolate_lod`, a HIP replacement for the
child/parent lerp `render_post` performs in Python (gaussian_renderer/__init__.py:304-339).
"""
import torch

from . import _C
from ._C import (expand_to_size, expand_to_size_dynamic, expand_to_target, get_interpolation_weights,  # noqa: F401
                 get_interpolation_weights_dynamic, get_morton_indices, get_spt_cut_cuda, load_dynamic_hierarchy,
                 load_hierarchy, write_dynamic_hierarchy, write_hierarchy)

__all__ = ["_C", "expand_to_size", "expand_to_size_dynamic", "expand_to_target", "get_interpolation_weights",
           "get_interpolation_weights_dynamic", "get_morton_indices", "get_spt_cut_cuda", "interpolate_lod",
           "load_dynamic_hierarchy", "load_hierarchy", "write_dynamic_hierarchy", "write_hierarchy"]


class _InterpolateLOD(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, scales, rotations, opacity, shs, render_indices, parent_indices, weights, skybox_points):
        ridx = render_indices.contiguous().to(torch.int32)
        pidx = parent_indices.contiguous().to(torch.int32)
        w = weights.contiguous().float()
        rots = rotations.contiguous().float()
        has_sh = shs is not None and shs.numel() > 0
        outs = _C.lod_interp_forward(int(skybox_points), ridx, pidx, w, means3D.contiguous().float(),
                                     scales.contiguous().float(), rots, opacity.contiguous().float(),
                                     shs.contiguous().float() if has_sh else None)
        ctx.save_for_backward(ridx, pidx, w, rots)
        ctx.S = int(skybox_points)
        ctx.P = means3D.size(0)
        ctx.sh_shape = tuple(shs.shape) if has_sh else None
        m, s, r, o, sh = outs
        return m, s, r, o, (sh if has_sh else torch.empty(0, device=means3D.device))

    @staticmethod
    def backward(ctx, g_m, g_s, g_r, g_o, g_sh):
        ridx, pidx, w, rots = ctx.saved_tensors
        c = lambda t: t.contiguous().float()  # noqa: E731
        d = _C.lod_interp_backward(ctx.S, ridx, pidx, w, rots, ctx.P, c(g_m), c(g_s), c(g_r), c(g_o),
                                   c(g_sh) if ctx.sh_shape is not None else None, ctx.sh_shape)
        d_m, d_s, d_r, d_o, d_sh = d
        return d_m, d_s, d_r, d_o, d_sh, None, None, None, None


def interpolate_lod(means3D, scales, rotations, opacity, shs, render_indices, parent_indices, interpolation_weights,
                    skybox_points=0):
    """Lerp every selected node with its parent (activated parameters; rotations sign-aligned, not
    renormalised), prepend the first `skybox_points` rows unchanged.  Returns (means3D, scales, rotations,
    opacity, shs) of S + n rows, differentiable w.r.t. every input row, exactly as autograd of
    gaussian_renderer/__init__.py:304-339 would be."""
    n = render_indices.size(0)
    return _InterpolateLOD.apply(means3D, scales, rotations, opacity, shs, render_indices, parent_indices[:n],
                                 interpolation_weights[:n], skybox_points)
