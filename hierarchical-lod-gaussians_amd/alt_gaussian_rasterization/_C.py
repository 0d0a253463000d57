"""`alt_gaussian_rasterization._C` on MI355X.

Same entry points, argument order and return tuples as the reference extension
(submodules/alt-rasterizer/ext.cpp:15-19: rasterize_gaussians, rasterize_gaussians_backward,
compute_relocation, mark_visible, adamUpdate; rasterize_points.cu:43-306).  The rasterizer runs in libhlgs.so
with variant = HLGS_VARIANT_ALT: SH split into dc + rest, optional antialiasing, eigen-radius tile rect with
exact per-tile culling, inverse depth always rendered, and the alt backward's gradient conventions.

`num_buckets` and `sampleBuffer` are the reference's per-32-splat backward state
(rasterizer_impl.cu:268-290); the MI355X backward replays tiles from the forward's per-pixel state instead
and needs none, so they are returned as 0 and an empty tensor (both are only handed back to backward).
"""
import ctypes as C

import torch

_vp = C.c_void_p

from hlgs_core import _lib as L
from hlgs_core import dp
from hlgs_core.dp import direct_grad


def _dev_f32(t, device):
    return t.to(device=device, dtype=torch.float32).contiguous()


def _dest(src, shape, f32, late=False):
    """Gradient output for input `src`: the view hlgs_core.dp.direct_grad offers (a view-DP exchange's flat buffer)
    when its shape matches, else a fresh tensor.  Every kernel output row is written, so no zero-fill either way.
    late: the output is completed by the SH backward (dmean3D, dsh, ddc)."""
    d = direct_grad(src, late) if src is not None else None
    return d if d is not None and tuple(d.shape) == tuple(shape) else torch.empty(shape, **f32)


def _opt(t):
    """Empty tensor -> None (NULL, as data_ptr() of an empty tensor is nullptr in the reference)."""
    if t is None or t.numel() == 0:
        return None
    return t.contiguous()


def _raster_args(bg, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
                 projmatrix, tan_fovx, tan_fovy, H, W, dc, sh, degree, campos, prefiltered, antialiasing, debug):
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    dev = means3D.device
    keep = dict(bg=_dev_f32(bg, dev), means3D=means3D.contiguous(), colors=_opt(colors), opacity=_opt(opacity),
                scales=_opt(scales), rotations=_opt(rotations), cov3D=_opt(cov3D_precomp),
                view=_dev_f32(viewmatrix, dev), proj=_dev_f32(projmatrix, dev), campos=_dev_f32(campos, dev),
                dc=_opt(dc), sh=_opt(sh))
    L.require_gpu(*[v for v in keep.values() if isinstance(v, torch.Tensor)])
    P = means3D.size(0)
    # rasterize_points.cu:97-101: M = sh.size(1) when sh is non-empty (the higher-order coefficients)
    M = sh.size(1) if (sh is not None and sh.size(0) != 0 and sh.dim() > 1) else 0
    a = L.RasterArgs(P=P, P_full=P, D=int(degree), M=M, W=int(W), H=int(H), bg=L.ptr(keep["bg"]),
                     means3D=L.ptr(keep["means3D"]), shs=L.ptr(keep["sh"]), colors_precomp=L.ptr(keep["colors"]),
                     opacities=L.ptr(keep["opacity"]), scales=L.ptr(keep["scales"]),
                     rotations=L.ptr(keep["rotations"]), cov3D_precomp=L.ptr(keep["cov3D"]),
                     viewmatrix=L.ptr(keep["view"]), projmatrix=L.ptr(keep["proj"]), campos=L.ptr(keep["campos"]),
                     scale_modifier=float(scale_modifier), tanfovx=float(tan_fovx), tanfovy=float(tan_fovy),
                     indices=None, parent_indices=None, ts=None, kids=None, prefiltered=int(bool(prefiltered)),
                     debug=int(bool(debug)), dc=L.ptr(keep["dc"]), antialiasing=int(bool(antialiasing)),
                     variant=L.VARIANT_ALT)
    return a, keep, P, M


_binning_hint = {}


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                        viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, dc, sh, degree, campos,
                        prefiltered, antialiasing, debug):
    """-> (num_rendered, num_buckets, color (3,H,W), invdepth (1,H,W), radii (P,), geomBuffer, binningBuffer,
    imgBuffer, sampleBuffer)  (rasterize_points.cu:43-136)."""
    lib = L.load()
    H, W = int(image_height), int(image_width)
    dev = means3D.device
    f32 = dict(dtype=torch.float32, device=dev)
    u8 = dict(dtype=torch.uint8, device=dev)
    P = means3D.size(0)
    if P == 0:  # rasterize_points.cu:88-90, 99: nothing is launched, the outputs stay 0
        return (0, 0, torch.zeros((3, H, W), **f32), torch.zeros((1, H, W), **f32),
                torch.zeros((0,), dtype=torch.int32, device=dev), torch.empty((0,), **u8), torch.empty((0,), **u8),
                torch.empty((0,), **u8), torch.empty((0,), **u8))
    a, keep, P, _ = _raster_args(background, means3D, colors, opacity, scales, rotations, scale_modifier,
                                 cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, H, W, dc, sh, degree,
                                 campos, prefiltered, antialiasing, debug)
    color = torch.empty((3, H, W), **f32)
    invdepth = torch.empty((1, H, W), **f32)
    radii = torch.empty((P,), dtype=torch.int32, device=dev)
    geom = torch.empty((lib.hlgs_geom_buffer_size(P),), **u8)
    img = torch.empty((lib.hlgs_image_buffer_size(W, H),), **u8)
    info = L.FrameInfo()
    binning = torch.empty((_binning_hint.get(dev, 0),), **u8)
    s = L.stream()
    L.check(lib.hlgs_rasterize_forward(C.byref(a), L.ptr(geom), L.ptr(img), L.ptr(radii), L.ptr(binning),
                                       binning.numel(), C.byref(info), L.ptr(color), L.ptr(invdepth), None, s))
    if not info.rendered:
        need = lib.hlgs_binning_buffer_size(info.num_binned)
        binning = torch.empty((need,), **u8)
        L.check(lib.hlgs_rasterize_forward_render(C.byref(a), L.ptr(radii), L.ptr(geom), L.ptr(img), L.ptr(binning),
                                                  C.byref(info), L.ptr(color), L.ptr(invdepth), None, s))
        _binning_hint[dev] = int(need * 1.15)
    del keep
    return (int(info.num_rendered), 0, color, invdepth, radii, geom, binning, img, torch.empty((0,), **u8))


def rasterize_gaussians_backward(background, means3D, radii, colors, opacities, scales, rotations, scale_modifier,
                                 cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, dc, sh,
                                 dL_dout_invdepth, degree, campos, geomBuffer, R, binningBuffer, imageBuffer, B,
                                 sampleBuffer, antialiasing, debug, *, need_cov3D=True):
    """-> (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_ddc, dL_dsh, dL_dscales,
    dL_drotations)  (rasterize_points.cu:138-232).  need_cov3D=False (the autograd wrapper without cov3D_precomp)
    returns an empty dL_dcov3D and skips writing its rows."""
    lib = L.load()
    H, W = int(dL_dout_color.size(1)), int(dL_dout_color.size(2))
    dev = means3D.device
    f32 = dict(dtype=torch.float32, device=dev)
    P = means3D.size(0)
    M = sh.size(1) if (sh is not None and sh.size(0) != 0 and sh.dim() > 1) else 0
    # a colour-factored view-DP exchange takes dL/dRGB instead of the dc / SH gradients (hlgs_core.dp.colour_factor);
    # not with an empty sh, whose SH backward does not run at all (A-19)
    fac = dp.colour_factor(sh, dc) if M > 0 and dc is not None and dc.numel() else None
    out = dict(dmean2D=torch.empty((P, 3), **f32), dcolor=torch.empty((P, 3), **f32),
               dopacity=_dest(opacities, (P, 1), f32), dmean3D=_dest(means3D, (P, 3), f32, True),
               dcov3D=torch.empty((P if need_cov3D else 0, 6), **f32),
               ddc=fac[2] if fac is not None else _dest(dc, (P, 1, 3), f32, True),
               dsh=fac[1] if fac is not None else _dest(sh, (P, M, 3), f32, True), dscale=_dest(scales, (P, 3), f32),
               drot=_dest(rotations, (P, 4), f32))
    order = ("dmean2D", "dcolor", "dopacity", "dmean3D", "dcov3D", "ddc", "dsh", "dscale", "drot")
    if P == 0:
        return tuple(out[k] for k in order)
    a, keep, P, M = _raster_args(background, means3D, colors, opacities, scales, rotations, scale_modifier,
                                 cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, H, W, dc, sh, degree,
                                 campos, False, antialiasing, debug)
    g = L.Grads(**{k: L.ptr(v) for k, v in out.items()}, drgb=L.ptr(fac[0]) if fac is not None else None)
    dpix = dL_dout_color.contiguous().float()
    dinv = dL_dout_invdepth.contiguous().float() if dL_dout_invdepth is not None and dL_dout_invdepth.numel() else None
    scratch = torch.empty((lib.hlgs_backward_scratch_size(P, int(R)),), dtype=torch.uint8, device=dev)
    # the SH backward on an overlapping exchange's late stream (hlgs_core.dp.late_stream_for), else in order
    late = dp.late_stream_for(out["dmean3D"], out["ddc"], out["dsh"])
    L.check(lib.hlgs_rasterize_backward_split(C.byref(a), L.ptr(radii.contiguous()), L.ptr(geomBuffer),
                                              L.ptr(imageBuffer), L.ptr(binningBuffer), int(R), L.ptr(scratch),
                                              L.ptr(dpix), L.ptr(dinv), C.byref(g), L.stream(),
                                              _vp(late.cuda_stream) if late is not None else None))
    if late is not None:
        dp.note_late_work(late, list(keep.values()) + list(out.values()) +
                          [radii, geomBuffer, imageBuffer, binningBuffer, scratch, dpix, dinv])
    if fac is not None:
        fac[3](keep["campos"], degree, L.VARIANT_ALT)
    del keep
    return tuple(out[k] for k in order)


def mark_visible(means3D, viewmatrix, projmatrix):
    """Frustum (z > 0.2) test per point (rasterizer_impl.cu:104-116, 235-247; rasterize_points.cu:234-253) -> bool tensor."""
    from diff_gaussian_rasterization import _C as HC
    return HC.mark_visible(means3D, viewmatrix, projmatrix)


def compute_relocation(opacity_old, scale_old, N, binoms, n_max):
    """MCMC relocation (rasterize_points.cu:284-306) -> (opacity (P,), scale (3P,))."""
    from diff_gaussian_rasterization import _C as HC
    return HC.compute_relocation(opacity_old, scale_old, N, binoms, n_max)


def adamUpdate(param, param_grad, exp_avg, exp_avg_sq, visible, lr, b1, b2, eps, N, M):
    """In-place sparse Adam step (rasterize_points.cu:255-281, adam.cu:9-36): element p of the N x M parameter
    is updated iff visible[p // M]."""
    lib = L.load()
    for t in (param, param_grad, exp_avg, exp_avg_sq):
        if not t.is_contiguous() or t.dtype != torch.float32:
            raise RuntimeError("adamUpdate expects contiguous float32 tensors (updated in place)")
    vis = visible.contiguous()
    if vis.dtype != torch.bool:
        vis = vis.to(torch.bool)
    L.require_gpu(param, param_grad, exp_avg, exp_avg_sq, vis)
    if int(N) * int(M) > param.numel():
        raise RuntimeError("adamUpdate: N * M exceeds the parameter size")
    L.check(lib.hlgs_adam_update(L.ptr(param), L.ptr(param_grad), L.ptr(exp_avg), L.ptr(exp_avg_sq), L.ptr(vis),
                                 float(lr), float(b1), float(b2), float(eps), int(N), int(M), L.stream()))
