"""`diff_gaussian_rasterization._C` on MI355X.

Same entry points, argument order and return tuples as the reference extension
(submodules/hierarchy-rasterizer/ext.cpp:15-19, rasterize_points.cu:36-271), plus `mark_visible`, which
the reference's Python wrapper calls (__init__.py:174) but never binds.  Tensors are
allocated with torch on the current device; every kernel runs inside libhlgs.so (gfx950) on torch's
current stream.
"""
import ctypes as C

import torch

_vp = C.c_void_p

from hlgs_core import _lib as L
from hlgs_core import dp
from hlgs_core.dp import direct_grad


def _dev_f32(t, device):
    """Small per-call tensors (bg, view/proj matrices, campos) must live on the device: the kernels
    dereference them (rasterize_points.cu:109-125)."""
    return t.to(device=device, dtype=torch.float32).contiguous()


def _dest(src, shape, f32, late=False):
    """Gradient output for input `src`: the view hlgs_core.dp.direct_grad offers (a view-DP exchange's flat buffer)
    when its shape matches, else a fresh tensor.  Every kernel output row is written, so no zero-fill either way.
    late: the output is completed by the SH backward (dmean3D, dsh, ddc)."""
    d = direct_grad(src, late) if src is not None else None
    return d if d is not None and tuple(d.shape) == tuple(shape) else torch.empty(shape, **f32)


def _opt(t, dtype=None):
    """Empty tensor -> None (NULL); otherwise a contiguous view (rasterize_points.cu calls .contiguous())."""
    if t is None or t.numel() == 0:
        return None
    t = t.contiguous()
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    return t


def _raster_args(bg, render_indices, parent_indices, ts, kids, means3D, colors, opacity, scales, rotations,
                 scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, H, W, sh, degree,
                 campos, prefiltered, debug):
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    dev = means3D.device
    keep = dict(
        bg=_dev_f32(bg, dev), means3D=means3D.contiguous(), colors=_opt(colors), opacity=_opt(opacity),
        scales=_opt(scales), rotations=_opt(rotations), cov3D=_opt(cov3D_precomp),
        view=_dev_f32(viewmatrix, dev), proj=_dev_f32(projmatrix, dev), campos=_dev_f32(campos, dev),
        sh=_opt(sh), indices=_opt(render_indices, torch.int32), parents=_opt(parent_indices, torch.int32),
        ts=_opt(ts, torch.float32), kids=_opt(kids, torch.int32))
    L.require_gpu(*[v for v in keep.values() if isinstance(v, torch.Tensor)])
    P_full = means3D.size(0)
    P = keep["indices"].size(0) if keep["indices"] is not None else P_full
    M = sh.size(1) if (sh is not None and sh.numel() and sh.size(0) != 0) else 0
    a = L.RasterArgs(P=P, P_full=P_full, D=int(degree), M=M, W=int(W), H=int(H),
                     bg=L.ptr(keep["bg"]), means3D=L.ptr(keep["means3D"]), shs=L.ptr(keep["sh"]),
                     colors_precomp=L.ptr(keep["colors"]), opacities=L.ptr(keep["opacity"]),
                     scales=L.ptr(keep["scales"]), rotations=L.ptr(keep["rotations"]),
                     cov3D_precomp=L.ptr(keep["cov3D"]), viewmatrix=L.ptr(keep["view"]),
                     projmatrix=L.ptr(keep["proj"]), campos=L.ptr(keep["campos"]),
                     scale_modifier=float(scale_modifier), tanfovx=float(tan_fovx), tanfovy=float(tan_fovy),
                     indices=L.ptr(keep["indices"]), parent_indices=L.ptr(keep["parents"]), ts=L.ptr(keep["ts"]),
                     kids=L.ptr(keep["kids"]), prefiltered=int(bool(prefiltered)), debug=int(bool(debug)),
                     dc=None, antialiasing=1, variant=L.VARIANT_HIERARCHY)
    return a, keep, P, P_full, M


_binning_hint = {}


def rasterize_gaussians(bg, render_indices, parent_indices, ts, kids, means3D, colors, opacity, scales, rotations,
                        scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height,
                        image_width, sh, degree, campos, prefiltered, debug, do_depth, *, need_seen=True):
    """-> (num_rendered, color, radii, geomBuffer, binningBuffer, imgBuffer, invdepth, seen)
    (rasterize_points.cu:36-139).  need_seen=False (used by the autograd wrapper, which drops it) returns an empty
    `seen` and skips its per-splat stores."""
    lib = L.load()
    H, W = int(image_height), int(image_width)
    a, keep, P, _, _ = _raster_args(bg, render_indices, parent_indices, ts, kids, means3D, colors, opacity, scales,
                                    rotations, scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tan_fovx,
                                    tan_fovy, H, W, sh, degree, campos, prefiltered, debug)
    dev = means3D.device
    f32 = dict(dtype=torch.float32, device=dev)
    color = torch.empty((3, H, W), **f32)
    invdepth = torch.empty((1 if do_depth else 0, H, W), **f32)
    radii = torch.empty((P,), dtype=torch.int32, device=dev)
    seen = torch.empty((P if need_seen else 0,), dtype=torch.int32, device=dev)
    u8 = dict(dtype=torch.uint8, device=dev)
    geom = torch.empty((lib.hlgs_geom_buffer_size(P),), **u8)
    img = torch.empty((lib.hlgs_image_buffer_size(W, H),), **u8)
    info = L.FrameInfo()
    # The binning buffer is sized from the largest frame seen on this device (+15%), so prepare and render
    # run in one library call; a frame that outgrows it gets an exact buffer and a second call.
    binning = torch.empty((_binning_hint.get(dev, 0),), **u8)
    s = L.stream()
    L.check(lib.hlgs_rasterize_forward(C.byref(a), L.ptr(geom), L.ptr(img), L.ptr(radii), L.ptr(binning),
                                       binning.numel(), C.byref(info), L.ptr(color),
                                       L.ptr(invdepth) if do_depth else None, L.ptr(seen) if need_seen else None,
                                       s))
    if not info.rendered:
        need = lib.hlgs_binning_buffer_size(info.num_binned)
        binning = torch.empty((need,), **u8)
        L.check(lib.hlgs_rasterize_forward_render(C.byref(a), L.ptr(radii), L.ptr(geom), L.ptr(img), L.ptr(binning),
                                                  C.byref(info), L.ptr(color), L.ptr(invdepth) if do_depth else None,
                                                  L.ptr(seen) if need_seen else None, s))
        _binning_hint[dev] = int(need * 1.15)
    del keep
    return int(info.num_rendered), color, radii, geom, binning, img, invdepth, seen


def rasterize_gaussians_backward(bg, render_indices, parent_indices, ts, kids, means3D, radii, colors, opacities,
                                 scales, rotations, scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tan_fovx,
                                 tan_fovy, dL_dout_color, dL_dout_invdepth, sh, degree, campos, geomBuffer, R,
                                 binningBuffer, imageBuffer, debug, *, need_cov3D=True):
    """-> (dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations)
    (rasterize_points.cu:141-245).  need_cov3D=False (the autograd wrapper without cov3D_precomp) returns an empty
    dL_dcov3D and skips writing its rows."""
    lib = L.load()
    H, W = int(dL_dout_color.size(1)), int(dL_dout_color.size(2))
    a, keep, P, P_full, M = _raster_args(bg, render_indices, parent_indices, ts, kids, means3D, colors, opacities,
                                         scales, rotations, scale_modifier, cov3D_precomp, viewmatrix, projmatrix,
                                         tan_fovx, tan_fovy, H, W, sh, degree, campos, False, debug)
    dev = means3D.device
    f32 = dict(dtype=torch.float32, device=dev)
    # a colour-factored view-DP exchange takes dL/dRGB instead of the SH gradient (hlgs_core.dp.colour_factor)
    fac = dp.colour_factor(sh) if M > 0 and keep["indices"] is None else None
    out = dict(dmean2D=torch.empty((P_full, 3), **f32), dcolor=torch.empty((P_full, 3), **f32),
               dopacity=_dest(opacities, (P_full, 1), f32), dmean3D=_dest(means3D, (P_full, 3), f32, True),
               dcov3D=torch.empty((P_full if need_cov3D else 0, 6), **f32),
               dsh=fac[1] if fac is not None else _dest(sh, (P_full, M, 3), f32, True),
               dscale=_dest(scales, (P_full, 3), f32), drot=_dest(rotations, (P_full, 4), f32))
    g = L.Grads(**{k: L.ptr(v) for k, v in out.items()}, drgb=L.ptr(fac[0]) if fac is not None else None)
    dpix = dL_dout_color.contiguous().float()
    dinv = None
    if dL_dout_invdepth is not None and dL_dout_invdepth.numel() and dL_dout_invdepth.size(0) != 0:
        dinv = dL_dout_invdepth.contiguous().float()
    scratch = torch.empty((lib.hlgs_backward_scratch_size(P, int(R)),), dtype=torch.uint8, device=dev)
    # the SH backward on an overlapping exchange's late stream (hlgs_core.dp.late_stream_for), else in order
    late = dp.late_stream_for(out["dmean3D"], out["dsh"])
    L.check(lib.hlgs_rasterize_backward_split(C.byref(a), L.ptr(radii.contiguous()), L.ptr(geomBuffer),
                                              L.ptr(imageBuffer), L.ptr(binningBuffer), int(R), L.ptr(scratch),
                                              L.ptr(dpix), L.ptr(dinv), C.byref(g), L.stream(),
                                              _vp(late.cuda_stream) if late is not None else None))
    if late is not None:
        dp.note_late_work(late, list(keep.values()) + list(out.values()) +
                          [radii, geomBuffer, imageBuffer, binningBuffer, scratch, dpix, dinv])
    if fac is not None:
        fac[3](keep["campos"], degree, L.VARIANT_HIERARCHY)
    del keep
    return (out["dmean2D"], out["dcolor"], out["dopacity"], out["dmean3D"], out["dcov3D"], out["dsh"], out["dscale"],
            out["drot"])


def mark_visible(means3D, viewmatrix, projmatrix):
    """z > 0.2 view-space test per point (rasterizer_impl.cu:54-66) -> bool tensor."""
    lib = L.load()
    dev = means3D.device
    m = means3D.contiguous().float()
    L.require_gpu(m)
    present = torch.zeros((m.size(0),), dtype=torch.bool, device=dev)
    view, proj = _dev_f32(viewmatrix, dev), _dev_f32(projmatrix, dev)
    L.check(lib.hlgs_mark_visible(m.size(0), L.ptr(m), L.ptr(view), L.ptr(proj), L.ptr(present), L.stream()))
    return present


def compute_relocation(opacity_old, scale_old, N, binoms, n_max):
    """MCMC relocation (rasterize_points.cu:248-271) -> (opacity (P,), scale (3P,))."""
    lib = L.load()
    o = opacity_old.contiguous().float()
    s = scale_old.contiguous().float()
    n = N.contiguous().to(torch.int32)
    b = binoms.contiguous().float()
    L.require_gpu(o, s, n, b)
    P = o.size(0)
    new_o = torch.zeros((P,), dtype=torch.float32, device=o.device)
    new_s = torch.zeros((3 * P,), dtype=torch.float32, device=o.device)
    L.check(lib.hlgs_compute_relocation(P, L.ptr(o), L.ptr(s), L.ptr(n), L.ptr(b), int(n_max), L.ptr(new_o),
                                        L.ptr(new_s), L.stream()))
    return new_o, new_s


def _field(buf, offset, count, dtype):
    base = buf.data_ptr()
    shift = ((base + 255) & ~255) - base
    nbytes = count * torch.tensor([], dtype=dtype).element_size()
    return buf[shift + offset: shift + offset + nbytes].view(dtype)


def inspect_point_list(binningBuffer, R, P=0):
    """Sorted per-tile Gaussian ids (tile-major, front to back) held in a forward's binning buffer of a P-Gaussian
    forward (the stored entries carry a footprint quadrant mask below the id: hlgs_point_list_entry_shift)."""
    lib = L.load()
    raw = _field(binningBuffer, lib.hlgs_binning_point_list_offset(int(R)), int(R), torch.int32)
    return (raw.to(torch.int64) & 0xFFFFFFFF) >> lib.hlgs_point_list_entry_shift(int(P))


def inspect_ranges(imageBuffer, W, H):
    """[start, end) of every tile's list (tiles row-major) held in a forward's image buffer."""
    T = ((W + 15) // 16) * ((H + 15) // 16)
    return _field(imageBuffer, L.load().hlgs_image_ranges_offset(int(W), int(H)), 2 * T, torch.int32).view(T, 2)


def inspect_splats(geomBuffer, P):
    """(P, 16) float32 per-Gaussian blend records held in a forward's geometry buffer:
    [0:4] x, y, conic a, b | [4:8] conic c, opacity, r, g | [8:12] b, 1/depth, t, 1/kids |
    [12:16] 0 (unused), x0 | y0 << 16 (int bits), rect width (int bits), alpha threshold on e2
    (csrc/hlgs_internal.h, Geom::splat; a culled Gaussian's record is unspecified)."""
    return _field(geomBuffer, L.load().hlgs_geom_splat_offset(int(P)), 16 * int(P), torch.float32).view(int(P), 16)
