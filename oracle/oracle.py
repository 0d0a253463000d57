"""ctypes front-end to the C restatement in oracle/hlgs_oracle.c.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product path.  All inputs/outputs
are numpy arrays (float32 / int32), mirroring the tensors the reference's torch
glue passes to its kernels (submodules/hierarchy-rasterizer/rasterize_points.cu:36-245).
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SRC = os.path.join(_HERE, "hlgs_oracle.c")
_LIB = os.path.join(_HERE, "build", "libhlgs_oracle.so")
_LIB_OMP = os.path.join(_HERE, "build", "libhlgs_oracle_omp.so")  # all-cores timing leg of bench.py only
# The same source with a*b+c contracted into FMAs (gcc -ffp-contract=fast -mfma): the reference is built by nvcc with
# its default --fmad=true (submodules/hierarchy-rasterizer/setup.py:31 passes no --fmad=false), so its float results
# are those of a contracted build.  Used only to measure how far two faithful builds of the reference's own operation
# order differ from each other (tests/test_gpu_refparity.py, bench.py parity.reference_order).
_LIB_FMA = os.path.join(_HERE, "build", "libhlgs_oracle_fma.so")

_f = C.POINTER(C.c_float)
_i = C.POINTER(C.c_int)
_u = C.POINTER(C.c_uint32)
_b = C.POINTER(C.c_uint8)


def build(force=False):
    """Compile the oracle with gcc (serial, no fast-math, no FMA contraction), and the same source with OpenMP
    for the all-cores CPU baseline (libhlgs_oracle_omp.so; its gradient sums use atomics, so it is never a
    parity reference)."""
    os.makedirs(os.path.dirname(_LIB), exist_ok=True)
    base = ["gcc", "-O2", "-fPIC", "-shared", "-std=c11", "-fno-fast-math"]
    for lib_, extra in ((_LIB, ["-ffp-contract=off"]), (_LIB_OMP, ["-ffp-contract=off", "-fopenmp"]),
                        (_LIB_FMA, ["-ffp-contract=fast", "-mfma"])):
        if force or not os.path.exists(lib_) or os.path.getmtime(lib_) < os.path.getmtime(_SRC):
            subprocess.check_call(base + extra + ["-o", lib_, _SRC, "-lm"])
    return _LIB


class _Args(C.Structure):
    _fields_ = [("P", C.c_int), ("D", C.c_int), ("M", C.c_int), ("W", C.c_int), ("H", C.c_int),
                ("bg", _f), ("means3D", _f), ("shs", _f), ("colors_precomp", _f), ("opacities", _f),
                ("scales", _f), ("rotations", _f), ("cov3D_precomp", _f), ("viewmatrix", _f),
                ("projmatrix", _f), ("campos", _f), ("scale_modifier", C.c_float), ("tanfovx", C.c_float),
                ("tanfovy", C.c_float), ("indices", _i), ("parent_indices", _i), ("ts", _f), ("kids", _i),
                ("dc", _f), ("antialiasing", C.c_int), ("alt", C.c_int), ("drop_empty", C.c_int)]


class _Geom(C.Structure):
    _fields_ = [("depths", _f), ("clamped", _b), ("means2D", _f), ("cov3D", _f), ("conic_opacity", _f),
                ("rgb", _f), ("tiles_touched", _u), ("point_offsets", _u), ("rects", _i), ("radii", _i)]


class _Img(C.Structure):
    _fields_ = [("final_T", _f), ("n_contrib", _u), ("ranges", _u), ("point_list", _u), ("pixel_colors", _f),
                ("pixel_invdepths", _f)]


class _Grads(C.Structure):
    _fields_ = [("dmean2D", _f), ("dconic", _f), ("dopacity", _f), ("dcolor", _f), ("dinvdepth", _f),
                ("dmean3D", _f), ("dcov3D", _f), ("dsh", _f), ("dscale", _f), ("drot", _f), ("ddc", _f)]


_libs = {}


def lib(omp=False):
    """The serial oracle (omp=False, every parity check), its OpenMP build (omp=True, timing only) or its contracted
    build (omp="fma", the reference-variance measurement)."""
    L = _libs.get(omp)
    if L is None:
        build()
        # HLGS_ORACLE_LIB: the serial oracle built with other flags (tests/sanitize/build.py: ASan + UBSan)
        L = C.CDLL(_LIB_FMA if omp == "fma" else _LIB_OMP if omp else os.environ.get("HLGS_ORACLE_LIB") or _LIB)
        L.orc_set_alpha_mode.argtypes = [C.c_int]
        L.orc_get_alpha_mode.restype = C.c_int
        L.orc_num_threads.restype = C.c_int
        L.orc_forward_preprocess.restype = C.c_int
        L.orc_forward_preprocess.argtypes = [C.POINTER(_Args), C.POINTER(_Geom)]
        L.orc_forward_render.restype = None
        L.orc_forward_render.argtypes = [C.POINTER(_Args), C.POINTER(_Geom), C.POINTER(_Img), C.c_int, _f, _f, _i]
        L.orc_backward.restype = None
        L.orc_backward.argtypes = [C.POINTER(_Args), C.POINTER(_Geom), C.POINTER(_Img), C.c_int, _f, _f,
                                   C.POINTER(_Grads)]
        L.orc_mark_visible.argtypes = [C.c_int, _f, _f, _f, _b]
        L.orc_compute_relocation.argtypes = [C.c_int, _f, _f, _i, _f, C.c_int, _f, _f]
        L.orc_expand_to_size_dynamic.restype = C.c_int
        L.orc_expand_to_size_dynamic.argtypes = [C.c_int, C.c_float, _i, _f, _f, _f, _f, _i, _i, _i]
        L.orc_interp_weights_dynamic.argtypes = [C.c_int, _i, C.c_float, _i, _f, _f, _f, _f, _i]
        L.orc_expand_to_size.restype = C.c_int
        L.orc_expand_to_size.argtypes = [C.c_int, C.c_float, _i, _f, _f, _i, _i, _i]
        L.orc_interp_weights.argtypes = [C.c_int, _i, C.c_float, _i, _f, _f, _f, _i]
        L.orc_spt_cut.restype = C.c_int
        L.orc_spt_cut.argtypes = [C.c_int, C.c_int, _i, _i, _f, _f, _i, _f, C.c_int, _i, _i, _i]
        L.orc_lod_interp_forward.argtypes = [C.c_int, C.c_int, C.c_int, _i, _i, _f, _f, _f, _f, _f, _f,
                                             _f, _f, _f, _f, _f]
        L.orc_lod_interp_backward.argtypes = [C.c_int, C.c_int, C.c_int, _i, _i, _f, _f, _f, _f, _f, _f,
                                              _f, _f, _f, _f, _f, _f]
        L.orc_sh_colors.argtypes = [C.c_int, C.c_int, C.c_int, _f, _f, _f, _f, _b]
        L.orc_pixel_pairs.restype = C.c_int
        L.orc_pixel_pairs.argtypes = [C.POINTER(_Args), C.POINTER(_Geom), C.POINTER(_Img), C.c_int, C.c_int, C.c_int,
                                      _i, _f, _i]
        _libs[omp] = L
    return L


def set_reference_order(on, omp=False):
    """Alpha decisions in the reference's own float op order (True) or the shared A-17 contract (False, the
    default and the bit-exact gate); see orc_set_alpha_mode in hlgs_oracle.c."""
    lib(omp).orc_set_alpha_mode(int(bool(on)))


class reference_order:
    """Context manager: the oracle decides alpha in the reference's float op order inside the block."""

    def __init__(self, omp=False):
        self.omp = omp

    def __enter__(self):
        self.prev = lib(self.omp).orc_get_alpha_mode()
        set_reference_order(True, self.omp)
        return self

    def __exit__(self, *exc):
        set_reference_order(self.prev, self.omp)
        return False


def num_threads(omp=True):
    return lib(omp).orc_num_threads()


def _p(a, t=_f):
    if a is None:
        return C.cast(None, t)
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(t)


def _f32(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float32)


def _i32(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.int32)


class Frame:
    """Everything one oracle forward produced (the analogue of geomBuffer/binningBuffer/imgBuffer)."""


def _make_args(scene, cam, keep):
    """scene: dict of numpy arrays; cam: dict(W,H,tanfovx,tanfovy,viewmatrix,projmatrix,campos,bg).
    scene["alt"] = True selects the alt-rasterizer variant: scene["dc"] (P,1,3) holds the degree-0
    coefficient, scene["shs"] (P,M,3) the M higher ones, scene["antialiasing"] the AA flag."""
    d = {k: (_f32(v) if k not in ("indices", "parent_indices", "kids") else _i32(v)) for k, v in scene.items()
         if not isinstance(v, (bool, int, float))}
    cd = {k: _f32(v) for k, v in cam.items() if k in ("viewmatrix", "projmatrix", "campos", "bg")}
    keep.extend(list(d.values()) + list(cd.values()))
    shs = d.get("shs")
    P = int(len(d["indices"])) if d.get("indices") is not None else int(d["means3D"].shape[0])
    M = int(shs.shape[1]) if shs is not None and shs.size else 0
    a = _Args(P=P, D=int(scene.get("sh_degree", 0)), M=M, W=int(cam["W"]), H=int(cam["H"]),
              bg=_p(cd["bg"]), means3D=_p(d["means3D"]), shs=_p(shs if M else None),
              colors_precomp=_p(d.get("colors_precomp")), opacities=_p(d["opacities"]),
              scales=_p(d.get("scales")), rotations=_p(d.get("rotations")),
              cov3D_precomp=_p(d.get("cov3D_precomp")), viewmatrix=_p(cd["viewmatrix"]),
              projmatrix=_p(cd["projmatrix"]), campos=_p(cd["campos"]),
              scale_modifier=float(scene.get("scale_modifier", 1.0)), tanfovx=float(cam["tanfovx"]),
              tanfovy=float(cam["tanfovy"]), indices=_p(d.get("indices"), _i),
              parent_indices=_p(d.get("parent_indices"), _i), ts=_p(d.get("ts")), kids=_p(d.get("kids"), _i),
              dc=_p(d.get("dc")), antialiasing=int(bool(scene.get("antialiasing", True))),
              alt=int(bool(scene.get("alt", False))))
    return a, P


def forward(scene, cam, do_depth=True, omp=False, drop_empty=False):
    """Full forward: returns a Frame with color (3,H,W), radii, invdepth, seen and all intermediates.
    drop_empty: bin no instance whose footprint quadrant mask is 0, as the HIP binning does when
    hlgs_point_list_drops_empty(P) (not the reference's binning: same images and gradients, shorter tile lists)."""
    L = lib(omp)
    keep = []
    a, P = _make_args(scene, cam, keep)
    a.drop_empty = int(bool(drop_empty))
    W, H = int(cam["W"]), int(cam["H"])
    fr = Frame()
    fr.keep = keep
    fr.args = a
    fr.P = P
    fr.depths = np.zeros(P, np.float32)
    fr.clamped = np.zeros(P, np.uint8)
    fr.means2D = np.zeros((P, 2), np.float32)
    fr.cov3D = np.zeros((P, 6), np.float32)
    fr.conic_opacity = np.zeros((P, 4), np.float32)
    fr.rgb = np.zeros((P, 3), np.float32)
    fr.tiles_touched = np.zeros(P, np.uint32)
    fr.point_offsets = np.zeros(P, np.uint32)
    fr.rects = np.zeros((P, 2), np.int32)
    fr.radii = np.zeros(P, np.int32)
    fr.geom = _Geom(_p(fr.depths), _p(fr.clamped, _b), _p(fr.means2D), _p(fr.cov3D), _p(fr.conic_opacity),
                    _p(fr.rgb), _p(fr.tiles_touched, _u), _p(fr.point_offsets, _u), _p(fr.rects, _i),
                    _p(fr.radii, _i))
    R = L.orc_forward_preprocess(C.byref(a), C.byref(fr.geom)) if P else 0
    fr.R = R
    gx, gy = (W + 15) // 16, (H + 15) // 16
    fr.final_T = np.zeros(W * H, np.float32)
    fr.n_contrib = np.zeros(W * H, np.uint32)
    fr.ranges = np.zeros((gx * gy, 2), np.uint32)
    fr.point_list = np.zeros(max(R, 1), np.uint32)
    fr.color = np.zeros((3, H, W), np.float32)
    do_depth = do_depth or bool(a.alt)  # the alt rasterizer always renders inverse depth
    fr.invdepth = np.zeros((1, H, W), np.float32) if do_depth else np.zeros((0, H, W), np.float32)
    fr.img = _Img(_p(fr.final_T), _p(fr.n_contrib, _u), _p(fr.ranges, _u), _p(fr.point_list, _u), _p(fr.color),
                  _p(fr.invdepth) if do_depth else C.cast(None, _f))
    fr.seen = np.zeros(P, np.int32)
    if P:
        L.orc_forward_render(C.byref(a), C.byref(fr.geom), C.byref(fr.img), R, _p(fr.color),
                             _p(fr.invdepth) if do_depth else C.cast(None, _f), _p(fr.seen, _i))
    fr.W, fr.H = W, H
    fr.omp = omp
    return fr


def backward(fr, scene, dL_dcolor, dL_dinvdepth=None):
    """Gradients in the reference's return order (rasterize_points.cu:244) as a dict."""
    L = lib(getattr(fr, "omp", False))
    Pf = int(np.asarray(scene["means3D"]).shape[0])
    M = fr.args.M
    g = {k: np.zeros(s, np.float32) for k, s in dict(
        dmean2D=(Pf, 3), dconic=(Pf, 4), dopacity=(Pf, 1), dcolor=(Pf, 3), dmean3D=(Pf, 3), dcov3D=(Pf, 6),
        dsh=(Pf, max(M, 0), 3), dscale=(Pf, 3), drot=(Pf, 4), ddc=(Pf, 1, 3)).items()}
    g["dinvdepth"] = np.zeros((Pf, 1), np.float32) if dL_dinvdepth is not None else None
    gr = _Grads(*[_p(g[k]) for k in ("dmean2D", "dconic", "dopacity", "dcolor", "dinvdepth", "dmean3D", "dcov3D",
                                    "dsh", "dscale", "drot", "ddc")])
    dpix = _f32(dL_dcolor)
    dinv = _f32(dL_dinvdepth) if dL_dinvdepth is not None else None
    if fr.P:
        L.orc_backward(C.byref(fr.args), C.byref(fr.geom), C.byref(fr.img), fr.R, _p(dpix), _p(dinv), C.byref(gr))
    return g


def pixel_pairs(fr, px, py, cap=4096):
    """Diagnostics: the threshold decisions of pixel (px, py)'s pairs on frame fr in both alpha modes (orc_pixel_pairs):
    dict(ids, keep (n, 2), alpha (n, 2), last (2,)) -- column 0 the shared contract (A-17), column 1 the reference's
    float order; last = each mode's n_contrib."""
    L = lib(getattr(fr, "omp", False))
    keep = np.zeros((cap, 2), np.int32)
    alpha = np.zeros((cap, 2), np.float32)
    last = np.zeros(2, np.int32)
    n = L.orc_pixel_pairs(C.byref(fr.args), C.byref(fr.geom), C.byref(fr.img), int(px), int(py), int(cap),
                          _p(keep, _i), _p(alpha), _p(last, _i))
    gx = (fr.W + 15) // 16
    t = (py // 16) * gx + px // 16
    rs = int(fr.ranges[t, 0])
    m = min(n, cap)
    return dict(ids=fr.point_list[rs:rs + m].copy(), keep=keep[:m], alpha=alpha[:m], last=last)


def mark_visible(means3D, viewmatrix, projmatrix):
    m = _f32(means3D)
    out = np.zeros(m.shape[0], np.uint8)
    lib().orc_mark_visible(m.shape[0], _p(m), _p(_f32(viewmatrix)), _p(_f32(projmatrix)), _p(out, _b))
    return out.astype(bool)


def compute_relocation(opacity_old, scale_old, N, binoms, n_max):
    o, s, n, b = _f32(opacity_old).reshape(-1), _f32(scale_old), _i32(N).reshape(-1), _f32(binoms)
    P = o.shape[0]
    on, sn = np.zeros(P, np.float32), np.zeros(3 * P, np.float32)
    lib().orc_compute_relocation(P, _p(o), _p(s), _p(n, _i), _p(b), int(n_max), _p(on), _p(sn))
    return on, sn


def expand_to_size_dynamic(nodes, pos, scales, target, viewpoint, viewdir):
    nd, p, s = _i32(nodes), _f32(pos), _f32(scales)
    N = nd.shape[0]
    ri, pi, ni = np.zeros(N, np.int32), np.zeros(N, np.int32), np.zeros(N, np.int32)
    n = lib().orc_expand_to_size_dynamic(N, float(target), _p(nd, _i), _p(p), _p(s), _p(_f32(viewpoint)),
                                         _p(_f32(viewdir)), _p(ri, _i), _p(pi, _i), _p(ni, _i))
    return n, ri, pi, ni


def interp_weights_dynamic(indices, target, nodes, pos, scales, viewpoint):
    ix, nd, p, s = _i32(indices), _i32(nodes), _f32(pos), _f32(scales)
    n = ix.shape[0]
    ts, kids = np.zeros(n, np.float32), np.zeros(n, np.int32)
    lib().orc_interp_weights_dynamic(n, _p(ix, _i), float(target), _p(nd, _i), _p(p), _p(s),
                                     _p(_f32(viewpoint)), _p(ts), _p(kids, _i))
    return ts, kids


def expand_to_size(nodes, boxes, target, viewpoint):
    nd, bx = _i32(nodes), _f32(boxes)
    N = nd.shape[0]
    cap = int(np.maximum(nd[:, 3], 0).sum() + np.maximum(nd[:, 4], 0).sum()) + 1
    ri, pi, ni = np.zeros(cap, np.int32), np.zeros(cap, np.int32), np.zeros(cap, np.int32)
    n = lib().orc_expand_to_size(N, float(target), _p(nd, _i), _p(bx), _p(_f32(viewpoint)), _p(ri, _i),
                                 _p(pi, _i), _p(ni, _i))
    return n, ri, pi, ni


def interp_weights(indices, target, nodes, boxes, viewpoint):
    ix, nd, bx = _i32(indices), _i32(nodes), _f32(boxes)
    n = ix.shape[0]
    ts, kids = np.zeros(n, np.float32), np.zeros(n, np.int32)
    lib().orc_interp_weights(n, _p(ix, _i), float(target), _p(nd, _i), _p(bx), _p(_f32(viewpoint)), _p(ts),
                             _p(kids, _i))
    return ts, kids


def spt_cut(gaussian_indices, starts, smax, smin, sidx, sdist, compat=True):
    gi, st, mx, mn, si, sd = (_i32(gaussian_indices), _i32(starts), _f32(smax), _f32(smin), _i32(sidx),
                              _f32(sdist))
    s = si.shape[0]
    cap = int(mx.shape[0]) + s + 1
    cut, cp, tot = np.zeros(cap, np.int32), np.zeros(max(s, 1), np.int32), np.zeros(1, np.int32)
    n = lib().orc_spt_cut(s, int(mx.shape[0]), _p(gi, _i), _p(st, _i), _p(mx), _p(mn), _p(si, _i), _p(sd),
                          int(bool(compat)), _p(cut, _i), _p(cp, _i), _p(tot, _i))
    return cut[:n].copy(), cp[:s].copy()


def lod_interp_forward(S, ridx, pidx, w, means, scales, rots, opac, shs):
    ri, pi, ww = _i32(ridx), _i32(pidx), _f32(w)
    m, s, r, o = _f32(means), _f32(scales), _f32(rots), _f32(opac).reshape(-1)
    sh = _f32(shs)
    n = ri.shape[0]
    M3 = int(sh[0].size) if sh is not None else 0
    out = dict(means=np.zeros((S + n, 3), np.float32), scales=np.zeros((S + n, 3), np.float32),
               rots=np.zeros((S + n, 4), np.float32), opac=np.zeros(S + n, np.float32),
               shs=np.zeros((S + n,) + sh.shape[1:], np.float32) if sh is not None else None)
    lib().orc_lod_interp_forward(S, n, M3, _p(ri, _i), _p(pi, _i), _p(ww), _p(m), _p(s), _p(r), _p(o), _p(sh),
                                 _p(out["means"]), _p(out["scales"]), _p(out["rots"]), _p(out["opac"]),
                                 _p(out["shs"]))
    return out


def lod_interp_backward(S, ridx, pidx, w, rots, P, g):
    ri, pi, ww, r = _i32(ridx), _i32(pidx), _f32(w), _f32(rots)
    n = ri.shape[0]
    gs = _f32(g.get("shs"))
    M3 = int(gs[0].size) if gs is not None else 0
    d = dict(means=np.zeros((P, 3), np.float32), scales=np.zeros((P, 3), np.float32),
             rots=np.zeros((P, 4), np.float32), opac=np.zeros(P, np.float32),
             shs=np.zeros((P,) + gs.shape[1:], np.float32) if gs is not None else None)
    lib().orc_lod_interp_backward(S, n, M3, _p(ri, _i), _p(pi, _i), _p(ww), _p(r), _p(_f32(g["means"])),
                                  _p(_f32(g["scales"])), _p(_f32(g["rots"])), _p(_f32(g["opac"]).reshape(-1)),
                                  _p(gs), _p(d["means"]), _p(d["scales"]), _p(d["rots"]), _p(d["opac"]),
                                  _p(d["shs"]))
    return d


def sh_colors(shs, means, campos, deg):
    s, m, c = _f32(shs), _f32(means), _f32(campos)
    P, M = s.shape[0], s.shape[1]
    rgb, cl = np.zeros((P, 3), np.float32), np.zeros(P, np.uint8)
    lib().orc_sh_colors(P, int(deg), M, _p(s), _p(m), _p(c), _p(rgb), _p(cl, _b))
    return rgb, cl
