"""configs[1] against the reference's OWN float operation order, gated.

The bit-exact gate (tests/test_gpu_configs.py) compares the GPU with an oracle that decides the four threshold tests
(power > 0, alpha < 1/255, T < 1e-4, alpha > 0.99) exactly as the GPU does (DESIGN A-17).  The reference decides them
in its own float order: power = -0.5f*(a*dx*dx + c*dy*dy) - b*dx*dy, expf(power), alpha < 1.0f/255.0f
(forward.cu:538-563, backward.cu:612-643), built by nvcc with its default --fmad=true
(submodules/hierarchy-rasterizer/setup.py:31).  A pair whose alpha lies within float rounding of 1/255 flips with the
rounding, so two faithful builds of that very source already disagree on a handful of pixels.  This test measures
three distances on the full 1M-Gaussian, 1920x1080 frame:

  gpu vs ref      the GPU against the oracle in reference order, no contraction (gcc -ffp-contract=off)
  gpu vs ref_fma  the GPU against the same oracle source with a*b+c contracted (gcc -ffp-contract=fast -mfma)
  ref_fma vs ref  the reference order's own build-to-build variance

and fails if the GPU is further from either reference-order build than a fixed bound: at most 10 pixels above
north_star's 1e-4, colour / inverse-depth L-inf <= 1e-3, and every gradient tensor within north_star's 1e-3
(max|d| / max|ref|).  The build-to-build variance is asserted to be of the same order (it is what makes the 1e-4
per-pixel bound unattainable for any reimplementation of this float order), and all three reports are printed.
"""
import json
import threading

import numpy as np
import pytest

from hlgs_core import synthetic as S
from helpers import gpu_render
from oracle import oracle as O

pytestmark = pytest.mark.gpu
PIX_BOUND = 10
LINF_BOUND = 1e-3
GRAD_REL = 1e-3
GRAD_KEYS = {"dmean3D": "dmean3D", "dmean2D": "dmean2D", "dopacity": "dopacity", "dscale": "d_scales",
             "drot": "d_rotations", "dsh": "d_shs"}


def _reference_order_frames(sc, cam, g, gd):
    """Both reference-order oracle frames, each on its own thread (ctypes releases the GIL)."""
    cn = S.cam_numpy(cam)
    out = {}

    def run(key):
        with O.reference_order(omp=key):
            fr = O.forward(sc, cn, do_depth=True, omp=key)
            gr = O.backward(fr, sc, g, gd)
        out[key] = dict(color=fr.color, invdepth=fr.invdepth, dmean3D=gr["dmean3D"], dmean2D=gr["dmean2D"],
                        dopacity=gr["dopacity"], dscale=gr["dscale"], drot=gr["drot"], dsh=gr["dsh"])
    th = [threading.Thread(target=run, args=(k,)) for k in (False, "fma")]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return out[False], out["fma"]


def _report(a, b):
    dc = np.abs(a["color"] - b["color"])
    di = np.abs(a["invdepth"] - b["invdepth"])
    rep = dict(color_linf=float(dc.max()), invdepth_linf=float(di.max()),
               pixels_above_1e_4=int((np.maximum(dc.max(0), di.max(0)) > 1e-4).sum()), grad_rel={})
    for k in GRAD_KEYS:
        x = a[k].reshape(b[k].shape[0], -1)[:, :b[k].reshape(b[k].shape[0], -1).shape[1]]
        y = b[k].reshape(b[k].shape[0], -1)
        rep["grad_rel"][k] = float(np.abs(x - y).max() / max(float(np.abs(y).max()), 1e-30))
    return rep


def test_configs1_reference_order_within_bound():
    P, deg, W, H = 1_000_000, 3, 1920, 1080
    cam = S.make_camera(W, H)
    sc = S.make_gaussians(P, deg, cam, seed=0)
    g, gd = S.upstream_grads(W, H, seed=1)
    out = gpu_render(sc, cam, grads=(g, gd))
    gpu = dict(color=out["color"], invdepth=out["invdepth"], **{k: out[v] for k, v in GRAD_KEYS.items()})
    ref, fma = _reference_order_frames(sc, cam, g, gd)
    reps = {"gpu_vs_ref": _report(gpu, ref), "gpu_vs_ref_fma": _report(gpu, fma), "ref_fma_vs_ref": _report(fma, ref)}
    print(json.dumps(reps, indent=1))
    for name in ("gpu_vs_ref", "gpu_vs_ref_fma"):
        r = reps[name]
        assert r["pixels_above_1e_4"] <= PIX_BOUND, (name, reps)
        assert max(r["color_linf"], r["invdepth_linf"]) <= LINF_BOUND, (name, reps)
        assert max(r["grad_rel"].values()) <= GRAD_REL, (name, reps)
    # the reference order's own variance is of the same order as the GPU's distance from it
    v = reps["ref_fma_vs_ref"]
    assert v["pixels_above_1e_4"] <= PIX_BOUND and max(v["grad_rel"].values()) <= GRAD_REL, reps
