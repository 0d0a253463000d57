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

and gates the GPU's distance on the measured build-to-build variance:
  - pixels above 1e-4: at most the builds' own count + 2;
  - colour L-inf: at most 2x the builds' mutual colour L-inf; inverse-depth L-inf <= 1e-3;
  - max per-tensor gradient error (max|d| / max|ref|): at most 2x the builds' own, and <= north_star's 1e-3;
  - every pixel above 1e-4 is explained: one of its pairs is kept by one order and skipped by the other (alpha within
    float rounding of 1/255, oracle.pixel_pairs), or the two forward walks stop at different contributors.
On the configs[1] frame (tools/ref_flips.py) each of the 3 pixels is one pair whose alpha rounds to 1/255f exactly in
the reference's order while its exact value is below 1/255 (or the reverse); the largest, pixel (668, 1033), is such a
pair that BOTH reference builds keep, so it is absent from their mutual variance, which is why the GPU's colour L-inf
(7.2e-4) exceeds the builds' mutual 3.9e-4.
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
    """Both reference-order oracle frames (and the frame objects, for pixel_pairs), each on its own thread (ctypes
    releases the GIL)."""
    cn = S.cam_numpy(cam)
    out, frs = {}, {}

    def run(key):
        with O.reference_order(omp=key):
            fr = O.forward(sc, cn, do_depth=True, omp=key)
            gr = O.backward(fr, sc, g, gd)
        frs[key] = fr
        out[key] = dict(color=fr.color, invdepth=fr.invdepth, dmean3D=gr["dmean3D"], dmean2D=gr["dmean2D"],
                        dopacity=gr["dopacity"], dscale=gr["dscale"], drot=gr["drot"], dsh=gr["dsh"])
    th = [threading.Thread(target=run, args=(k,)) for k in (False, "fma")]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return out[False], out["fma"], frs[False], frs["fma"]


def _unexplained(gpu, ref, fr_contract_lists, fr_ref, tol=1e-4):
    """Pixels where the GPU (bit-exact with the shared contract) and a reference-order frame differ by more than tol
    without a threshold flip: no pair kept by one order and skipped by the other, and equal walk lengths."""
    d = np.maximum(np.abs(gpu["color"] - ref["color"]).max(0), np.abs(gpu["invdepth"] - ref["invdepth"]).max(0))
    bad = []
    for y, x in zip(*np.nonzero(d > tol)):
        pc, pr = O.pixel_pairs(fr_contract_lists, int(x), int(y)), O.pixel_pairs(fr_ref, int(x), int(y))
        flips = np.nonzero(pc["keep"][:, 0] != pr["keep"][:, 1])[0]
        if not len(flips) and pc["last"][0] == pr["last"][1]:
            bad.append((int(x), int(y), float(d[y, x])))
    return bad


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
    ref, fma, fr_ref, fr_fma = _reference_order_frames(sc, cam, g, gd)
    reps = {"gpu_vs_ref": _report(gpu, ref), "gpu_vs_ref_fma": _report(gpu, fma), "ref_fma_vs_ref": _report(fma, ref)}
    print(json.dumps(reps, indent=1))
    v = reps["ref_fma_vs_ref"]
    v_grad = max(v["grad_rel"].values())
    assert v["pixels_above_1e_4"] <= PIX_BOUND and v_grad <= GRAD_REL, reps
    for name, fr_b in (("gpu_vs_ref", fr_ref), ("gpu_vs_ref_fma", fr_fma)):
        r = reps[name]
        assert r["pixels_above_1e_4"] <= v["pixels_above_1e_4"] + 2, (name, reps)
        assert r["color_linf"] <= 2 * v["color_linf"], (name, reps)
        assert r["invdepth_linf"] <= LINF_BOUND, (name, reps)
        assert max(r["grad_rel"].values()) <= min(2 * v_grad, GRAD_REL), (name, reps)
        # the serial reference-order frame's build also decides in the shared contract (mode 0): its lists are the
        # GPU's (bit-exact), so its mode-0 decisions are the GPU's
        bad = _unexplained(gpu, ref if fr_b is fr_ref else fma, fr_ref, fr_b)
        assert not bad, (name, "pixels above 1e-4 without a threshold flip", bad)
