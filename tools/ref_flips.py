"""Which pixels differ between the shared arithmetic contract (DESIGN A-17; the GPU is bit-exact with it) and the
reference's own float operation order on the configs[1] frame, and why: for every pixel above 1e-4, the pairs whose
threshold decision (power > 0, alpha < 1/255) flips between the two orders, and the forward walks' contributor counts
(a T < 1e-4 stop that flips shows there).  CPU only (the oracle builds), ~1 min.

    python tools/ref_flips.py [--P 1000000] [--W 1920] [--H 1080] [--json out.json]
"""
import argparse
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]

import numpy as np  # noqa: E402

from hlgs_core import synthetic as S  # noqa: E402
from oracle import oracle as O  # noqa: E402


def frames(sc, cn):
    out = {}

    def run(key, ref_order, omp):
        if ref_order:
            with O.reference_order(omp=omp):
                out[key] = O.forward(sc, cn, do_depth=True, omp=omp)
        else:
            out[key] = O.forward(sc, cn, do_depth=True, omp=omp)
    th = [threading.Thread(target=run, args=("contract", False, False)),
          threading.Thread(target=run, args=("ref_fma", True, "fma"))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    run("ref", True, False)  # the serial build's alpha mode is global: after the contract frame is done
    return out


def explain(a, b, ca, cb, tol=1e-4, max_pixels=64):
    """Pixels where frames a and b differ by more than tol, each with the pairs whose keep decision differs between a
    (alpha mode ca of a's oracle build: 0 the shared contract, 1 the reference's order) and b (mode cb of b's build) --
    the tile lists are identical in every frame -- and both walks' contributor counts."""
    d = np.maximum(np.abs(a.color - b.color).max(0), np.abs(a.invdepth - b.invdepth).max(0))
    ys, xs = np.nonzero(d > tol)
    rows = []
    for y, x in list(zip(ys.tolist(), xs.tolist()))[:max_pixels]:
        pa, pb = O.pixel_pairs(a, x, y), O.pixel_pairs(b, x, y)
        assert np.array_equal(pa["ids"], pb["ids"])
        la, lb = int(pa["last"][ca]), int(pb["last"][cb])
        ka, kb = pa["keep"][:, ca], pb["keep"][:, cb]
        flips = [dict(pos=int(k), id=int(pa["ids"][k]), alpha_a=float(pa["alpha"][k, ca]),
                      alpha_b=float(pb["alpha"][k, cb]), kept_a=bool(ka[k]), kept_b=bool(kb[k]))
                 for k in range(min(max(la, lb) + 1, len(ka))) if ka[k] != kb[k]]
        rows.append(dict(x=x, y=y, diff=float(d[y, x]), color_diff=float(np.abs(a.color - b.color)[:, y, x].max()),
                         invdepth_diff=float(np.abs(a.invdepth - b.invdepth)[0, y, x]),
                         n_contrib=[int(a.n_contrib[y * a.W + x]), int(b.n_contrib[y * b.W + x])],
                         walk_last=[la, lb], flips=flips, explained=bool(flips) or la != lb))
    return dict(pixels_above=int((d > tol).sum()), linf=float(d.max()), pixels=rows)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    cam = S.make_camera(args.W, args.H)
    sc = S.make_gaussians(args.P, 3, cam, seed=0)
    fr = frames(sc, S.cam_numpy(cam))
    rep = {"contract_vs_ref": explain(fr["contract"], fr["ref"], 0, 1),
           "contract_vs_ref_fma": explain(fr["contract"], fr["ref_fma"], 0, 1),
           "ref_fma_vs_ref": explain(fr["ref_fma"], fr["ref"], 1, 1)}
    s = json.dumps(rep, indent=1)
    if args.json:
        open(args.json, "w").write(s)
    print(s)


if __name__ == "__main__":
    main()
