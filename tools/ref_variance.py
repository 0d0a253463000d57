"""How far two faithful builds of the reference's own float operation order differ on one frame: the oracle in
reference-order mode built without contraction (gcc -ffp-contract=off) and with a*b+c contracted into FMAs (the
reference is built by nvcc with its default --fmad=true, submodules/hierarchy-rasterizer/setup.py:31).  CPU only.

    python tools/ref_variance.py [P] [deg] [W] [H]      (default: configs[1], 1M Gaussians, SH 3, 1920x1080)
"""
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "hierarchical-lod-gaussians_amd"))

from oracle import oracle as O  # noqa: E402
from hlgs_core import synthetic as S  # noqa: E402
import bench  # noqa: E402


def frames(P, deg, W, H):
    cam = S.make_camera(W, H)
    sc = S.make_gaussians(P, deg, cam, seed=0)
    g, gd = S.upstream_grads(W, H, seed=1)
    cn = S.cam_numpy(cam)
    out = {}

    def run(key):
        with O.reference_order(omp=key):
            out[key] = bench._oracle_frame(O, sc, cn, g, gd, omp=key)[1]
    th = [threading.Thread(target=run, args=(k,)) for k in (False, "fma")]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return out[False], out["fma"]


if __name__ == "__main__":
    a = [int(x) for x in sys.argv[1:]] + [1_000_000, 3, 1920, 1080][len(sys.argv) - 1:]
    ref, fma = frames(*a[:4])
    rep = bench.parity_report(fma, ref, "reference order, contracted vs uncontracted build")
    print(json.dumps(rep, indent=1))
