"""How far faithful float32 builds of the same arithmetic differ on the configs[2] LOD-chain frame (CPU only).

The test_gpu_configs.py::test_configs2_lod_chain_1080p gradients of the lerped parents go through an ill-conditioned
conic -> cov2D -> cov3D backward.  This runs the chain on the CPU (oracle cut, weights and lerp: the GPU matches
them bit for bit / to 1e-6) and renders the lerped scene with
  - the oracle (A-17 contract, uncontracted: the test's reference),
  - the oracle built with a*b+c contracted (-ffp-contract=fast -mfma),
  - the reference's own alpha order, uncontracted and contracted (nvcc's default --fmad=true),
then reports grad_check's element-wise ratio (row_rtol as the test uses) between each pair.

    python tools/diag/lod_chain_variance.py [n_leaves]
"""
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

from hlgs_core import synthetic as S  # noqa: E402
from helpers import grad_check, rel_err  # noqa: E402
from oracle import oracle as O  # noqa: E402


def lerped_scene(n_leaves, W=1920, H=1080, deg=3, tau_px=6.0):
    cam = S.make_camera(W, H)
    h = S.make_dynamic_hierarchy(S.make_gaussians(n_leaves, deg, cam, seed=0), seed=0)
    tau = (2 * (tau_px + 0.5)) * cam["tanfovx"] / (0.5 * W)
    vp, vd = cam["campos"].numpy(), np.array([0.0, 0.0, 1.0], np.float32)
    n, ri, pi, ni = O.expand_to_size_dynamic(h["nodes"], h["means3D"], h["scales"], tau, vp, vd)
    ts, kids = O.interp_weights_dynamic(ni[:n], tau, h["nodes"], h["means3D"], h["scales"], vp)
    has_parent = h["nodes"][ri[:n], 1] >= 0
    pi = pi[:n].copy()
    pi[~has_parent] = 0
    ref_l = O.lod_interp_forward(0, ri[:n], pi, ts[:n], h["means3D"], h["scales"], h["rotations"], h["opacities"],
                                 h["shs"])
    sc = dict(means3D=ref_l["means"], scales=ref_l["scales"], rotations=ref_l["rots"], opacities=ref_l["opac"],
              shs=ref_l["shs"], sh_degree=deg)
    return sc, cam


def render(sc, cam, g, gd, lib, ref_order):
    cn = S.cam_numpy(cam)
    prev = O.lib(lib).orc_get_alpha_mode()
    O.set_reference_order(ref_order, lib)
    try:
        fr = O.forward(sc, cn, omp=lib)
        gr = O.backward(fr, sc, g, gd)
    finally:
        O.set_reference_order(bool(prev), lib)
    return dict(dmean3D=gr["dmean3D"], dopacity=gr["dopacity"], d_shs=gr["dsh"], d_scales=gr["dscale"],
                d_rotations=gr["drot"], color=fr.color)


if __name__ == "__main__":
    n_leaves = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    sc, cam = lerped_scene(n_leaves)
    g, gd = S.upstream_grads(cam["W"], cam["H"], seed=1)
    runs = {}

    def run(name, lib, ref_order):
        runs[name] = render(sc, cam, g, gd, lib, ref_order)
    # the plain and the contracted builds are separate libraries, so the two modes of each run one after the other
    def both(lib, names):
        run(names[0], lib, False)
        run(names[1], lib, True)
    th = [threading.Thread(target=both, args=(False, ("oracle", "ref_order"))),
          threading.Thread(target=both, args=("fma", ("oracle_fma", "ref_order_fma")))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    out = {}
    for a, b in (("oracle_fma", "oracle"), ("ref_order", "oracle"), ("ref_order_fma", "ref_order"),
                 ("ref_order_fma", "oracle")):
        rep = {}
        for k in ("dmean3D", "dopacity", "d_shs", "d_scales", "d_rotations"):
            row = 1e-3 if k in ("d_scales", "d_rotations") else 0.0
            ratio, _ = grad_check(runs[a][k], runs[b][k], row_rtol=row)
            rep[k] = dict(elementwise_ratio=round(ratio, 4), rel=float(f"{rel_err(runs[a][k], runs[b][k]):.3g}"))
        out[f"{a} vs {b}"] = rep
    print(json.dumps(out, indent=1))
