"""Diagnose the configs[2] chain's worst element-wise gradient entries (GPU vs oracle on the GPU's lerped scene)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import test_gpu_configs as T
from helpers import grad_check, oracle_render

captured = {}
orig = T._check_frame
def spy(gpu, ref):
    captured["gpu"], captured["ref"] = gpu, ref
    raise SystemExit(0)
T._check_frame = spy
try:
    T.test_configs2_lod_chain_1080p()
except SystemExit:
    pass
gpu, ref = captured["gpu"], captured["ref"]
fr = ref["frame"]
tt = fr.tiles_touched
for k in ("dmean3D", "dmean2D", "dopacity", "d_shs", "d_scales", "d_rotations"):
    a = gpu[k][..., :ref[k].shape[-1]].astype(np.float64).reshape(len(tt), -1)
    b = ref[k].astype(np.float64).reshape(len(tt), -1)
    mx = np.abs(b).max()
    bound = 1e-3 * np.abs(b) + 1e-5 * mx
    r = np.abs(a - b) / bound
    bad = np.argwhere(r > 1)
    print(k, "max ratio", r.max(), "violations", len(bad), "max|b|", mx)
    for i, j in bad[:8]:
        print("   g", i, "c", j, "gpu", a[i, j], "ref", b[i, j], "row max|b|", np.abs(b[i]).max(), "tiles", tt[i],
              "radius", fr.radii[i])
