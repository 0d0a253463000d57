"""Full-size forward parity diagnosis (GPU vs oracle, configs[1] scene): where and why pixels differ.
Prints the error distribution and, for the worst pixels, n_contrib / final T on both sides."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hlgs_core import synthetic as S  # noqa: E402
from oracle import oracle as O  # noqa: E402

P, W, H = int(os.environ.get("P", 1_000_000)), 1920, 1080
cam = S.make_camera(W, H)
sc = S.make_gaussians(P, 3, cam, seed=0)
O.build()
fr = O.forward(sc, S.cam_numpy(cam), do_depth=True)
from diff_gaussian_rasterization import _C  # noqa: E402
t = lambda a: torch.tensor(a, device="cuda")  # noqa: E731
e = torch.empty(0, device="cuda")
out = _C.rasterize_gaussians(cam["bg"].cuda(), e, e, e, e, t(sc["means3D"]), e, t(sc["opacities"]), t(sc["scales"]),
                             t(sc["rotations"]), 1.0, e, cam["viewmatrix"].cuda(), cam["projmatrix"].cuda(),
                             cam["tanfovx"], cam["tanfovy"], H, W, t(sc["shs"]), 3, cam["campos"].cuda(), False, False,
                             True)
color = out[1].cpu().numpy()
img = out[5]
N = W * H
off_nc = (4 * N + 255) // 256 * 256
fT = _C._field(img, 0, N, torch.float32).cpu().numpy()
nc = _C._field(img, off_nc, N, torch.int32).cpu().numpy()
err = np.abs(color - fr.color).max(0).reshape(-1)
print("R gpu/oracle", out[0], fr.R)
for thr in (1e-6, 1e-5, 3e-5, 1e-4, 2e-4):
    print(f"pixels with err > {thr:g}: {(err > thr).sum()}")
print("n_contrib differs:", int((nc != fr.n_contrib.astype(np.int32)).sum()))
worst = np.argsort(-err)[:12]
for p in worst:
    print(f"px {p % W},{p // W} err {err[p]:.3g}  nc gpu {nc[p]} ora {fr.n_contrib[p]}  T gpu {fT[p]:.6g} ora {fr.final_T[p]:.6g}")
