"""Rect instances (num_rendered, culled ones included) against binned instances (after alt_tile_keep) of the alt
rasterizer on bench.py's config5 frame: how much of the binning walk the exact per-tile culling discards."""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
import numpy as np, torch
import bench
from hlgs_core import synthetic as S
from hlgs_core.spt_cache import SPTCache
from alt_gaussian_rasterization import _C
from diff_gaussian_rasterization import _C as HC
b, storage, _, G = bench.merged_two_chunk_scene(1_000_000)
cache = SPTCache(storage, b, 0, reuse_tolerance=0.9)
W, H = 1920, 1080
for k in range(3):
    cam = {k_: (v.cuda() if torch.is_tensor(v) else v) for k_, v in S.make_camera(W, H, T=np.array([0.03 * k, 0.01 * k, 0.2 * math.sin(0.3 * k)])).items()}
    cache.step(cam["projmatrix"], cam["campos"])
    p = cache.params
    e = torch.empty(0, device="cuda")
    out = _C.rasterize_gaussians(torch.zeros(3, device="cuda"), p["xyz"].detach(), e, torch.sigmoid(p["opacity"]).detach(),
                                 torch.exp(p["scaling"]).detach(), torch.nn.functional.normalize(p["rotation"]).detach(), 1.0, e,
                                 cam["viewmatrix"], cam["projmatrix"], cam["tanfovx"], cam["tanfovy"], H, W,
                                 p["f_dc"].detach(), p["f_rest"].detach(), 1, cam["campos"], False, True, False)
    R = out[0]
    rg = HC.inspect_ranges(out[7], W, H).cpu().numpy().astype(np.int64)
    kept = int((rg[:, 1] - rg[:, 0]).sum())
    radii = out[4]
    print(f"step {k}: resident {p['xyz'].shape[0]} visible {int((radii > 0).sum())} rect instances {R} binned {kept} "
          f"({kept / max(R, 1):.3f}) longest tile list {int((rg[:, 1] - rg[:, 0]).max())}")
