#!/usr/bin/env python3
"""Lane utilisation of the blend backward on the bench frame (needs the `stats` variant built by
tools/build_variant.py from a raster_bwd.hip with pair counters; experiment only)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["HLGS_LIBRARY"] = os.path.join(ROOT, "hierarchical-lod-gaussians_amd", "lib", "variants", "stats.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hlgs_core import _lib as L  # noqa: E402
from hlgs_core import synthetic as S  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "tools"))
from bench_extras import settings  # noqa: E402

W, H, P = 1920, 1080, 1_000_000
cam = S.make_camera(W, H)
h = S.make_gaussians(P, 3, cam, seed=0)
t = lambda a: torch.tensor(np.ascontiguousarray(a), device="cuda", requires_grad=True)  # noqa: E731
m, sc, r, o, sh = t(h["means3D"]), t(h["scales"]), t(h["rotations"]), t(h["opacities"]), t(h["shs"])
g_np, gd_np = S.upstream_grads(W, H, seed=1)
from diff_gaussian_rasterization import GaussianRasterizer  # noqa: E402
rast = GaussianRasterizer(settings(cam, 3))
lib = L.load()
lib.hlgs_pair_stats.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
out = (C.c_ulonglong * 8)()
m2 = torch.zeros_like(m, requires_grad=True)
c, _, inv = rast(means3D=m, means2D=m2, opacities=o, shs=sh, scales=sc, rotations=r)
torch.cuda.synchronize()
lib.hlgs_pair_stats(out, 1)
torch.autograd.backward([c, inv], [torch.tensor(g_np, device="cuda"), torch.tensor(gd_np, device="cuda")])
torch.cuda.synchronize()
lib.hlgs_pair_stats(out, 1)
quads, valid, empty_quads, iters, no_reduce = list(out)[:5]
print(dict(quad_evals=quads, valid_lanes=valid, lane_util=valid / (64 * quads), empty_quad_evals=empty_quads,
           splat_iters=iters, splat_iters_without_valid_lane=no_reduce, quads_per_iter=quads / iters))
