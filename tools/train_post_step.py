#!/usr/bin/env python3
"""Config #5's training step (train_post.py with Cache_SPTs, the alt rasterizer and the photometric loss) end to end
on one MI355X, on a synthetic hierarchy (BASELINE config #5 names the example dataset, which is not available here).

Per iteration, as train_post.py:323-812 orders it:
  1. SPTCache.step(view)             coarse cut, cache bookkeeping, SPT cut, write-back / load (pinned host storage)
  2. activations                     sigmoid(opacity), exp(scaling), normalize(rotation)  (:499-505)
  3. alt rasterizer forward          antialiasing on, active SH degree 1 (Max_SH_Degree, :110) (render_vanilla)
  4. loss                            (1 - 0.2) L1 + 0.2 (1 - fused_ssim) (:558-559), optionally + depth L1
  5. backward
  6. dense Adam                      skybox gradients zeroed, OurAdam._single_tensor_adam2 (:786-812)

Prints one JSON object: per-stage medians (CUDA events on torch's stream) and the whole step (host clock around
a synchronised step), plus Mpix/s of the step.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from hlgs_core import synthetic as S  # noqa: E402


def build(P, sky, seed=0):
    from hlgs_core import spt
    cam = S.make_camera(1920, 1080)
    leaves = S.make_gaussians(P, 3, cam, seed=seed)
    h = S.make_dynamic_hierarchy(leaves, skybox_points=sky, seed=seed)
    nodes = torch.tensor(h["nodes"])
    nodes[:, 3] = torch.where(nodes[:, 2] == 2, nodes[:, 3], torch.zeros_like(nodes[:, 3]))
    xyz = torch.tensor(h["means3D"])
    log_s = torch.log(torch.tensor(h["scales"]))
    t0 = time.perf_counter()
    b = spt.build_hierarchical_spt(nodes, xyz, log_s, sky, 0.5, 0.00228, 256)
    build_s = time.perf_counter() - t0
    shs = torch.tensor(h["shs"])
    op = torch.tensor(h["opacities"]).reshape(-1, 1).clamp(1e-4, 1 - 1e-4)
    storage = dict(xyz=xyz, f_dc=shs[:, :1].contiguous(), f_rest=shs[:, 1:].contiguous(),
                   opacity=torch.log(op / (1 - op)), scaling=log_s, rotation=torch.tensor(h["rotations"]))
    return b, storage, build_s, nodes.shape[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000, help="leaves of the synthetic hierarchy")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--sky", type=int, default=0)
    ap.add_argument("--sh-degree", type=int, default=1)
    ap.add_argument("--depth", action="store_true", help="add the masked inverse-depth L1 term (train_single.py)")
    args = ap.parse_args()
    from alt_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from hlgs_core.loss import photometric_loss
    from hlgs_core.spt_cache import SPTCache

    b, storage, build_s, G = build(args.P, args.sky)
    cache = SPTCache(storage, b, args.sky, reuse_tolerance=0.9)
    W, H = 1920, 1080
    rng = np.random.default_rng(1)
    gt = torch.tensor(rng.uniform(0, 1, (3, H, W)).astype(np.float32), device="cuda")
    mono = torch.tensor(rng.uniform(0.05, 0.5, (1, H, W)).astype(np.float32), device="cuda")
    mask = torch.ones((1, H, W), device="cuda")
    bg = torch.zeros(3, device="cuda")
    lrs = dict(xyz=1.6e-4, f_dc=2.5e-3, f_rest=2.5e-3 / 20, opacity=5e-2, scaling=5e-3, rotation=1e-3)
    path = [S.make_camera(W, H, T=np.array([0.03 * k, 0.01 * k, 0.2 * math.sin(0.3 * k)])) for k in range(args.steps + 3)]

    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    stages = {k: [] for k in ("cache", "forward", "loss", "backward", "adam")}
    step_ms, resident = [], []
    for it, cam in enumerate(path):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e = [ev() for _ in range(6)]
        e[0].record()
        cache.step(cam["projmatrix"], cam["campos"])
        e[1].record()
        p = cache.params
        means3D = p["xyz"]
        opac = torch.sigmoid(p["opacity"])
        scales = torch.exp(p["scaling"])
        rots = torch.nn.functional.normalize(p["rotation"])
        s = GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"],
                                          bg=bg, scale_modifier=1.0, viewmatrix=cam["viewmatrix"].cuda(),
                                          projmatrix=cam["projmatrix"].cuda(), sh_degree=args.sh_degree,
                                          campos=cam["campos"].cuda(), prefiltered=False, debug=False,
                                          antialiasing=True)
        means2D = torch.zeros_like(means3D, requires_grad=True)
        img, radii, invd = GaussianRasterizer(s)(means3D=means3D, means2D=means2D, dc=p["f_dc"], shs=p["f_rest"],
                                                 opacities=opac, scales=scales, rotations=rots)
        img = img.clamp(0, 1)
        e[2].record()
        if args.depth:
            loss = photometric_loss(img, gt, 0.2, invd, mono, mask, 0.5)[0]
        else:
            loss = photometric_loss(img, gt, 0.2)[0]
        e[3].record()
        loss.backward()
        e[4].record()
        cache.optimizer_step(it, lrs)
        e[5].record()
        torch.cuda.synchronize()
        if it >= 3:
            step_ms.append((time.perf_counter() - t0) * 1e3)
            for k, (a, bb) in zip(stages, zip(e[:-1], e[1:])):
                stages[k].append(a.elapsed_time(bb))
            resident.append(cache.render_indices.numel())
        for q in p.values():
            q.grad = None
    ms = float(np.median(step_ms))
    out = dict(workload=f"train_post.py step with the SPT cache: {G}-node synthetic hierarchy ({args.P} leaves), "
                        f"{W}x{H}, alt rasterizer (antialiasing, SH degree {args.sh_degree}), "
                        f"L1 + D-SSIM{' + depth L1' if args.depth else ''}, dense Adam",
               data="synthetic (seeded PCG64 hierarchy, target image and camera path)",
               spt_build_s=round(build_s, 3), resident_median=int(np.median(resident)), step_ms=round(ms, 3),
               Mpix_s=round(W * H / ms / 1e3, 1),
               stages_ms={k: round(float(np.median(v)), 3) for k, v in stages.items()}, steps=len(step_ms))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
