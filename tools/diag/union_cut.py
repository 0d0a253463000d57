"""What the config #5 union cut costs a rank.

At N > 1 every rank's SPTCache.step cuts the hierarchy for the union of the step's G views (a node survives the cull
if it reaches into any view's frustum; the nearest camera decides each LOD test), so a rank renders its own view from
a resident set that is not its own view's cut.  On one GPU, for G = 1, 2, 4, 8 views of bench.py's config5 camera
paths (rank r's camera offset 0.4 units sideways, as the N > 1 bench leg places them) and of synthetic.ring_camera,
this measures:
  - resident count of the union cut against each view's own cut (fresh-cache plans, no rows moved);
  - per-rank raster time (alt rasterizer, antialiasing, SH degree 1, fwd + bwd, 1080p) over the union set against the
    view's own set (median of event spans);
  - cache rows moved per step (write-back and load) along a path of steps, union batch against one view alone;
  - the per-view image difference, rendered from the union set against the view's own set.

    python tools/diag/union_cut.py [--P 1000000] [--json gpurun_out/union_cut.json]
"""
import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

W, H = 1920, 1080


def bench_view(k, r):
    from hlgs_core import synthetic as S
    return S.make_camera(W, H, T=np.array([0.03 * k + 0.4 * r, 0.01 * k, 0.2 * math.sin(0.3 * k)]))


def ring_view(k, r, G):
    from hlgs_core import synthetic as S
    cam = S.ring_camera(W, H, r, G, radius=0.4 * max(G - 1, 0) / 2 + 1e-9)
    return cam


def batch(cams, dev):
    fpt = torch.stack([c["projmatrix"] for c in cams]).to(dev)
    cc = torch.stack([c["campos"] for c in cams]).to(dev)
    return fpt, cc


def gather_params(storage, idx, dev):
    from hlgs_core.spt_cache import NAMES
    i = idx.long().cpu()
    return {k: storage[k][i].to(dev).contiguous().requires_grad_(True) for k in NAMES}


def render(p, cam, dev, grads=None):
    from alt_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    s = GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"],
                                      bg=torch.zeros(3, device=dev), scale_modifier=1.0,
                                      viewmatrix=cam["viewmatrix"].to(dev), projmatrix=cam["projmatrix"].to(dev),
                                      sh_degree=1, campos=cam["campos"].to(dev), prefiltered=False, debug=False,
                                      antialiasing=True)
    means2D = torch.zeros_like(p["xyz"], requires_grad=True)
    img, radii, invd = GaussianRasterizer(s)(
        means3D=p["xyz"], means2D=means2D, dc=p["f_dc"], shs=p["f_rest"], opacities=torch.sigmoid(p["opacity"]),
        scales=torch.exp(p["scaling"]), rotations=torch.nn.functional.normalize(p["rotation"]))
    if grads is not None:
        torch.autograd.backward([img, invd], list(grads))
    return img.detach(), invd.detach()


def raster_ms(p, cam, dev, iters=10):
    g = (torch.randn(3, H, W, device=dev), torch.randn(1, H, W, device=dev) * 0.1)
    ts = []
    for i in range(iters + 2):
        for t in p.values():
            t.grad = None
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        render(p, cam, dev, g)
        b.record()
        b.synchronize()
        if i >= 2:
            ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--json", default=None)
    ap.add_argument("--steps", type=int, default=6)
    args = ap.parse_args()
    import bench
    from hlgs_core.spt_cache import SPTCache
    dev = torch.device("cuda", 0)
    b, storage, _, nodes = bench.merged_two_chunk_scene(args.P)
    cache = SPTCache(storage, b, 0, reuse_tolerance=0.9, device=dev)
    out = dict(P=args.P, nodes=nodes, W=W, H=H, paths={})
    for path_name in ("bench_config5", "ring"):
        res = {}
        for G in (1, 2, 4, 8):
            k0 = 3
            cams = [bench_view(k0, r) if path_name == "bench_config5" else ring_view(k0, r, G) for r in range(G)]
            union = cache.plan(*batch(cams, dev))["render_indices"]
            own = [cache.plan(*batch([c], dev))["render_indices"] for c in cams]
            pu = gather_params(cache.storage, union, dev)
            rows = []
            for c, o in zip(cams, own):
                po = gather_params(cache.storage, o, dev)
                iu, du = render(pu, c, dev)
                io, do = render(po, c, dev)
                d = (iu - io).abs()
                mse = float(((iu.clamp(0, 1) - io.clamp(0, 1)) ** 2).mean())
                rows.append(dict(own_resident=int(o.numel()), raster_ms_union=round(raster_ms(pu, c, dev), 4),
                                 raster_ms_own=round(raster_ms(po, c, dev), 4), image_linf=float(d.max()),
                                 image_mean_abs=float(d.mean()),
                                 psnr_union_vs_own=round(10 * math.log10(1.0 / max(mse, 1e-12)), 2),
                                 invdepth_linf=float((du - do).abs().max())))
                del po
            del pu
            # rows moved along a path of steps: the union batch against view 0 alone
            moved = {}
            for tag, views in (("union", lambda k: [bench_view(k, r) if path_name == "bench_config5" else
                                                    ring_view(k, r, G) for r in range(G)]),
                               ("view0", lambda k: [bench_view(k, 0) if path_name == "bench_config5" else
                                                    ring_view(k, 0, G)])):
                c2 = SPTCache(storage, b, 0, reuse_tolerance=0.9, device=dev)
                loads, wbs, res_n = [], [], []
                for k in range(args.steps):
                    c2.step(*batch(views(k), dev))
                    pl = c2.last_plan
                    if k >= 1:
                        loads.append(int(pl["load_from_disk_indices"].numel()))
                        wbs.append(int(pl["write_back_rows"].numel()))
                        res_n.append(int(pl["render_indices"].numel()))
                moved[tag] = dict(load_per_step=float(np.mean(loads)), write_back_per_step=float(np.mean(wbs)),
                                  resident=float(np.mean(res_n)))
                del c2
                torch.cuda.empty_cache()
            res[G] = dict(union_resident=int(union.numel()), views=rows, moved=moved,
                          union_over_mean_own=round(union.numel() / np.mean([r["own_resident"] for r in rows]), 3))
            print(path_name, G, json.dumps(res[G]), flush=True)
        out["paths"][path_name] = res
    s = json.dumps(out, indent=1)
    if args.json:
        os.makedirs(os.path.dirname(args.json), exist_ok=True)
        open(args.json, "w").write(s)
    print(s)


if __name__ == "__main__":
    main()
