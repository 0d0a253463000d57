#!/usr/bin/env python3
"""Benchmark: forward+backward Mpix/s of the MI355X Gaussian-splat rasterizer at 1080p, 1M Gaussians,
SH degree 3 (BASELINE.json configs[1]), one training view per GPU.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one view rendered through the public GaussianRasterizer API (forward, including its
num_rendered host sync), full backward of fixed synthetic upstream gradients dL/dcolor and dL/dinvdepth
(fed to autograd directly: the gradient of loss = <dL/dcolor, color> + <dL/dinvdepth, invdepth>), and -- for N > 1 -- the RCCL all-reduce of every Gaussian gradient
(view-data parallel, weak scaling: each rank renders its own view of its own 1M-Gaussian replica).
Inputs are synthetic (seeded), resident in HBM before timing starts.  Rank 0 prints one JSON line.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "hierarchical-lod-gaussians_amd")
sys.path[:0] = [ROOT, PKG]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# VALU issue ceiling: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 4 cycles each, 2400 MHz max clock
VALU_PEAK_GINSTR = 256 * 4 * 2.4 / 4


def algorithmic_bytes(stage, P, V, R, N, T, M, D):
    """Per-launch algorithmic HBM bytes of each stage."""
    return {
        "preprocess": P * (44 + 12 * M) + 83 * P,
        "scan": 8 * P,
        "count_tiles": 20 * P + 4 * T,
        "scatter": 28 * V + 12 * R,
        "tile_sort": 24 * R,
        "tile_ranges": 8 * R + 8 * T,
        "blend_fwd": 8 * T + R * (40 + 4 * D) + N * (20 + 4 * D),
        "blend_bwd": 8 * T + R * (40 + 4 * D) + N * (20 + 4 * D) + V * (36 + 4 * D),
        "gauss_bwd": V * (60 + 4 * D) + 40 * V + V * (107 + 12 * M) + V * (40 + 12 * M),
    }[stage]


STAGE_KERNEL = {"preprocess": "k_preprocess", "count_tiles": "k_count_tiles", "scatter": "k_scatter_keys",
                "tile_sort": "k_tile_sort", "tile_ranges": "k_tile_ranges", "blend_fwd": "k_blend_fwd",
                "blend_bwd": "k_blend_bwd", "gauss_bwd": "k_gauss_bwd"}


def pmc_traffic(stage, field="hbm_bytes"):
    """Per-launch HBM bytes (2 x FETCH_SIZE + WRITE_SIZE) -- or another field, e.g. valu_wave_instr -- of the
    stage's kernel from the latest committed rocprofv3 PMC profile (tools/profile_round.sh +
    tools/summarize_profile.py), or None."""
    prof = os.path.join(ROOT, "profiles")
    rounds = sorted(d for d in os.listdir(prof) if os.path.exists(os.path.join(prof, d, "pmc_traffic.json"))) \
        if os.path.isdir(prof) else []
    if not rounds or stage not in STAGE_KERNEL:
        return None, None
    path = os.path.join(prof, rounds[-1], "pmc_traffic.json")
    ks = json.load(open(path))["kernels"]
    hits = [v[field] for k, v in ks.items() if STAGE_KERNEL[stage] in k and v.get(field)]
    return (sum(hits) if hits else None), os.path.relpath(path, ROOT)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(P, deg, W, H):
    """The oracle (C restatement of the reference algorithm, 1 thread) on one full frame: fwd + bwd.
    Returns the timing summary and the oracle's outputs (same scene, camera and upstream gradients as
    rank 0's GPU step) for the full-size parity check."""
    from oracle import oracle as O
    from hlgs_core import synthetic as S
    cam = S.make_camera(W, H)
    sc = S.make_gaussians(P, deg, cam, seed=0)
    g, gd = S.upstream_grads(W, H, seed=1)
    O.build()
    t0 = time.perf_counter()
    fr = O.forward(sc, S.cam_numpy(cam), do_depth=True)
    gr = O.backward(fr, sc, g, gd)
    dt = time.perf_counter() - t0
    summary = dict(value=round(W * H / dt / 1e6, 4), unit="Mpix/s", cores=1, kind="port",
                   sample=f"one full frame: {P} Gaussians, SH deg {deg}, {W}x{H}, forward+backward, "
                          f"{dt:.2f} s on 1 thread of {cpu_model()} (os.cpu_count()={os.cpu_count()})")
    ref = dict(color=fr.color, invdepth=fr.invdepth, dmean3D=gr["dmean3D"], dmean2D=gr["dmean2D"],
               dopacity=gr["dopacity"], dscale=gr["dscale"], drot=gr["drot"], dsh=gr["dsh"])
    return summary, ref


def parity_report(gpu, ref):
    """Full-size parity of rank 0's step against the oracle: forward per-pixel L-inf and, per gradient
    tensor, max-abs error and max-abs error relative to the oracle tensor's max-abs."""
    out = dict(vs="oracle (C restatement of the reference), identical inputs, full configs[1] frame")
    out["color_linf"] = float(np.abs(gpu["color"] - ref["color"]).max())
    out["invdepth_linf"] = float(np.abs(gpu["invdepth"] - ref["invdepth"]).max())
    per = {}
    for k in ("dmean3D", "dmean2D", "dopacity", "dscale", "drot", "dsh"):
        a, b = gpu[k].reshape(ref[k].shape[0], -1), ref[k].reshape(ref[k].shape[0], -1)
        a = a[:, :b.shape[1]]
        err = float(np.abs(a - b).max())
        per[k] = dict(max_abs_err=err, rel=err / max(float(np.abs(b).max()), 1e-30))
    out["grad_max_abs_err"] = max(v["max_abs_err"] for v in per.values())
    out["grad_max_rel_err"] = max(v["rel"] for v in per.values())
    out["grads"] = per
    out["tolerance"] = dict(fwd_linf=1e-4, grad_rel=1e-3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--sh-degree", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stage-timing", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # HLGS_DIST_BACKEND=gloo with more ranks than GPUs rehearses the multi-rank path on a one-GPU box (ranks share
    # the card); the driver's N-GPU runs use the default, RCCL ("nccl"), one rank per GPU.
    backend = os.environ.get("HLGS_DIST_BACKEND", "nccl")
    gpu = local % max(1, torch.cuda.device_count()) if world > 1 else 0
    if world > 1:
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", gpu)

    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from hlgs_core import _lib as L
    from hlgs_core import synthetic as S
    from hlgs_core.dp import FlatGradExchange

    W, H, P, deg = args.W, args.H, args.P, args.sh_degree
    # every rank: the same scene replica, its own view (ring of cameras); rank 0 = configs[1] camera
    cam = S.make_camera(W, H) if world == 1 else S.ring_camera(W, H, rank, world)
    host = S.make_gaussians(P, deg, S.make_camera(W, H), seed=0)
    to = lambda a: torch.tensor(a, device=dev, requires_grad=True)  # noqa: E731
    means3D, scales, rots, opac, shs = (to(host["means3D"]), to(host["scales"]), to(host["rotations"]),
                                        to(host["opacities"]), to(host["shs"]))
    g_np, gd_np = S.upstream_grads(W, H, seed=1 + rank)
    g_col, g_inv = torch.tensor(g_np, device=dev), torch.tensor(gd_np, device=dev)
    e_i = torch.empty(0, dtype=torch.int32, device=dev)
    e_f = torch.empty(0, dtype=torch.float32, device=dev)
    rs = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"],
        bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=cam["viewmatrix"].to(dev),
        projmatrix=cam["projmatrix"].to(dev), sh_degree=deg, campos=cam["campos"].to(dev), prefiltered=False,
        debug=False, render_indices=e_i, parent_indices=e_i, interpolation_weights=e_f, num_node_kids=e_i,
        do_depth=True)
    rast = GaussianRasterizer(rs)
    params = [means3D, scales, rots, opac, shs]
    exchange = FlatGradExchange(params) if world > 1 else None
    stats = {}

    def step():
        for p in params:
            p.grad = None
        means2D = torch.zeros_like(means3D, requires_grad=True)
        color, radii, invd = rast(means3D=means3D, means2D=means2D, opacities=opac, shs=shs, scales=scales,
                                  rotations=rots)
        torch.autograd.backward([color, invd], [g_col, g_inv])
        if exchange is not None:
            exchange.allreduce()
        return radii

    for _ in range(args.warmup):
        radii = step()
    torch.cuda.synchronize()
    # frame statistics for the algorithmic-byte model
    with torch.no_grad():
        V = int((radii > 0).sum().item())
    from diff_gaussian_rasterization import _C as DC
    nr = DC.rasterize_gaussians(rs.bg, e_i, e_i, e_f, e_i, means3D.detach(), e_f, opac.detach(), scales.detach(),
                                rots.detach(), 1.0, e_f, rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, H, W,
                                shs.detach(), deg, rs.campos, False, False, True)[0]
    # Per-stage breakdown from an untimed pass with events around every stage; the timed region below
    # then brackets only the dominant stage's kernel (each timed event is a queue barrier).
    breakdown, dom = {}, None
    if not args.no_stage_timing:
        L.set_stage_timing(True)
        for _ in range(max(3, args.steps // 2)):
            step()
        torch.cuda.synchronize()
        breakdown = L.stage_stats()
        L.set_stage_timing(False)
        dom = max(breakdown, key=lambda k: breakdown[k][0])
        L.set_stage_timing(True, stages=[dom])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dom is not None:
        stats = L.stage_stats()
        L.set_stage_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_per_step = elapsed / args.steps * 1e3
    value = world * W * H * args.steps / elapsed / 1e6
    T = math.ceil(W / 16) * math.ceil(H / 16)
    M = (deg + 1) ** 2
    roofline = None
    stage_report = {}
    for name, (ms, calls) in breakdown.items():
        if calls <= 0 or ms <= 0:
            continue
        b = algorithmic_bytes(name, P, V, nr, W * H, T, M, 1)
        stage_report[name] = dict(ms=round(ms, 4), calls=calls, alg_GBs=round(b / (ms * 1e-3) / 1e9, 1))
    if dom is not None and stats.get(dom, (0, 0))[1] > 0:
        ms = stats[dom][0]
        ach = round(algorithmic_bytes(dom, P, V, nr, W * H, T, M, 1) / (ms * 1e-3) / 1e9, 1)
        traffic, src = pmc_traffic(dom)
        roofline = dict(bound="hbm", achieved=ach, peak=HBM_PEAK_GBS, unit="GB/s", frac=round(ach / HBM_PEAK_GBS, 4),
                        traffic=traffic, traffic_unit="bytes/launch", traffic_source=src, kernel=dom,
                        kernel_ms=round(ms, 4), launches=stats[dom][1])
        valu, _ = pmc_traffic(dom, "valu_wave_instr")
        if valu:
            rate = valu / (ms * 1e-3) / 1e9
            roofline["valu_issue"] = dict(wave_instr_per_launch=valu, achieved_Ginstr_s=round(rate, 1),
                                          peak_Ginstr_s=VALU_PEAK_GINSTR, frac=round(rate / VALU_PEAK_GINSTR, 4))
    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, ref = cpu_baseline(P, deg, W, H)
        for p in params:  # one more step on the same inputs, outputs kept for the parity check
            p.grad = None
        means2D = torch.zeros_like(means3D, requires_grad=True)
        color, _, invd = rast(means3D=means3D, means2D=means2D, opacities=opac, shs=shs, scales=scales,
                              rotations=rots)
        torch.autograd.backward([color, invd], [g_col, g_inv])
        npy = lambda t: t.detach().cpu().numpy()  # noqa: E731
        gpu = dict(color=npy(color), invdepth=npy(invd), dmean3D=npy(means3D.grad), dmean2D=npy(means2D.grad),
                   dopacity=npy(opac.grad), dscale=npy(scales.grad), drot=npy(rots.grad), dsh=npy(shs.grad))
        parity = parity_report(gpu, ref)
    if rank == 0:
        line = {
            "metric": "forward+backward Mpix/s at 1080p (1M Gaussians); grad max-abs-err vs ref",
            "value": round(value, 3), "unit": "Mpix/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded PCG64 scene and upstream gradients; no dataset)",
            "config": {"workload": f"configs[1]: {P} Gaussians, SH deg {deg}, {W}x{H}, fwd+bwd with depth, "
                                   f"one view per GPU" + ((", RCCL" if backend == "nccl" else ", " + backend) + " grad all-reduce"
                                                          if world > 1 else ""),
                       "num_rendered": nr, "visible": V, "tiles": T,
                       "parallelism": f"view-dp{world}"},
            "roofline": roofline, "cpu_baseline": cpu, "parity": parity,
            "stages": stage_report, "stages_note": "untimed pass with events around every stage",
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
