#!/usr/bin/env python3
"""Benchmark: forward+backward Mpix/s of the MI355X Gaussian-splat rasterizer at 1080p, 1M Gaussians,
SH degree 3 (BASELINE.json configs[1]), one training view per GPU.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one view rendered through the public GaussianRasterizer API (forward, including its
num_rendered host sync), full backward of fixed synthetic upstream gradients dL/dcolor and dL/dinvdepth
(fed to autograd directly: the gradient of loss = <dL/dcolor, color> + <dL/dinvdepth, invdepth>), and -- for N > 1 --
the RCCL all-reduce of every Gaussian gradient.

N = 1 measures configs[1] (1M Gaussians); the line also carries, each timed on the GPU in the same run:
  config3            configs[2]: LOD cut -> weights -> render_post lerp -> rasterize fwd+bwd -> lerp bwd on a
                     synthetic binary hierarchy over configs[1]'s 1M leaves (the example dataset is not available
                     offline), stages separately and inclusive;
  config4_one_gpu    configs[3]'s per-GPU work (4M Gaussians, one view) on one GPU, the N = 1 point of the
                     multi-GPU curve;
  config5            configs[4]: train_post.py's step (SPT cache, alt rasterizer, L1 + D-SSIM + depth L1, Adam) on a
                     synthetic 2-chunk merged hierarchy over 1M leaves, camera moving every step;
  cpu_baseline       the oracle on one full frame on all host threads (OpenMP) and on one thread;
  parity             the GPU step against the oracle on the same inputs, in the shared arithmetic contract and in
                     the reference's own float operation order.
N > 1: view-data parallel, weak scaling -- each rank renders its own view of its own replica of the same 1M-Gaussian
scene (--P overrides) and the gradients are all-reduced (RCCL over xGMI), so the per-GPU work equals the N = 1 line's
and the driver's per-N values form one weak-scaling curve.  The line then also carries config4: configs[3] (4M
Gaussians per replica, one view per GPU, the same exchange) timed on the same N ranks.
Inputs are synthetic (seeded), resident in HBM before timing starts.  Rank 0 prints one JSON line.
"""
import argparse
import json
import math
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "hierarchical-lod-gaussians_amd")
sys.path[:0] = [ROOT, PKG]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# VALU issue ceiling: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles on each SIMD-32 (across its
# waves; MI355X_MICROARCH.md cycle constants, v_fma_f32 wave64), 2400 MHz max clock = 1228.8 G wave-instr/s
VALU_PEAK_GINSTR = 256 * 4 * 2.4 / 2


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


def running_lib_sha16():
    """Hash of the libhlgs.so this process loaded (the build identity PMC profiles are matched against)."""
    import hashlib
    from hlgs_core import _lib as L
    path = getattr(L.load(), "_name", None)
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]
    except (OSError, TypeError):
        return None


def pmc_profile(name="pmc_traffic.json"):
    """The latest committed PMC summary (tools/profile_round.sh + tools/summarize_profile.py / summarize_stalls.py):
    (dict, path relative to the repo, matches) where matches says whether it was measured on the library running
    now (the hashes in its build block agree); (None, None, False) when there is none."""
    prof = os.path.join(ROOT, "profiles")
    rounds = sorted(d for d in os.listdir(prof) if os.path.exists(os.path.join(prof, d, name))) \
        if os.path.isdir(prof) else []
    if not rounds:
        return None, None, False
    path = os.path.join(prof, rounds[-1], name)
    d = json.load(open(path))
    sha = (d.get("build") or {}).get("lib_sha16")
    return d, os.path.relpath(path, ROOT), bool(sha) and sha == running_lib_sha16()


def pmc_traffic(stage, field="hbm_bytes"):
    """Per-launch HBM bytes (2 x FETCH_SIZE + WRITE_SIZE) -- or another field, e.g. valu_wave_instr -- of the
    stage's kernel from the latest committed rocprofv3 PMC profile, with its source and whether that profile is of
    the running library (None values when there is no profile)."""
    d, src, match = pmc_profile()
    if d is None or stage not in STAGE_KERNEL:
        return None, None, False
    hits = [v[field] for k, v in d["kernels"].items() if STAGE_KERNEL[stage] in k and v.get(field)]
    return (sum(hits) if hits else None), src, match


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _mem(tag):
    """A progress line per leg on stderr (so a long run is visibly alive); with HLGS_BENCH_MEM=1 also the peak and
    current host RSS (diagnostics only)."""
    print(f"[bench] {tag} ({time.strftime('%H:%M:%S')})", file=sys.stderr, flush=True)
    if os.environ.get("HLGS_BENCH_MEM"):
        import resource
        cur = int(open("/proc/self/statm").read().split()[1]) * os.sysconf("SC_PAGE_SIZE")
        print(f"[mem] {tag}: rss {cur / 2**30:.2f} GiB, peak {resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20:.2f} GiB",
              file=sys.stderr, flush=True)


def _mem_watchdog(limit_gib=40):
    """HLGS_BENCH_MEM=1: dump every thread's stack and exit if host RSS passes limit_gib (diagnostics only)."""
    import faulthandler
    import threading

    def watch():
        while True:
            time.sleep(0.05)
            cur = int(open("/proc/self/statm").read().split()[1]) * os.sysconf("SC_PAGE_SIZE")
            if cur > limit_gib * 2**30:
                print(f"[mem] RSS over {limit_gib} GiB; stacks:", file=sys.stderr, flush=True)
                faulthandler.dump_traceback(all_threads=True)
                sys.stderr.flush()
                os._exit(3)
    threading.Thread(target=watch, daemon=True).start()


def _oracle_frame(O, sc, cam, g, gd, omp=False):
    t0 = time.perf_counter()
    fr = O.forward(sc, cam, do_depth=True, omp=omp)
    gr = O.backward(fr, sc, g, gd)
    dt = time.perf_counter() - t0
    ref = dict(color=fr.color, invdepth=fr.invdepth, dmean3D=gr["dmean3D"], dmean2D=gr["dmean2D"],
               dopacity=gr["dopacity"], dscale=gr["dscale"], drot=gr["drot"], dsh=gr["dsh"], radii=fr.radii)
    return dt, ref


def cpu_baseline(P, deg, W, H, reference_order=True):
    """The oracle (C restatement of the reference algorithm) on one full frame, fwd + bwd: on every host thread
    OpenMP gives it (the box's CPU share: OMP_NUM_THREADS) and on one thread.  Returns the timing summary, the
    serial oracle's outputs (same scene, camera and upstream gradients as rank 0's GPU step) for the full-size
    parity check, and the same frame with alpha decided in the reference's own float op order."""
    from oracle import oracle as O
    from hlgs_core import synthetic as S
    cam = S.make_camera(W, H)
    sc = S.make_gaussians(P, deg, cam, seed=0)
    g, gd = S.upstream_grads(W, H, seed=1)
    O.build()
    cn = S.cam_numpy(cam)
    dt1, ref = _oracle_frame(O, sc, cn, g, gd)
    threads = O.num_threads(omp=True)
    dtn = min(_oracle_frame(O, sc, cn, g, gd, omp=True)[0] for _ in range(2))
    sample = (f"one full frame: {P} Gaussians, SH deg {deg}, {W}x{H}, forward+backward (preprocess, binning, "
              f"stable sort, blend, blend backward, Gaussian backward), {cpu_model()}, os.cpu_count()={os.cpu_count()}")
    summary = dict(value=round(W * H / dtn / 1e6, 4), unit="Mpix/s", cores=threads, kind="port",
                   sample=f"{sample}; {dtn:.2f} s on {threads} OpenMP threads (best of 2)",
                   single_thread=dict(value=round(W * H / dt1 / 1e6, 4), unit="Mpix/s", cores=1,
                                      sample=f"same frame, {dt1:.2f} s on 1 thread"))
    ref_order = None
    if reference_order:
        # the reference order twice: uncontracted, and with a*b+c contracted (the reference is built by nvcc with
        # --fmad=true); each serial, on its own thread (ctypes releases the GIL)
        ref_order = {}

        def run(key):
            with O.reference_order(omp=key):
                ref_order[key] = _oracle_frame(O, sc, cn, g, gd, omp=key)[1]
        th = [threading.Thread(target=run, args=(k,)) for k in (False, "fma")]
        for t in th:
            t.start()
        for t in th:
            t.join()
    return summary, ref, ref_order


def rotated_parity(P, deg, W, H, dev, cam_index=5):
    """configs[1]'s workload (P Gaussians, SH deg, W x H, inverse depth) seen through one of the reference's own
    cameras (cameras.json entry in tests/golden/golden_realcam.npz: rotated view matrix, fx != fy, kept at its own FoV
    at W x H), GPU step against the serial oracle: the full-size check of computeCov2D's T = W J and the mean gradient
    through the view matrix (forward.cu:141-176, backward.cu:285-312, 433-447)."""
    from diff_gaussian_rasterization import GaussianRasterizer
    from hlgs_core import synthetic as S
    from oracle import oracle as O
    entry = S.load_real_cameras()[cam_index]
    cam = S.real_camera(entry, W=W, H=H)
    host = S.make_gaussians(P, deg, cam, seed=0)
    g, gd = S.upstream_grads(W, H, seed=1)
    to = lambda a: torch.tensor(a, device=dev, requires_grad=True)  # noqa: E731
    means3D, scales, rots, opac, shs = (to(host[k]) for k in ("means3D", "scales", "rotations", "opacities", "shs"))
    means2D = torch.zeros_like(means3D, requires_grad=True)
    color, radii, invd = GaussianRasterizer(settings_for(cam, deg, dev))(
        means3D=means3D, means2D=means2D, opacities=opac, shs=shs, scales=scales, rotations=rots)
    torch.autograd.backward([color, invd], [torch.tensor(g, device=dev), torch.tensor(gd, device=dev)])
    npy = lambda t: t.detach().cpu().numpy()  # noqa: E731
    gpu = dict(color=npy(color), invdepth=npy(invd), dmean3D=npy(means3D.grad), dmean2D=npy(means2D.grad),
               dopacity=npy(opac.grad), dscale=npy(scales.grad), dsh=npy(shs.grad), drot=npy(rots.grad))
    gpu_radii = npy(radii)
    del means3D, scales, rots, opac, shs, means2D, color, radii, invd
    sc = {k: host[k] for k in ("means3D", "scales", "rotations", "opacities", "shs")}
    sc["sh_degree"] = deg
    _, ref = _oracle_frame(O, sc, S.cam_numpy(cam), g, gd)
    rep = parity_report(gpu, ref, f"oracle, same inputs, configs[1] workload through the reference's camera "
                                  f"cameras.json id {entry['id']} ({entry['width']}x{entry['height']}, fx {entry['fx']:.2f}, "
                                  f"fy {entry['fy']:.2f}) kept at its FoV at {W}x{H}")
    rep["radii_equal"] = bool(np.array_equal(gpu_radii, ref["radii"]))
    return rep


def parity_report(gpu, ref, vs):
    """Full-size parity of rank 0's step against an oracle frame: forward per-pixel L-inf and the count of pixels
    above the 1e-4 tolerance; per gradient tensor, max-abs error, max-abs error relative to the oracle tensor's
    max-abs, and the elements violating |gpu - ref| <= 1e-3 |ref| + 1e-6 max|ref| (element-wise)."""
    out = dict(vs=vs)
    dc = np.abs(gpu["color"] - ref["color"])
    di = np.abs(gpu["invdepth"] - ref["invdepth"])
    out["color_linf"] = float(dc.max())
    out["invdepth_linf"] = float(di.max())
    out["pixels_above_1e-4"] = int((np.maximum(dc.max(0), di.max(0)) > 1e-4).sum())
    per = {}
    for k in ("dmean3D", "dmean2D", "dopacity", "dscale", "drot", "dsh"):
        a, b = gpu[k].reshape(ref[k].shape[0], -1), ref[k].reshape(ref[k].shape[0], -1)
        a = a[:, :b.shape[1]]
        d = np.abs(a - b)
        mx = max(float(np.abs(b).max()), 1e-30)
        err = float(d.max())
        per[k] = dict(max_abs_err=err, rel=err / mx,
                      elementwise_violations=int((d > 1e-3 * np.abs(b) + 1e-6 * mx).sum()))
    out["grad_max_abs_err"] = max(v["max_abs_err"] for v in per.values())
    out["grad_max_rel_err"] = max(v["rel"] for v in per.values())
    out["grad_elementwise_violations"] = sum(v["elementwise_violations"] for v in per.values())
    out["grads"] = per
    out["tolerance"] = dict(fwd_linf=1e-4, grad_rel=1e-3, grad_elementwise="|d| <= 1e-3 |ref| + 1e-6 max|ref|")
    return out


def _median_ms(fn, iters, warmup=2):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def settings_for(cam, deg, dev, do_depth=True):
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    e_i = torch.empty(0, dtype=torch.int32, device=dev)
    e_f = torch.empty(0, dtype=torch.float32, device=dev)
    return GaussianRasterizationSettings(
        image_height=cam["H"], image_width=cam["W"], tanfovx=cam["tanfovx"], tanfovy=cam["tanfovy"],
        bg=torch.zeros(3, device=dev), scale_modifier=1.0, viewmatrix=cam["viewmatrix"].to(dev),
        projmatrix=cam["projmatrix"].to(dev), sh_degree=deg, campos=cam["campos"].to(dev), prefiltered=False,
        debug=False, render_indices=e_i, parent_indices=e_i, interpolation_weights=e_f, num_node_kids=e_i,
        do_depth=do_depth)


def bench_config3(P, deg, W, H, dev, iters=20, tau_px=6.0):
    """configs[2]: the hierarchical-LOD training step of train_single.py / render_post
    (gaussian_renderer/__init__.py:304-347): expand_to_size_dynamic at tau -> get_interpolation_weights_dynamic
    -> the child/parent lerp (interpolate_lod) -> rasterize forward + backward at W x H -> lerp backward, on a
    synthetic binary hierarchy over P leaves (hlgs_core.synthetic.make_dynamic_hierarchy).  Median event spans
    on torch's stream; the cut and interpolation separately and the whole chain inclusive."""
    import gaussian_hierarchy as GH
    from diff_gaussian_rasterization import GaussianRasterizer
    from hlgs_core import synthetic as S
    cam = S.make_camera(W, H)
    t0 = time.perf_counter()
    hier = S.make_dynamic_hierarchy(S.make_gaussians(P, deg, cam, seed=0), seed=0)
    build_s = time.perf_counter() - t0
    _mem("config3 hierarchy built")
    N = hier["nodes"].shape[0]
    d = lambda a, **kw: torch.tensor(np.ascontiguousarray(a), device=dev, **kw)  # noqa: E731
    nodes = d(hier["nodes"])
    xyz, scales, rots, opac, shs = (d(hier[k], requires_grad=True)
                                    for k in ("means3D", "scales", "rotations", "opacities", "shs"))
    tau = (2 * (tau_px + 0.5)) * cam["tanfovx"] / (0.5 * W)
    vp, vd = cam["campos"].to(dev), torch.tensor([0.0, 0.0, 1.0])
    ri, pi, ni, kids = (torch.zeros(N, dtype=torch.int32, device=dev) for _ in range(4))
    ts = torch.zeros(N, device=dev)
    rast = GaussianRasterizer(settings_for(cam, deg, dev))
    g_np, gd_np = S.upstream_grads(W, H, seed=1)
    g, gd = torch.tensor(g_np, device=dev), torch.tensor(gd_np, device=dev)
    st = {}

    def cut():
        st["n"] = GH.expand_to_size_dynamic(nodes, xyz.detach(), scales.detach(), tau, vp, vd, ri, pi, ni)

    def weights():
        GH.get_interpolation_weights_dynamic(ni[:st["n"]], tau, nodes, xyz.detach(), scales.detach(), vp.cpu(), vd,
                                             ts, kids)

    def lerp():
        st["outs"] = GH.interpolate_lod(xyz, scales, rots, opac, shs, ri[:st["n"]], pi, ts, 0)

    def raster():
        m, s_, r_, o_, sh_ = st["outs"]
        m2 = torch.zeros_like(m, requires_grad=True)
        st["graph"] = rast(means3D=m, means2D=m2, opacities=o_, shs=sh_, scales=s_, rotations=r_)

    def backward():
        c, _, inv = st["graph"]
        torch.autograd.backward([c, inv], [g, gd])
        for p in (xyz, scales, rots, opac, shs):
            p.grad = None

    def full():
        cut(); weights(); lerp(); raster(); backward()  # noqa: E702

    def lerp_raster_bwd():
        lerp(); raster(); backward()  # noqa: E702

    full()
    _mem("config3 first chain")
    stages = {"expand_to_size_dynamic": _median_ms(cut, iters),
              "get_interpolation_weights_dynamic": _median_ms(weights, iters),
              "interpolate_lod_fwd": _median_ms(lerp, iters),
              "rasterizer_fwd": _median_ms(raster, iters)}
    stages["rasterizer_bwd+lerp_bwd"] = (_median_ms(lerp_raster_bwd, iters) - stages["interpolate_lod_fwd"]
                                         - stages["rasterizer_fwd"])
    incl = _median_ms(full, iters)
    lod = sum(stages[k] for k in ("expand_to_size_dynamic", "get_interpolation_weights_dynamic",
                                  "interpolate_lod_fwd"))
    return dict(workload=f"configs[2]: synthetic binary hierarchy over {P} leaves ({N} nodes), SH deg {deg}, "
                         f"{W}x{H}, tau={tau_px} px ({tau:.3e}), cut -> weights -> lerp -> rasterize fwd+bwd -> "
                         f"lerp bwd", nodes=N, selected=int(st["n"]), hierarchy_build_s=round(build_s, 1),
                stages_ms={k: round(v, 4) for k, v in stages.items()}, lod_cut_and_interp_ms=round(lod, 4),
                inclusive_ms=round(incl, 4), value=round(W * H / incl / 1e3, 1), unit="Mpix/s",
                timing=f"median of {iters} event spans per stage on torch's stream")


EXCHANGE = os.environ.get("HLGS_EXCHANGE", "factored")  # "plain": every gradient all-reduced (the A/B reference)


def make_exchange(params, means, sh, dc=None):
    """The view-DP gradient exchange of the N > 1 legs: colour-factored SH gradients by default (hlgs_core.dp: the SH
    leaves are exchanged as 3-float colour gradients, all-gathered, and rebuilt on every rank); HLGS_EXCHANGE=plain
    all-reduces every gradient, with the SH backward overlapping the early collective (the rasterizer is the only
    consumer of means3D / shs in these steps)."""
    from hlgs_core.dp import FlatGradExchange
    if EXCHANGE == "plain":
        return FlatGradExchange(params, overlap=True)
    return FlatGradExchange(params, colour_factor=dict(means=means, sh=sh, dc=dc))


def exchange_fields(ex, world, ms):
    """bytes and achieved per-GPU link rate of one exchange (ms: its measured time)."""
    ar, ag, link = ex.link_bytes(world)
    return dict(mode=EXCHANGE, allreduce_bytes=ar, allgather_bytes_per_rank=ag, link_bytes_per_gpu=link,
                link_GBs=round(link / (ms * 1e-3) / 1e9, 1) if ms > 0 else None)


def make_step(P, deg, W, H, dev, rank, world, exchange_on=True):
    """One rank's training view: its scene replica, rasterizer and upstream gradients; returns step() and state."""
    from diff_gaussian_rasterization import GaussianRasterizer
    from hlgs_core import synthetic as S
    from hlgs_core.dp import FlatGradExchange
    # every rank: the same scene replica, its own view (ring of cameras); rank 0 = configs[1] camera
    cam = S.make_camera(W, H) if world == 1 else S.ring_camera(W, H, rank, world)
    host = S.make_gaussians(P, deg, S.make_camera(W, H), seed=0)
    to = lambda a: torch.tensor(a, device=dev, requires_grad=True)  # noqa: E731
    params = [to(host[k]) for k in ("means3D", "scales", "rotations", "opacities", "shs")]
    del host
    means3D, scales, rots, opac, shs = params
    g_np, gd_np = S.upstream_grads(W, H, seed=1 + rank)
    g_col, g_inv = torch.tensor(g_np, device=dev), torch.tensor(gd_np, device=dev)
    rs = settings_for(cam, deg, dev)
    rast = GaussianRasterizer(rs)
    exchange = make_exchange(params, means3D, shs) if (world > 1 and exchange_on) else None
    st = dict(params=params, rs=rs, rast=rast, exchange=exchange, g_col=g_col, g_inv=g_inv, ar_events=[])

    def step(time_exchange=False):
        for p in params:
            p.grad = None
        means2D = torch.zeros_like(means3D, requires_grad=True)
        color, radii, invd = rast(means3D=means3D, means2D=means2D, opacities=opac, shs=shs, scales=scales,
                                  rotations=rots)
        torch.autograd.backward([color, invd], [g_col, g_inv])
        if exchange is not None:
            if time_exchange:
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                exchange.allreduce()
                b.record()
                st["ar_events"].append((a, b))
            else:
                exchange.allreduce()
        st["means2D"], st["color"], st["invd"] = means2D, color, invd
        return radii

    return step, st


def num_rendered(st, H, W, deg):
    from diff_gaussian_rasterization import _C as DC
    rs = st["rs"]
    means3D, scales, rots, opac, shs = (p.detach() for p in st["params"])
    e_i, e_f = rs.render_indices, rs.interpolation_weights
    return int(DC.rasterize_gaussians(rs.bg, e_i, e_i, e_f, e_i, means3D, e_f, opac, scales, rots, 1.0, e_f,
                                      rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, H, W, shs, deg,
                                      rs.campos, False, False, True)[0])


def bench_config4_one_gpu(P, deg, W, H, dev, steps, warmup):
    """configs[3]'s per-GPU work (P Gaussians, one 1080p view, fwd+bwd) on one GPU with no exchange: the N = 1
    point against which the driver's N > 1 lines (same per-rank work plus the all-reduce) scale."""
    step, st = make_step(P, deg, W, H, dev, 0, 1)
    _mem("config4 scene")
    for _ in range(warmup):
        step()
        _mem("config4 warmup step")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    out = dict(workload=f"configs[3] per-GPU work on one GPU: {P} Gaussians, SH deg {deg}, {W}x{H}, fwd+bwd with "
                        f"depth, one view, no exchange", value=round(W * H * steps / el / 1e6, 3), unit="Mpix/s",
               ms_per_step=round(el / steps * 1e3, 4), steps=steps, num_rendered=num_rendered(st, H, W, deg))
    del step, st
    torch.cuda.empty_cache()
    return out


def merged_two_chunk_scene(P, seed=0):
    """configs[4]'s scene: two chunks of P/2 leaves each (the second shifted 4 units right and 6 deeper), merged
    under one root (hlgs_core.synthetic.make_merged_hierarchy, after mainHierarchyMerger.cpp:94-140), the SPT
    structures of build_hierarchical_spt (train_post.py's setup) and the host parameter storage of a cached run."""
    from hlgs_core import spt
    from hlgs_core import synthetic as S
    cam = S.make_camera(1920, 1080)
    c0 = S.make_gaussians(P // 2, 3, cam, seed=seed + 1)
    c1 = S.make_gaussians(P - P // 2, 3, cam, seed=seed + 2)
    c1["means3D"] = c1["means3D"] + np.array([4.0, 0.0, 6.0], np.float32)
    h = S.make_merged_hierarchy([c0, c1], np.array([[0, 0, 12], [4, 0, 18]], np.float32), seed=seed)
    nodes = torch.tensor(h["nodes"])
    xyz = torch.tensor(h["means3D"])
    log_s = torch.log(torch.tensor(h["scales"]))
    t0 = time.perf_counter()
    b = spt.build_hierarchical_spt(nodes, xyz, log_s, 0, 0.5, 0.00228, 256)
    build_s = time.perf_counter() - t0
    shs = torch.tensor(h["shs"])
    op = torch.tensor(h["opacities"]).reshape(-1, 1).clamp(1e-4, 1 - 1e-4)
    storage = dict(xyz=xyz, f_dc=shs[:, :1].contiguous(), f_rest=shs[:, 1:].contiguous(),
                   opacity=torch.log(op / (1 - op)), scaling=log_s, rotation=torch.tensor(h["rotations"]))
    return b, storage, build_s, int(nodes.shape[0])


def bench_config5(P, dev, steps=20, sh_degree=1, depth=True, W=1920, H=1080, rank=0, world=1, backend=None):
    """configs[4]: train_post.py's training step on a 2-chunk merged hierarchy (synthetic: the example dataset is
    not available offline), per iteration as train_post.py:323-812 orders it: SPTCache.step (coarse cut, cache
    bookkeeping, SPT cut, write-back / load through pinned host storage) -> activations -> alt rasterizer
    (antialiasing, active SH degree 1) -> L1 + D-SSIM (+ masked inverse-depth L1, train_single.py:111-118) ->
    backward -> dense Adam.  The activations (sigmoid opacity, exp scale, normalised rotation) run as one HIP pass
    each way (hlgs_core.activations).  The camera moves every step.  Median host-clock step and per-stage event medians.

    world > 1: view-data parallel, one view per rank.  Each step the ranks gather every rank's view
    (gather_views), every rank's SPTCache.step computes the union cut of the batch, so all replicas hold the same
    resident set; each rank renders its own view, the gradients of SPTCache.params are all-reduced (RCCL, averaged;
    the rasterizer backward writes them straight into the exchange's flat buffer) and the dense Adam runs replicated.
    Barrier + synchronise around the timed steps, max over ranks; all-reduce time and bus bandwidth reported."""
    from alt_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from hlgs_core import synthetic as S
    from hlgs_core.activations import activate
    from hlgs_core.loss import photometric_loss
    from hlgs_core.spt_cache import NAMES, SPTCache, gather_views
    b, storage, build_s, G = merged_two_chunk_scene(P)
    _mem("config5 scene")
    cache = SPTCache(storage, b, 0, reuse_tolerance=0.9, device=dev)
    rng = np.random.default_rng(1 + rank)
    gt = torch.tensor(rng.uniform(0, 1, (3, H, W)).astype(np.float32), device=dev)
    mono = torch.tensor(rng.uniform(0.05, 0.5, (1, H, W)).astype(np.float32), device=dev)
    mask = torch.ones((1, H, W), device=dev)
    bg = torch.zeros(3, device=dev)
    lrs = dict(xyz=1.6e-4, f_dc=2.5e-3, f_rest=2.5e-3 / 20, opacity=5e-2, scaling=5e-3, rotation=1e-3)
    # rank r's camera path is offset sideways: the views of one step differ
    path = [S.make_camera(W, H, T=np.array([0.03 * k + 0.4 * rank, 0.01 * k, 0.2 * math.sin(0.3 * k)]))
            for k in range(steps + 3)]
    # camera tensors live on the GPU, as the reference's Camera objects do (scene/cameras.py:102-107 .cuda())
    path = [{k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in c.items()} for c in path]
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    stages = {k: [] for k in ("cache", "forward", "loss", "backward", "allreduce", "adam")}
    step_ms, resident, nbytes = [], [], []
    t_loop = None
    for it, cam in enumerate(path):
        if world > 1 and it == 3:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if it == 3:
            t_loop = t0
        e = [ev() for _ in range(7)]
        e[0].record()
        trace = os.environ.get("HLGS_BENCH_TRACE")
        if trace:
            print(f"[config5 r{rank}] step {it}", file=sys.stderr, flush=True)
        if world > 1:
            fpts, cams = gather_views(cam["projmatrix"], cam["campos"])
            cache.step(fpts, cams)
        else:
            cache.step(cam["projmatrix"], cam["campos"])
        e[1].record()
        p = cache.params
        if trace:
            print(f"[config5 r{rank}] resident {cache.render_indices.numel()}", file=sys.stderr, flush=True)
        ex = make_exchange([p[k] for k in NAMES], p["xyz"], p["f_rest"], p["f_dc"]) if world > 1 else None
        s = GaussianRasterizationSettings(image_height=H, image_width=W, tanfovx=cam["tanfovx"],
                                          tanfovy=cam["tanfovy"], bg=bg, scale_modifier=1.0,
                                          viewmatrix=cam["viewmatrix"].to(dev), projmatrix=cam["projmatrix"].to(dev),
                                          sh_degree=sh_degree, campos=cam["campos"].to(dev), prefiltered=False,
                                          debug=False, antialiasing=True)
        means2D = torch.zeros_like(p["xyz"], requires_grad=True)
        # get_opacity / get_scaling / get_rotation (sigmoid, exp, normalize) of every resident row in one HIP pass
        opac, scales, rots = activate(p["opacity"], p["scaling"], p["rotation"])
        img, radii, invd = GaussianRasterizer(s)(
            means3D=p["xyz"], means2D=means2D, dc=p["f_dc"], shs=p["f_rest"], opacities=opac, scales=scales,
            rotations=rots)
        e[2].record()
        # the renderer's rendered_image.clamp(0, 1) folded into the loss kernels (clamp_image)
        loss = (photometric_loss(img, gt, 0.2, invd, mono, mask, 0.5, clamp_image=True) if depth else
                photometric_loss(img, gt, 0.2, clamp_image=True))[0]
        e[3].record()
        # the cache's write-back crosses the host link beside the backward (its blend kernel is VALU-bound) instead of
        # beside the next step's bookkeeping
        cache.flush_write_back()
        loss.backward()
        e[4].record()
        if ex is not None:
            if trace:
                print(f"[config5 r{rank}] allreduce {ex.flat.numel()}", file=sys.stderr, flush=True)
            ex.allreduce()
            nbytes.append(ex.link_bytes(world))
            ex.close()
        e[5].record()
        cache.optimizer_step(it, lrs)
        e[6].record()
        torch.cuda.synchronize()
        if it >= 3:
            step_ms.append((time.perf_counter() - t0) * 1e3)
            for k, (a, bb) in zip(stages, zip(e[:-1], e[1:])):
                stages[k].append(a.elapsed_time(bb))
            resident.append(cache.render_indices.numel())
        for q in p.values():
            q.grad = None
    el = time.perf_counter() - t_loop
    if world > 1:
        torch.cuda.synchronize()
        dist.barrier()
        el = time.perf_counter() - t_loop
        ar = float(np.mean(stages["allreduce"]))
        t = torch.tensor([el, ar], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, ar = float(t[0].item()), float(t[1].item())
    ms = float(np.median(step_ms)) if world == 1 else el / len(step_ms) * 1e3
    out = dict(workload=f"configs[4]: train_post.py step with the SPT cache on a 2-chunk merged hierarchy ({G} "
                        f"nodes over {P} leaves), {W}x{H}, alt rasterizer (antialiasing, SH degree {sh_degree}), "
                        f"L1 + D-SSIM{' + depth L1' if depth else ''}, dense Adam, camera moving every step" +
                        ("" if world == 1 else f"; view-data parallel over {world} ranks: union cut of the gathered "
                                               f"views, {'RCCL' if backend == 'nccl' else backend} all-reduce of the "
                                               f"resident gradients, replicated Adam"),
               spt_build_s=round(build_s, 3), resident_median=int(np.median(resident)), ms_per_step=round(ms, 3),
               value=round(world * W * H / ms / 1e3, 1), unit="Mpix/s", steps=len(step_ms), n_gpus=world,
               stages_ms={k: round(float(np.median(v)), 3) for k, v in stages.items() if world > 1 or k != "allreduce"},
               timing=("median host clock around a synchronised step; stages: median event spans on torch's stream"
                       if world == 1 else "barrier + synchronise around the timed steps, max over ranks; stages: "
                                          "median event spans on torch's stream"))
    if world > 1:
        ar_b, ag_b, link = (int(np.median([x[i] for x in nbytes])) for i in range(3))
        out.update(exchange_ms=round(ar, 4), exchange=dict(
            mode=EXCHANGE, allreduce_bytes=ar_b, allgather_bytes_per_rank=ag_b, link_bytes_per_gpu=link,
            link_GBs=round(link / (ar * 1e-3) / 1e9, 1) if ar > 0 else None))
    del cache
    torch.cuda.empty_cache()
    return out


def bench_config4_dp(P, deg, W, H, dev, rank, world, steps, warmup, backend):
    """configs[3] on the launched ranks: P Gaussians per replica, one 1080p view per GPU, fwd+bwd, RCCL all-reduce of
    every gradient; barrier + synchronise around the timed steps, the max over ranks."""
    step, st = make_step(P, deg, W, H, dev, rank, world)
    for _ in range(warmup):
        step()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(time_exchange=True)
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    ar_ms = float(np.mean([a.elapsed_time(b) for a, b in st["ar_events"]]))
    t = torch.tensor([el, ar_ms], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el, ar_ms = float(t[0].item()), float(t[1].item())
    out = dict(workload=f"configs[3]: {P} Gaussians per replica, SH deg {deg}, {W}x{H}, fwd+bwd with depth, one view "
                        f"per GPU, {'RCCL' if backend == 'nccl' else backend} gradient exchange ({EXCHANGE})",
               value=round(world * W * H * steps / el / 1e6, 3), unit="Mpix/s", n_gpus=world,
               ms_per_step=round(el / steps * 1e3, 4), steps=steps, exchange_ms=round(ar_ms, 4),
               exchange=exchange_fields(st["exchange"], world, ar_ms),
               timing="barrier + synchronise around the timed steps, max over ranks; exchange: events around "
                      "FlatGradExchange.allreduce() (mean, max over ranks)")
    st["exchange"].close()
    del step, st
    torch.cuda.empty_cache()
    return out


def launch_ranks(n):
    """`bench.py --gpus N` run without a launcher: the same command under torch.distributed.run with N ranks on this
    node (rendezvous on 127.0.0.1, a free port), as a child process -- never an exec, and before any GPU call in this
    process.  Returns the child's exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] --gpus {n} without WORLD_SIZE: launching {n} ranks", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def dry_run(world, rank, backend, args):
    """--dry-run: join the process group (when world > 1), agree on the world size with one collective, and have
    rank 0 print the line's rank fields; no GPU work (the CPU test of the launch path, tests/test_bench_cpu.py)."""
    seen = world
    if world > 1:
        dist.init_process_group(backend)
        t = torch.ones(1)
        dist.all_reduce(t)
        seen = int(t.item())
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_joined": seen, "gpus_arg": args.gpus,
                          "backend": backend if world > 1 else None}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--P", type=int, default=None, help="Gaussians per replica (default 1M, configs[1])")
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--sh-degree", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stage-timing", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the config3, config4_one_gpu and config5 legs")
    ap.add_argument("--settle-max", type=int, default=200,
                    help="at most this many untimed steps before the timed ones, until the step time stops falling "
                         "(the core clock's ramp under load); 0: none")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch and join the ranks, print the line's rank fields, run no GPU work (launcher test)")
    args = ap.parse_args()
    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus must be >= 1 (got {args.gpus})")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # --gpus N without a launcher: start N ranks as a child process (before anything touches the GPU) and exit
        # with its code, so the command cannot silently measure one rank
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per GPU "
                 f"(torch.distributed.run --nproc-per-node {args.gpus}) or pass --gpus {world}")
    if os.environ.get("HLGS_BENCH_MEM"):
        _mem_watchdog()

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # HLGS_DIST_BACKEND=gloo with more ranks than GPUs rehearses the multi-rank path on a one-GPU box (ranks share
    # the card); the driver's N-GPU runs use the default, RCCL ("nccl"), one rank per GPU.
    backend = os.environ.get("HLGS_DIST_BACKEND", "nccl")
    if args.dry_run:
        return dry_run(world, rank, backend, args)
    gpu = local % max(1, torch.cuda.device_count()) if world > 1 else 0
    if world > 1:
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", gpu)

    from hlgs_core import _lib as L

    W, H, deg = args.W, args.H, args.sh_degree
    P = args.P if args.P is not None else 1_000_000
    step, st = make_step(P, deg, W, H, dev, rank, world)
    params, exchange = st["params"], st["exchange"]

    for _ in range(args.warmup):
        radii = step()
    torch.cuda.synchronize()
    # frame statistics for the algorithmic-byte model
    with torch.no_grad():
        V = int((radii > 0).sum().item())
    nr = num_rendered(st, H, W, deg)
    # Per-stage breakdown from an untimed pass with events around every stage; the timed region below
    # then brackets only the dominant stage's kernel (each timed event is a queue barrier).
    breakdown, dom, stats = {}, None, {}
    n_stage = 0
    if not args.no_stage_timing:
        L.set_stage_timing(True)
        n_stage = max(3, args.steps // 2)
        for _ in range(n_stage):
            step()
        torch.cuda.synchronize()
        breakdown = L.stage_stats()
        L.set_stage_timing(False)
        dom = max(breakdown, key=lambda k: breakdown[k][0])
    # Clock settle: the compute-bound kernels (both blends, the tile sort) run ~8% faster after ~50 back-to-back steps
    # than in the first ones, while the HBM-bound ones do not change (the core clock ramps under sustained load;
    # profiles/r04/timing.json), so the timed steps start from the clock a training run holds: untimed blocks of 10
    # steps, at least 50, until two blocks in a row are no faster than the best one by 0.5%, at most args.settle_max.
    settle = 0
    settle_blocks = []  # ms per step of each untimed settle block: the clock ramp the settle phase waits out
    if args.settle_max > 0:
        best, flat = None, 0
        while settle < args.settle_max:
            torch.cuda.synchronize()
            tb = time.perf_counter()
            for _ in range(10):
                step()
            torch.cuda.synchronize()
            dt = time.perf_counter() - tb
            settle_blocks.append(dt / 10 * 1e3)
            settle += 10
            flat = flat + 1 if best is not None and dt > best * 0.995 else 0
            best = dt if best is None else min(best, dt)
            if settle >= 50 and flat >= 2:
                break
    # The dominant kernel is timed with HIP events on its own stream in the last K_EV timed steps only: each event
    # is a queue barrier (~6 us of idle GPU apiece at config #2), which the other steps then do not pay.
    K_EV = min(args.steps, 5)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if dom is not None and i == args.steps - K_EV:
            L.set_stage_timing(True, stages=[dom])
        step(time_exchange=exchange is not None)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dom is not None:
        stats = L.stage_stats()
        L.set_stage_timing(False)
    exchange_report = None
    if world > 1:
        ar_ms = float(np.mean([a.elapsed_time(b) for a, b in st["ar_events"]])) if st["ar_events"] else 0.0
        t = torch.tensor([elapsed, ar_ms], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, ar_ms = float(t[0].item()), float(t[1].item())
        exchange_report = dict(
            collective=(f"all_reduce {'AVG' if backend == 'nccl' else 'SUM + 1/N scale'}" +
                        (" + all_gather of the colour-gradient rows" if EXCHANGE != "plain" else "") + f", {backend}"),
            collectives_per_step=getattr(exchange, "last_collectives", None), exchange_ms=round(ar_ms, 4),
            **exchange_fields(exchange, world, ar_ms),
            note="events around FlatGradExchange.allreduce() on torch's stream in each timed step (mean; max over "
                 "ranks), the SH rebuild included; link bytes per GPU = 2(N-1)/N x all-reduced bytes + (N-1) x gathered "
                 "row bytes")

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
        traffic, src, fresh = pmc_traffic(dom) if P == 1_000_000 else (None, None, False)
        # counter traffic is attached only when the committed PMC profile was measured on the library running now
        roofline = dict(bound="hbm", achieved=ach, peak=HBM_PEAK_GBS, unit="GB/s", frac=round(ach / HBM_PEAK_GBS, 4),
                        traffic=traffic if fresh else None, traffic_unit="bytes/launch", traffic_source=src,
                        kernel=dom, kernel_ms=round(ms, 4), launches=stats[dom][1], lib_sha16=running_lib_sha16(),
                        timing=f"HIP events around each launch on its stream, last {K_EV} of the {args.steps} timed steps")
        if traffic and not fresh:
            roofline["traffic_stale"] = dict(bytes_per_launch=traffic, note=f"{src} was measured on another build "
                                                                             "of libhlgs.so; not attached")
        valu, _, vfresh = pmc_traffic(dom, "valu_wave_instr") if P == 1_000_000 else (None, None, False)
        if valu and vfresh:
            rate = valu / (ms * 1e-3) / 1e9
            roofline["valu_issue"] = dict(wave_instr_per_launch=valu, achieved_Ginstr_s=round(rate, 1),
                                          peak_Ginstr_s=VALU_PEAK_GINSTR, frac=round(rate / VALU_PEAK_GINSTR, 4))
            stalls, _, sfresh = pmc_profile("stalls.json")
            clk = [v.get("clock_GHz") for k, v in (stalls or {}).get("kernels", {}).items()
                   if STAGE_KERNEL[dom] in k and v.get("clock_GHz")] if sfresh else []
            if clk:  # the same rate against the ceiling at the clock the PMC pass measured for this kernel
                peak_m = 256 * 4 * clk[0] / 2
                roofline["valu_issue"].update(measured_clock_GHz=clk[0], peak_at_measured_clock_Ginstr_s=round(peak_m, 1),
                                              frac_at_measured_clock=round(rate / peak_m, 4))
    cpu = parity = config3 = config4 = config5 = None
    _mem("main step")
    if rank == 0 and world == 1 and not args.no_extras:
        config3 = bench_config3(1_000_000 if args.P is None else P, deg, W, H, dev)
        torch.cuda.empty_cache()
        _mem("config3")
        config4 = bench_config4_one_gpu(4_000_000, deg, W, H, dev, max(5, args.steps // 2), 2)
        _mem("config4")
        config5 = bench_config5(1_000_000, dev)
        _mem("config5")
    if world > 1 and not args.no_extras:
        if not os.environ.get("HLGS_BENCH_SKIP_CONFIG4"):  # rehearsals over gloo skip the 944 MB exchange
            config4 = bench_config4_dp(4_000_000, deg, W, H, dev, rank, world, max(5, args.steps // 2), 2, backend)
            _mem("config4 view-dp")
        config5 = bench_config5(int(os.environ.get("HLGS_BENCH_CONFIG5_P", "1000000")), dev, rank=rank, world=world,
                                backend=backend,
                                steps=int(os.environ.get("HLGS_BENCH_CONFIG5_STEPS", "20")))
        _mem("config5 view-dp")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, ref, ref_order = cpu_baseline(P, deg, W, H)
        step()  # one more step on the same inputs, outputs kept for the parity check
        npy = lambda t: t.detach().cpu().numpy()  # noqa: E731
        means3D, scales, rots, opac, shs = params
        gpu = dict(color=npy(st["color"]), invdepth=npy(st["invd"]), dmean3D=npy(means3D.grad),
                   dmean2D=npy(st["means2D"].grad), dopacity=npy(opac.grad), dscale=npy(scales.grad),
                   dsh=npy(shs.grad), drot=npy(rots.grad))
        parity = parity_report(gpu, ref, "oracle (C restatement of the reference; alpha decided in the shared "
                                         "arithmetic contract, A-17), identical inputs, full configs[1] frame")
        parity["reference_order"] = parity_report(
            gpu, ref_order[False], "oracle with alpha decided in the reference's own float op order (power, expf, "
                                   "alpha < 1/255; forward.cu:538-560, backward.cu:614-643), no contraction, same frame")
        parity["reference_order_fma"] = parity_report(
            gpu, ref_order["fma"], "the same reference-order oracle built with a*b+c contracted (nvcc's default "
                                   "--fmad=true; hierarchy-rasterizer/setup.py:31), same frame")
        parity["reference_variance"] = parity_report(
            ref_order["fma"], ref_order[False], "the reference order's own build-to-build variance: contracted vs "
                                                "uncontracted oracle, same frame (no GPU involved)")
        _mem("parity")
        parity["reference_camera"] = rotated_parity(P, deg, W, H, dev)
        _mem("parity, reference camera")
    if rank == 0:
        wl = (f"configs[1]: {P} Gaussians, SH deg {deg}, {W}x{H}, fwd+bwd with depth, one view" if world == 1 else
              f"configs[1] per GPU, view-data parallel: {P} Gaussians per replica, SH deg {deg}, {W}x{H}, fwd+bwd "
              f"with depth, one view per GPU, " + ("RCCL" if backend == "nccl" else backend) + " grad all-reduce")
        line = {
            "metric": "forward+backward Mpix/s at 1080p (1M Gaussians); grad max-abs-err vs ref",
            "value": round(value, 3), "unit": "Mpix/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            # every untimed step before the timed ones: warm-up, the stage-timing pass and the clock settle (launch_plan)
            "untimed_steps": args.warmup + n_stage + settle,
            "clock": ("sustained: the timed steps follow untimed ones until the step time stops falling (the core "
                      "clock's ramp under load); settle_ms_per_step is each untimed settle block's time, so the first "
                      "against the last shows what the settle phase changed"),
            "settle_ms_per_step": [round(x, 4) for x in settle_blocks],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded PCG64 scene and upstream gradients; no dataset)",
            "config": {"workload": wl, "num_rendered": nr, "visible": V, "tiles": T,
                       "parallelism": f"view-dp{world}"},
            "roofline": roofline, "cpu_baseline": cpu, "parity": parity, "exchange": exchange_report,
            "config3": config3, ("config4_one_gpu" if world == 1 else "config4"): config4, "config5": config5,
            "stages": stage_report, "stages_note": "untimed pass with events around every stage",
            # steps in launch order (one launch of each rasterizer kernel per step), so a kernel trace of this run can be
            # cut into its phases (tools/summarize_profile.py timing.json): warm-up, the stage-timing pass, the timed
            # steps (the last `evented` of them bracket the dominant kernel with HIP events)
            "launch_plan": dict(warmup=args.warmup, stage_timing=n_stage, settle=settle, timed=args.steps, evented=K_EV),
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
