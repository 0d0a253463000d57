"""Per-level clocks of k_upper_cut on bench.py's config5 scene (round 2-4 diagnostic: needs stream.hip with the
HLGS_CUT_CLOCKS timer block, which round 5 removed from the product source -- `git show c236d54:hierarchical-lod-gaussians_amd/csrc/stream.hip`,
built with tools/build_variant.py CUTCLK <that file> stream.hip after adding -DHLGS_CUT_CLOCKS; HLGS_LIBRARY=.../CUTCLK.so)."""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
import numpy as np, torch
import bench
from hlgs_core import synthetic as S
from hlgs_core import spt as SP
b, storage, _, G = bench.merged_two_chunk_scene(1_000_000)
dev = "cuda"
nodes = b["upper_tree_nodes"].to(dev, torch.int32); xyz = b["upper_tree_xyz"].to(dev); bounds = b["bounding_sphere_radii"].to(dev)
md = b["min_distance_squared"].to(dev)
cam = S.make_camera(1920, 1080, T=np.array([0.15, 0.05, 0.2 * math.sin(1.5)]))
planes = SP.extract_frustum_planes(cam["projmatrix"].to(dev))
for rep in range(3):
    lib = SP.L.load()
    N = nodes.size(0)
    cut = torch.zeros((N,), dtype=torch.int32, device=dev)
    scratch = torch.empty(lib.hlgs_upper_cut_scratch_size(N), dtype=torch.uint8, device=dev)
    import ctypes as C
    count = C.c_int(0)
    camp = cam["campos"].reshape(-1)[:3].to(dev).float().contiguous()
    torch.cuda.synchronize()
    SP.L.check(lib.hlgs_upper_tree_cut(N, SP.L.ptr(nodes), SP.L.ptr(xyz), SP.L.ptr(bounds), SP.L.ptr(md), SP.L.ptr(planes),
                                       SP.L.ptr(camp), 1.0, 1, 1, SP.L.ptr(scratch), SP.L.ptr(cut), C.byref(count), SP.L.stream()))
    torch.cuda.synchronize()
    tail = cut[N - 256:].cpu().numpy().view(np.int64)[:120].reshape(-1, 3)
    tail = tail[tail[:, 0] != 0]
    rt = (tail[:, 0] - tail[0, 0]) / 100.0  # us at 100 MHz
    ck = tail[:, 1] - tail[0, 1]
    print("count", count.value, "levels", len(tail))
    for k in range(len(tail)):
        dt = (rt[k + 1] - rt[k]) if k + 1 < len(tail) else float("nan")
        dc = (ck[k + 1] - ck[k]) if k + 1 < len(tail) else 0
        print(f"level {k:2d} size {tail[k, 2]:6d} start {rt[k]:8.1f} us  level {dt:7.1f} us  clk {dc} ({dc / max(dt, 1e-9) / 1e3:.2f} GHz)")
