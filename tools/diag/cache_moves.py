"""Rows the SPT cache moves per step on bench.py's config5 camera path (load from host, write back, kept)."""
import math, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
import numpy as np, torch
import bench
from hlgs_core import synthetic as S
from hlgs_core.spt_cache import SPTCache
b, storage, _, G = bench.merged_two_chunk_scene(1_000_000)
cache = SPTCache(storage, b, 0, reuse_tolerance=0.9)
W, H = 1920, 1080
for k in range(12):
    cam = {k_: (v.cuda() if torch.is_tensor(v) else v) for k_, v in S.make_camera(W, H, T=np.array([0.03 * k, 0.01 * k, 0.2 * math.sin(0.3 * k)])).items()}
    torch.cuda.synchronize(); t0 = time.perf_counter()
    cache.step(cam["projmatrix"], cam["campos"])
    torch.cuda.synchronize(); dt = (time.perf_counter() - t0) * 1e3
    pl = cache.last_plan
    print(f"step {k}: resident {cache.render_indices.numel()} kept_rows {pl['keep_rows'].numel()} "
          f"load {pl['load_from_disk_indices'].numel()} write_back {pl['write_back_rows'].numel()} "
          f"spts kept {pl['n_kept']} loaded {pl['load_SPT_indices'].numel()}  {dt:.2f} ms")
