"""Host-side profile (cProfile) of SPTCache.step on bench.py's config5 camera path: where the Python / ctypes /
synchronisation time of a cache step goes."""
import cProfile, io, math, os, pstats, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
import numpy as np, torch
import bench
from hlgs_core import synthetic as S
from hlgs_core.spt_cache import SPTCache
b, storage, _, G = bench.merged_two_chunk_scene(1_000_000)
cache = SPTCache(storage, b, 0, reuse_tolerance=0.9)
W, H = 1920, 1080
cams = [{k_: (v.cuda() if torch.is_tensor(v) else v) for k_, v in S.make_camera(W, H, T=np.array([0.03 * k, 0.01 * k, 0.2 * math.sin(0.3 * k)])).items()} for k in range(24)]
for k in range(4):
    cache.step(cams[k]["projmatrix"], cams[k]["campos"])
torch.cuda.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
for k in range(4, 24):
    cache.step(cams[k]["projmatrix"], cams[k]["campos"])
torch.cuda.synchronize()
pr.disable()
print(f"{(time.perf_counter() - t0) / 20 * 1e3:.3f} ms per step (host clock, synchronised at the end)")
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(s.getvalue())
