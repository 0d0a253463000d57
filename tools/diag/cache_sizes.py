"""Config #5's cache bookkeeping sizes per step (k_cache_lists' three loops: the coarse cut's length, the SPTs in it,
the previous step's SPTs), printed as JSON lines to stderr.  Runs bench.py's config5 leg for a few steps."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from hlgs_core import spt_cache  # noqa: E402

_step = spt_cache.SPTCache.step


def step(self, *a, **k):
    m = self.prev_SPT_indices.numel()
    out = _step(self, *a, **k)
    pl = self.last_plan
    print(json.dumps(dict(n_cut=int(self._cut_count[0].item()), prev_spts=m, kept=int(pl["n_kept"]),
                          loaded=int(pl["load_SPT_indices"].numel()),
                          upper=int(pl["upper_tree_nodes_to_render"].numel()),
                          resident=int(out.numel()))), file=sys.stderr, flush=True)
    return out


spt_cache.SPTCache.step = step
bench.bench_config5(1_000_000, torch.device("cuda", 0), steps=3, sh_degree=1, depth=True)
