#!/usr/bin/env python3
"""Config #5's training step (train_post.py with Cache_SPTs, the alt rasterizer and the photometric loss) end to end
on one MI355X, on a synthetic 2-chunk merged hierarchy (BASELINE config #5 names the example dataset, which is not
available here).  The step itself is bench.py's config5 leg (bench_config5), which the default bench run reports;
this wrapper runs it alone with other sizes.  Prints one JSON object."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000, help="leaves over both chunks")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--sh-degree", type=int, default=1)
    ap.add_argument("--no-depth", action="store_true", help="drop the masked inverse-depth L1 term")
    args = ap.parse_args()
    out = bench.bench_config5(args.P, torch.device("cuda", 0), steps=args.steps, sh_degree=args.sh_degree,
                              depth=not args.no_depth)
    out["data"] = "synthetic (seeded PCG64 hierarchy, target image and camera path)"
    print(json.dumps(out))


if __name__ == "__main__":
    main()
