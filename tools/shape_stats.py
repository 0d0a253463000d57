#!/usr/bin/env python3
"""Pass counts of the blend kernels for different 64-pixel pass shapes, on the bench frame (configs[1]).

Both blends run one wave-wide pass per (splat, 64-pixel block of the tile) that the splat's alpha footprint reaches
and that still holds a pixel whose last contributor lies behind the splat.  Their cost follows that pass count, and the
share of useful lanes is valid pairs / (64 x passes).  This counts both for a 16x16 tile split into
  quad:  four 8x8 quadrants (the layout of rounds 1-5),
  strip: four 16x4 row strips,
  col:   four 4x16 column strips,
from the CPU oracle's frame (float64 footprints).  Statistics only; experiment tooling, not product code.

    python tools/shape_stats.py [P] [W] [H] [STRIDE]

STRIDE > 1 counts every STRIDE-th tile only (a sample: the ratios between the shapes are what matter).
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
from hlgs_core import synthetic as S  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main(P=1_000_000, W=1920, H=1080, stride=1):
    cam = S.make_camera(W, H)
    sc = S.make_gaussians(P, 3, cam, seed=0)
    t0 = time.time()
    fr = O.forward(sc, S.cam_numpy(cam) if hasattr(S, "cam_numpy") else cam, do_depth=True, omp=True, drop_empty=True)
    print(f"oracle forward {time.time() - t0:.1f} s, R = {fr.R}", flush=True)
    gx = (W + 15) // 16
    Rb = int((fr.ranges[:, 1] - fr.ranges[:, 0]).sum())
    ids = fr.point_list[:Rb].astype(np.int64)
    tile = np.repeat(np.arange(gx * ((H + 15) // 16)), (fr.ranges[:, 1] - fr.ranges[:, 0]).astype(np.int64))
    li = np.arange(Rb) - fr.ranges[tile, 0].astype(np.int64)
    sel = np.flatnonzero(tile % stride == 0)
    ids, tile, li = ids[sel], tile[sel], li[sel]
    Rb = len(sel)
    ncon = fr.n_contrib.reshape(H, W)
    xy = fr.means2D[ids].astype(np.float32)
    co = fr.conic_opacity[ids].astype(np.float32)
    thr = -np.log2(255.0 * co[:, 3])
    ly, lx = np.mgrid[0:16, 0:16]
    lx = lx.ravel()
    ly = ly.ravel()
    shapes = {"quad": (lx >= 8) + 2 * (ly >= 8), "strip": ly // 4, "col": lx // 4}
    tot = {k: 0 for k in shapes}
    sets = np.zeros(16, np.int64)  # quadrant layout: instances by visited-quadrant set (bit k = quadrant k)
    fwd = {k: 0 for k in shapes}
    valid_n = 0
    CH = 20_000
    for s in range(0, Rb, CH):
        e = min(Rb, s + CH)
        t = tile[s:e]
        px = (t % gx)[:, None] * 16 + lx[None, :]
        py = (t // gx)[:, None] * 16 + ly[None, :]
        inside = (px < W) & (py < H)
        dx = xy[s:e, 0:1] - px
        dy = xy[s:e, 1:2] - py
        a, b, c = co[s:e, 0:1], co[s:e, 1:2], co[s:e, 2:3]
        e2 = -0.5 * np.log2(np.e) * (a * dx * dx + 2 * b * dx * dy + c * dy * dy)
        foot = (e2 >= thr[s:e, None]) & (e2 <= 0) & inside
        last = np.where(inside, ncon[np.minimum(py, H - 1), np.minimum(px, W - 1)], 0)
        valid_n += int((foot & (li[s:e, None] < last)).sum())
        for name, blk in shapes.items():
            vset = np.zeros(e - s, np.int64)
            for k in range(4):
                m = blk[None, :] == k
                bl = np.where(m, last, 0).max(1)
                bf = (foot & m).any(1)
                vk = bf & (li[s:e] < bl)
                tot[name] += int(vk.sum())
                vset |= vk.astype(np.int64) << k
            if name == "quad":
                sets += np.bincount(vset, minlength=16)
                fwd[name] += int(bf.sum())  # the forward's waves visit every splat that reaches them (until done)
    out = {"R_binned_sampled": Rb, "tile_stride": stride, "valid_pairs": valid_n}
    for name in shapes:
        out[name] = {"bwd_passes": tot[name], "fwd_visits_upper": fwd[name], "lane_use": valid_n / (64 * tot[name])}
    out["quad_visit_sets"] = {format(k, "04b")[::-1]: int(sets[k]) for k in range(16)}  # string: quadrants 0..3
    out["quad_pairs"] = {"h01": int(sum(sets[k] for k in range(16) if k & 3 == 3)),
                         "h23": int(sum(sets[k] for k in range(16) if k & 12 == 12)),
                         "v02": int(sum(sets[k] for k in range(16) if k & 5 == 5)),
                         "v13": int(sum(sets[k] for k in range(16) if k & 10 == 10))}
    print(out)


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:]])
