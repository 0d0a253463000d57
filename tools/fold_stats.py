#!/usr/bin/env python3
"""Visit statistics of the blend backward on the bench frame (configs[1]), from the CPU oracle's frame.

For every (tile, splat) instance: the quadrants the current backward visits (footprint reaches the quadrant and the
splat lies in front of the quadrant's furthest contributor), the valid pixels (alpha >= 1/255, in front of the pixel's
last contributor), and whether the splat's alpha footprint inside the tile fits one 8x8 window -- then one folded pass
(each lane serving the one window pixel that falls on it) replaces the quadrant passes.  Statistics only (float64
footprints); experiment tooling, not product code.

    python tools/fold_stats.py [P] [W] [H]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
from hlgs_core import synthetic as S  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main(P=1_000_000, W=1920, H=1080):
    cam = S.make_camera(W, H)
    sc = S.make_gaussians(P, 3, cam, seed=0)
    t0 = time.time()
    fr = O.forward(sc, S.cam_numpy(cam) if hasattr(S, "cam_numpy") else cam, do_depth=True, omp=True, drop_empty=True)
    print(f"oracle forward {time.time() - t0:.1f} s, R = {fr.R}", flush=True)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    Rb = int((fr.ranges[:, 1] - fr.ranges[:, 0]).sum())  # binned instances (drop_empty)
    ids = fr.point_list[:Rb].astype(np.int64)
    tile = np.repeat(np.arange(gx * gy), (fr.ranges[:, 1] - fr.ranges[:, 0]).astype(np.int64))
    li = np.arange(Rb) - fr.ranges[tile, 0].astype(np.int64)
    ncon = fr.n_contrib.reshape(H, W)
    xy = fr.means2D[ids].astype(np.float64)
    co = fr.conic_opacity[ids].astype(np.float64)
    thr = -np.log2(255.0 * co[:, 3])  # alpha >= 1/255 <=> e2 >= thr
    ly, lx = np.mgrid[0:16, 0:16]
    lx = lx.ravel()
    ly = ly.ravel()
    quad = (lx >= 8) + 2 * (ly >= 8)
    tot = dict(inst=0, passes=0, folded=0, valid=0, fold2=0, fold3=0, fold4=0, nofold_multi=0, single=0, none=0)
    hist = np.zeros(5, np.int64)
    CH = 100_000
    acc_g = []
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
        valid = foot & (li[s:e, None] < last)
        # quadrant visit: footprint reaches quadrant k and some pixel of k has last > li
        qlast = np.stack([np.where(quad[None, :] == k, last, 0).max(1) for k in range(4)], 1)
        qfoot = np.stack([(foot & (quad[None, :] == k)).any(1) for k in range(4)], 1)
        visit = qfoot & (li[s:e, None] < qlast)
        nv = visit.sum(1)
        hist += np.bincount(nv, minlength=5)[:5]
        # footprint box inside the tile
        fx = np.where(foot, lx[None, :], 99)
        bx0 = fx.min(1)
        bx1 = np.where(foot, lx[None, :], -1).max(1)
        by0 = np.where(foot, ly[None, :], 99).min(1)
        by1 = np.where(foot, ly[None, :], -1).max(1)
        fits = (bx1 - bx0 < 8) & (by1 - by0 < 8)
        fold = fits & (nv >= 2)
        # one-axis folds: x extent < 8 folds each quadrant row's two quadrants into one pass (and y likewise)
        rows = (visit[:, 0] | visit[:, 1]).astype(int) + (visit[:, 2] | visit[:, 3])
        cols = (visit[:, 0] | visit[:, 2]).astype(int) + (visit[:, 1] | visit[:, 3])
        best = nv.copy()
        best = np.where(bx1 - bx0 < 8, np.minimum(best, rows), best)
        best = np.where(by1 - by0 < 8, np.minimum(best, cols), best)
        best = np.where(fits & (nv >= 1), 1, best)
        sub = (lx // 4) + 4 * (ly // 4)  # 4x4 sub-blocks
        slast = np.stack([np.where(sub[None, :] == k, last, 0).max(1) for k in range(16)], 1)
        sfoot = np.stack([(foot & (sub[None, :] == k)).any(1) for k in range(16)], 1)
        sv = sfoot & (li[s:e, None] < slast)  # (inst, 16) sub-block visits
        grp = np.array([(k % 4) % 2 + 2 * ((k // 4) % 2) for k in range(16)])  # lattice: group = (sx & 1) + 2 (sy & 1)
        gcount = np.stack([sv[:, grp == gg].sum(1) for gg in range(4)], 1)
        gq = np.array([(k % 4) // 2 + 2 * ((k // 4) // 2) for k in range(16)])  # quadrant-as-group layout
        qcount = np.stack([sv[:, gq == gg].sum(1) for gg in range(4)], 1)
        # uniform slot (quadrant k), group = 4x4 sub-block inside it: per (inst, quadrant, group) visits
        kq = np.stack([sv[:, (gq == k) & (grp == gg)].sum(1) for k in range(4) for gg in range(4)], 1)
        acc_g.append((t, li[s:e], gcount, qcount, kq))
        tot["sub4_visits"] = tot.get("sub4_visits", 0) + int((sfoot & (li[s:e, None] < slast)).sum())
        tot["axisfold"] = tot.get("axisfold", 0) + int(best.sum())
        tot["axisfold_2way_only"] = tot.get("axisfold_2way_only", 0) + int(
            np.where((bx1 - bx0 < 8) & (nv >= 2), np.minimum(nv, rows), np.where((by1 - by0 < 8) & (nv >= 2), np.minimum(nv, cols), nv)).sum())
        tot["inst"] += e - s
        tot["passes"] += int(nv.sum())
        tot["folded"] += int(np.where(fold, 1, nv).sum())
        tot["valid"] += int(valid.sum())
        tot["fold2"] += int((fold & (nv == 2)).sum())
        tot["fold3"] += int((fold & (nv == 3)).sum())
        tot["fold4"] += int((fold & (nv == 4)).sum())
        tot["nofold_multi"] += int((~fits & (nv >= 2)).sum())
        tot["single"] += int((nv == 1).sum())
        tot["none"] += int((nv == 0).sum())
    tot["visit_hist"] = hist.tolist()
    tot["lane_use_now"] = tot["valid"] / (64 * tot["passes"])
    tot["lane_use_folded"] = tot["valid"] / (64 * tot["folded"])
    t_all = np.concatenate([a[0] for a in acc_g]); li_all = np.concatenate([a[1] for a in acc_g])
    cnt = (fr.ranges[:, 1] - fr.ranges[:, 0]).astype(np.int64)
    clen = np.maximum(((cnt + 2) // 3 + 63) & ~63, 192)
    chunk = li_all // clen[t_all]
    # batches counted from the chunk's end (back to front)
    cend = np.minimum(cnt[t_all], (chunk + 1) * clen[t_all])
    batch = (cend - 1 - li_all) // 64
    key = (t_all * 4 + chunk) * 64 + batch
    for name, idx in (("lattice", 2), ("quadrant", 3)):
        gc = np.concatenate([a[idx] for a in acc_g])
        order = np.argsort(key, kind="stable")
        k_s = key[order]
        bounds = np.flatnonzero(np.r_[True, k_s[1:] != k_s[:-1], True])
        sums = np.add.reduceat(gc[order], bounds[:-1], axis=0)
        tot["sub4_iters_" + name] = int(sums.max(1).sum())
        tot["sub4_batches"] = len(bounds) - 1
    kq = np.concatenate([a[4] for a in acc_g])
    sums = np.add.reduceat(kq[order], bounds[:-1], axis=0).reshape(-1, 4, 4)
    tot["sub4_iters_uniform_quadrant"] = int(sums.max(2).sum())
    tot["lane_use_sub4"] = tot["valid"] / (16 * tot["sub4_visits"])
    tot["sub4_group_passes_lower_bound"] = tot["sub4_visits"] / 4
    print(tot)


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:]])
