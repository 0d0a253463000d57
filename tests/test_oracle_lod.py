"""Pin the LOD part of the oracle against independent vectorised numpy / torch restatements.

expand_to_size_dynamic / get_interpolation_weights_dynamic (runtime_switching.cu:147-233, 533-684),
the static box variant (:189-219, 495-634), the SPT cut -- intended semantics against the pure-Python
formulation the reference keeps in scene/gaussian_model.py:163-181, compat semantics against
hand-derived vectors showing App. A-10 -- and the render_post lerp against autograd of
gaussian_renderer/__init__.py:304-339 restated in torch.
"""
import numpy as np
import torch

from hlgs_core import synthetic as S
from oracle import oracle as O


def _tree(n_leaves=300, seed=0, sky=0):
    cam = S.make_camera(128, 96)
    leaves = S.make_gaussians(n_leaves, 1, cam, seed=seed)
    return S.make_dynamic_hierarchy(leaves, skybox_points=sky, seed=seed), cam


def _np_size(pos, sc, vp):
    d = np.sqrt(((vp[None] - pos) ** 2).sum(1).astype(np.float32))
    return sc.max(1) / d


def test_hierarchy_generator_layout():
    h, _ = _tree(257)
    nodes = h["nodes"]
    G = nodes.shape[0]
    assert G == 2 * 257 - 1
    root = np.where(nodes[:, 1] == -1)[0]
    assert list(root) == [0] and nodes[0, 0] == 0
    internal = nodes[:, 2] == 2
    assert np.all(nodes[internal, 3] == np.where(internal)[0] + 1)  # first child follows in pre-order
    kids = np.bincount(nodes[1:, 1], minlength=G)
    np.testing.assert_array_equal(kids, nodes[:, 2])
    assert np.all(nodes[1:, 0] == nodes[nodes[1:, 1], 0] + 1)


def test_expand_dynamic_matches_numpy():
    h, cam = _tree(400, sky=5)
    nodes, pos, sc = h["nodes"], h["means3D"], h["scales"]
    vp = np.array([0.1, -0.2, 0.0], np.float32)
    vd = np.array([0.0, 0.0, 1.0], np.float32)
    for target in (0.001, 0.005, 0.02):
        n, ri, pi, ni = O.expand_to_size_dynamic(nodes, pos, sc, target, vp, vd)
        size = _np_size(pos, sc, vp)
        diff = vp[None] - pos
        cosang = (diff / np.linalg.norm(diff, axis=1, keepdims=True) * vd).sum(1)
        par = nodes[:, 1]
        ps = np.where(par >= 0, size[np.maximum(par, 0)], 0)
        sel = (cosang < -0.5) & (nodes[:, 0] >= 0) & (
            ((size >= target) & (nodes[:, 2] == 0)) | ((par >= 0) & (ps >= target) & (size < target)))
        exp = np.where(sel)[0]
        assert n == len(exp)
        np.testing.assert_array_equal(ri[:n], exp)
        np.testing.assert_array_equal(ni[:n], exp)
        has_p = par[exp] != -1
        np.testing.assert_array_equal(pi[:n][has_p], par[exp][has_p])


def test_interp_weights_dynamic_matches_numpy():
    h, _ = _tree(300)
    nodes, pos, sc = h["nodes"], h["means3D"], h["scales"]
    vp = np.array([0.0, 0.0, 0.0], np.float32)
    idx = np.arange(nodes.shape[0], dtype=np.int32)
    target = 0.004
    ts, kids = O.interp_weights_dynamic(idx, target, nodes, pos, sc, vp)
    size = _np_size(pos, sc, vp)
    par = nodes[:, 1]
    t = np.ones(len(idx), np.float32)
    for i in idx:
        p = par[i]
        if p < 0:
            continue
        psz = size[p]
        if psz > 2 * target:
            continue
        start = max(0.5 * psz, size[i])
        diff = psz - start
        if diff > 0:
            t[i] = max(1 - max(0.0, target - start) / diff, 0.0)
    np.testing.assert_allclose(ts, t, rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(kids, np.where(par < 0, 1, nodes[np.maximum(par, 0), 2]))


def test_expand_static_and_weights():
    rng = np.random.default_rng(0)
    N = 200
    nodes = np.zeros((N, 7), np.int32)
    nodes[:, 1] = [-1] + [int(rng.integers(0, i)) for i in range(1, N)]
    nodes[:, 0] = rng.integers(0, 4, N)
    nodes[:, 2] = np.arange(N) * 3
    nodes[:, 3] = rng.integers(0, 3, N)
    nodes[:, 4] = rng.integers(0, 2, N)
    nodes[:, 6] = np.bincount(nodes[1:, 1], minlength=N)
    c = rng.uniform(-3, 3, (N, 3))
    e = rng.uniform(0.05, 1.0, (N, 3))
    boxes = np.zeros((N, 8), np.float32)
    boxes[:, :3], boxes[:, 4:7] = c - e, c + e
    boxes[:, 3] = e.max(1) * 2
    vp = np.array([0.3, 0.1, -0.2], np.float32)
    target = 0.3
    n, ri, pi, ni = O.expand_to_size(nodes, boxes, target, vp)

    def bsize(i):
        b = boxes[i]
        if np.all(vp >= b[:3]) and np.all(vp <= b[4:7]):
            return np.finfo(np.float32).max
        cl = np.maximum(b[:3], np.minimum(b[4:7], vp))
        return b[3] / np.sqrt(((vp - cl) ** 2).sum())

    exp_r, exp_p, exp_n = [], [], []
    for i in range(N):
        s = bsize(i)
        cnt = 0
        if s >= target:
            cnt = nodes[i, 3]
        elif nodes[i, 1] != -1 and bsize(nodes[i, 1]) >= target:
            cnt = nodes[i, 3] + (nodes[i, 4] if nodes[i, 0] != 0 else 0)
        pg = nodes[nodes[i, 1], 2] if nodes[i, 1] != -1 else -1
        for k in range(cnt):
            exp_r.append(nodes[i, 2] + k)
            exp_p.append(pg)
            exp_n.append(i)
    assert n == len(exp_r)
    np.testing.assert_array_equal(ri[:n], exp_r)
    np.testing.assert_array_equal(pi[:n], exp_p)
    np.testing.assert_array_equal(ni[:n], exp_n)
    ts, kids = O.interp_weights(np.arange(N, dtype=np.int32), target, nodes, boxes, vp)
    assert np.all((ts >= 0) & (ts <= 1))
    np.testing.assert_array_equal(kids, np.where(nodes[:, 1] == -1, 1, nodes[np.maximum(nodes[:, 1], 0), 6]))


def _spt_python(gidx, starts, smax, smin, sidx, sdist):
    """The per-SPT formulation of scene/gaussian_model.py:163-181 (binary search for the first entry
    whose max distance is not above d, then keep entries whose min distance is below d)."""
    out, counts = [], []
    for k, d in zip(sidx, sdist):
        lo, hi = starts[k], starts[k + 1]
        spt_max, spt_min, spt_g = smax[lo:hi], smin[lo:hi], gidx[lo:hi]
        a, b = 0, len(spt_max)
        piv = b // 2
        while b - a > 1:
            if spt_max[piv] > d:
                a = piv
            else:
                b = piv
            piv = (a + b) // 2
        keep = np.where(spt_min[:b] < d)[0]
        out.extend(spt_g[keep].tolist())
        counts.append(len(keep))
    return np.array(out, np.int32), np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int32)


def _random_spts(seed, S_count=40, sel=25):
    rng = np.random.default_rng(seed)
    sizes = rng.integers(1, 60, S_count)
    starts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    E = int(starts[-1])
    smax = np.empty(E, np.float32)
    smin = np.empty(E, np.float32)
    for k in range(S_count):
        lo, hi = starts[k], starts[k + 1]
        mx = np.sort(rng.uniform(0.5, 20, hi - lo))[::-1]
        mx[0] = 1e12
        smax[lo:hi] = mx
        smin[lo:hi] = mx * rng.uniform(0.3, 1.0, hi - lo)
    gidx = rng.permutation(E).astype(np.int32) + 1
    sidx = rng.choice(S_count, sel, replace=False).astype(np.int32)
    sdist = rng.uniform(1, 25, sel).astype(np.float32)
    return gidx, starts, smax, smin, sidx, sdist


def test_spt_cut_intended_semantics_match_python():
    for seed in range(5):
        args = _random_spts(seed)
        cut, cp = O.spt_cut(*args, compat=False)
        ecut, ecp = _spt_python(*args)
        np.testing.assert_array_equal(cut, ecut)
        np.testing.assert_array_equal(cp, ecp)


def test_spt_cut_compat_reproduces_boundary_quirk():
    # two SPTs, both fully candidate; interval sizes 3 and 2 -> prefix [0, 3].  The reference attributes
    # candidate idx=3 (first of SPT 1) to SPT 0 at offset 3 (= SPT 1's first entry, stored right after),
    # tested against SPT 0's distance; and it drops Gaussian index 0.
    gidx = np.array([0, 11, 12, 20, 21], np.int32)
    starts = np.array([0, 3, 5], np.int32)
    smax = np.array([1e12, 9, 8, 1e12, 9], np.float32)
    smin = np.array([1, 2, 3, 5.5, 1], np.float32)
    sidx = np.array([0, 1], np.int32)
    sdist = np.array([5.0, 6.0], np.float32)
    cut, cp = O.spt_cut(gidx, starts, smax, smin, sidx, sdist, compat=True)
    # intended: SPT0 keeps {0, 11, 12}; SPT1 keeps {20, 21}.  compat: index 0 dropped, entry 3 (g=20,
    # min 5.5) judged with SPT 0's d=5 -> rejected and counted for SPT 0's interval.
    np.testing.assert_array_equal(cut, [11, 12, 21])
    np.testing.assert_array_equal(cp, [0, 3])
    cut2, cp2 = O.spt_cut(gidx, starts, smax, smin, sidx, sdist, compat=False)
    np.testing.assert_array_equal(cut2, [0, 11, 12, 20, 21])
    np.testing.assert_array_equal(cp2, [0, 3])


def test_lod_interp_matches_torch_autograd():
    rng = np.random.default_rng(4)
    P, n, Sk = 60, 25, 3
    means = rng.normal(size=(P, 3)).astype(np.float32)
    scales = rng.uniform(0.01, 1, (P, 3)).astype(np.float32)
    rots = rng.normal(size=(P, 4)).astype(np.float32)
    rots /= np.linalg.norm(rots, axis=1, keepdims=True)
    opac = rng.uniform(0, 1, (P, 1)).astype(np.float32)
    shs = rng.normal(size=(P, 16, 3)).astype(np.float32)
    ridx = rng.choice(np.arange(Sk, P), n, replace=False).astype(np.int32)
    pidx = rng.integers(Sk, P, n).astype(np.int32)
    w = rng.uniform(0, 1, n).astype(np.float32)
    out = O.lod_interp_forward(Sk, ridx, pidx, w, means, scales, rots, opac, shs)
    # torch restatement of gaussian_renderer/__init__.py:304-339 (interp_python=True)
    T = lambda a: torch.tensor(a, dtype=torch.float64, requires_grad=True)  # noqa: E731
    m, s, r, o, sh = T(means), T(scales), T(rots), T(opac), T(shs)
    ri, pi = torch.tensor(ridx).long(), torch.tensor(pidx).long()
    wi = torch.tensor(w, dtype=torch.float64)[:, None]
    wv = 1 - wi
    mb = wi * m[ri] + wv * m[pi]
    sb = wi * s[ri] + wv * s[pi]
    shb = wi[:, :, None] * sh[ri] + wv[:, :, None] * sh[pi]
    par = r[pi]
    rr = r[ri]
    dots = torch.bmm(rr.unsqueeze(1), par.unsqueeze(2)).flatten()
    par = torch.where((dots < 0)[:, None], -par, par)
    rb = wi * rr + wv * par
    ob = wi * o[ri] + wv * o[pi]
    sky = torch.arange(Sk)
    outs = [torch.cat([m[sky], mb]), torch.cat([s[sky], sb]), torch.cat([r[sky], rb]), torch.cat([o[sky], ob]),
            torch.cat([sh[sky], shb])]
    for got, ref in zip([out["means"], out["scales"], out["rots"], out["opac"][:, None], out["shs"]], outs):
        np.testing.assert_allclose(got, ref.detach().numpy(), rtol=1e-6, atol=1e-6)
    gs = [rng.normal(size=tuple(x.shape)).astype(np.float32) for x in outs]
    sum(((x * torch.tensor(g, dtype=torch.float64)).sum() for x, g in zip(outs, gs))).backward()
    d = O.lod_interp_backward(Sk, ridx, pidx, w, rots, P, dict(means=gs[0], scales=gs[1], rots=gs[2], opac=gs[3],
                                                               shs=gs[4]))
    for got, leaf in zip([d["means"], d["scales"], d["rots"], d["opac"][:, None], d["shs"]], [m, s, r, o, sh]):
        np.testing.assert_allclose(got, leaf.grad.numpy(), rtol=1e-5, atol=1e-5)
