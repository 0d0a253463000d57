"""The SPT-cache restatement (oracle/spt_ref.py cache_pass, adam_dense) pinned against torch's own primitives on
the CPU: searchsorted over an unsorted list, isclose in float32, Python slice bounds, isin, and a second
restatement of train_post.py:346-430 written with the torch calls the reference makes."""
import numpy as np
import pytest
import torch

from oracle import spt_ref as SR


def test_lower_bound_is_torch_searchsorted_on_unsorted_lists():
    rng = np.random.default_rng(0)
    for n in (0, 1, 2, 7, 64, 300):
        arr = rng.permutation(1000)[:n].astype(np.int32)
        q = rng.integers(-5, 1005, 200).astype(np.int32)
        want = torch.searchsorted(torch.tensor(arr), torch.tensor(q)).numpy()
        got = np.array([SR.lower_bound(arr, v) for v in q])
        np.testing.assert_array_equal(got, want)


def test_isclose32_is_torch_isclose():
    rng = np.random.default_rng(1)
    a = rng.uniform(0, 10, 5000).astype(np.float32)
    b = (a * rng.uniform(0.8, 1.2, 5000)).astype(np.float32)
    b[:50] = a[:50]
    np.seterr(invalid="ignore")
    b[50:60] = np.inf
    a[60:65] = np.inf
    b[60:65] = np.inf
    for rtol in (0.9, 0.05, 0.0):
        want = torch.isclose(torch.tensor(a), torch.tensor(b), rtol=rtol, atol=0.05).numpy()
        got = np.array([SR.isclose32(x, y, rtol, 0.05) for x, y in zip(a, b)])
        np.testing.assert_array_equal(got, want)


def _torch_pass(nodes, xyz, coarse, cam, dm, prev_idx, prev_dist, prev_counts, render, n_loaded, sky, rtol, spt_cut):
    """train_post.py:346-430 with the torch calls the reference makes (searchsorted, isclose, isin, cat, the
    per-kept-SPT slice loop); an independent second restatement for pinning cache_pass."""
    nodes, xyz, coarse = torch.tensor(nodes), torch.tensor(xyz), torch.tensor(coarse, dtype=torch.int64)
    cam = torch.tensor(cam)
    prev_idx, prev_dist, prev_counts = torch.tensor(prev_idx), torch.tensor(prev_dist), torch.tensor(prev_counts)
    render = torch.tensor(render)
    leaf = coarse[nodes[coarse, 2] == 0]
    has_spt = nodes[leaf, 3] >= 0
    spt_idx = nodes[leaf][has_spt, 3]
    upper = nodes[leaf][nodes[leaf, 3] <= 0, 5]
    # the reference runs this on the GPU, where sqrt is correctly rounded; torch's CPU vector sqrt is not (it is
    # off by one ulp on ~0.7% of inputs), so the square root is taken in float64 and rounded once
    dist = (xyz[leaf[has_spt]] - cam).pow(2).sum(1).double().sqrt().float() * dm
    pos = torch.searchsorted(spt_idx, prev_idx)
    valid = pos < spt_idx.numel()
    valid[valid.clone()] &= spt_idx[pos[valid]] == prev_idx[valid]
    close = torch.isclose(dist[pos[valid]], prev_dist[valid], rtol=rtol, atol=0.05)
    kept_j = torch.nonzero(valid, as_tuple=True)[0][torch.nonzero(close, as_tuple=True)[0]]
    keep_vals = spt_idx[pos[valid][close]]
    keep = torch.zeros(len(render), dtype=torch.bool)
    ends = []
    for j in kept_j.tolist():
        end = len(render) - n_loaded if j == len(prev_counts) - 1 else prev_counts[j + 1]
        ends.append(int(end))
        keep[prev_counts[j]:end] = True
    keep[:sky] = True
    load = ~torch.isin(spt_idx, keep_vals)
    if int(load.sum()):
        cut, counts = spt_cut(spt_idx[load].numpy(), dist[load].numpy())
        cut, counts = torch.tensor(cut), torch.tensor(counts)
    else:
        cut, counts = torch.zeros(0, dtype=torch.int32), torch.zeros(0, dtype=torch.int32)
    counts = counts + sky
    new_counts = torch.zeros(len(kept_j) + len(counts), dtype=torch.int32)
    prefix = 0
    for k, (j, end) in enumerate(zip(kept_j.tolist(), ends)):
        new_counts[k] = prefix
        prefix += end - int(prev_counts[j])
    new_counts[len(kept_j):] = counts + prefix
    lfd = torch.cat([cut.to(torch.int32), upper.to(torch.int32)])
    return dict(SPT_indices=torch.cat([keep_vals, spt_idx[load]]).numpy(),
                SPT_distances=torch.cat([prev_dist[kept_j], dist[load]]).numpy(), SPT_counts=new_counts.numpy(),
                keep_mask=keep.numpy(), render_indices=torch.cat([render[keep], lfd]).numpy())


def _fake_cut(starts):
    def cut(idx, dist):
        parts = [np.arange(starts[i], starts[i] + 1 + int(d * 3) % 4, dtype=np.int32) for i, d in zip(idx, dist)]
        sizes = np.array([len(p) for p in parts], np.int64)
        return np.concatenate(parts), np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int32)
    return cut


@pytest.mark.parametrize("seed", range(6))
def test_cache_pass_matches_torch_restatement(seed):
    rng = np.random.default_rng(seed)
    n = 400
    nodes = np.zeros((n, 6), np.int32)
    nodes[:, 2] = (rng.uniform(size=n) < 0.3) * 2              # some inner nodes
    nodes[:, 3] = np.where(rng.uniform(size=n) < 0.7, rng.permutation(n), -1)
    nodes[:, 5] = rng.integers(0, 10000, n)
    xyz = rng.normal(size=(n, 3)).astype(np.float32)
    cam = rng.normal(size=3).astype(np.float32)
    sky = int(rng.integers(0, 4))
    starts = np.arange(0, 5 * n, 5)
    cut_fn = _fake_cut(starts)
    render, n_loaded = np.arange(sky, dtype=np.int32), 0
    prev_idx, prev_dist, prev_counts = (np.zeros(0, np.int32), np.zeros(0, np.float32), np.zeros(0, np.int32))
    for step in range(4):
        coarse = rng.permutation(n)[: int(rng.integers(50, 300))]
        dm = 1.5 ** int(rng.integers(0, 3))
        rtol = (0.9, 0.05)[step % 2]
        a = SR.cache_pass(nodes, xyz, coarse, cam, dm, prev_idx, prev_dist, prev_counts, render, n_loaded, sky,
                          rtol, 0.05, cut_fn)
        b = _torch_pass(nodes, xyz, coarse, cam, dm, prev_idx, prev_dist, prev_counts, render, n_loaded, sky,
                        rtol, cut_fn)
        for k in b:
            np.testing.assert_array_equal(a[k], b[k], err_msg=f"{k} step {step}")
        prev_idx, prev_dist, prev_counts = a["SPT_indices"], a["SPT_distances"], a["SPT_counts"]
        render, n_loaded = a["render_indices"], len(a["load_from_disk_indices"])
        cam = (cam + rng.normal(size=3) * 0.05).astype(np.float32)


def test_adam_dense_restatement_is_torch_adam_math():
    """adam_dense (the reference's mul_/add_ form) against torch.optim.Adam (whose moment update is a lerp, so
    agreement is to rounding), three steps, with the skybox rows' gradients zeroed first."""
    g = torch.Generator().manual_seed(0)
    p = torch.randn(50, 3, generator=g)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    q = torch.nn.Parameter(p.clone())
    opt = torch.optim.Adam([q], lr=1e-3, betas=(0.9, 0.999), eps=1e-8, foreach=False)
    for it in range(3):
        grad = torch.randn(50, 3, generator=g)
        gr = grad.clone()
        SR.adam_dense(p, gr, m, v, 1e-3, it + 1, sky=2)
        assert (gr[:2] == 0).all()
        grad[:2] = 0
        q.grad = grad
        opt.step()
    torch.testing.assert_close(p, q.detach(), rtol=1e-6, atol=1e-7)
