"""View-data-parallel config #5 step (SURVEY 8(e) applied to train_post.py's SPT cache) on gloo, world
size 2, CPU only.

Each rank trains its own view.  The ranks gather every rank's view (hlgs_core.spt_cache.gather_views), each
computes the union cut of the batch -- visible in any frustum, the nearest camera deciding each LOD test and SPT
distance -- and the cache bookkeeping from the same inputs, so all ranks hold the same resident set in the same order.
Each rank renders its own view over that set, and the gradient all-reduce (FlatGradExchange, gloo) averages them.
Here the cut and bookkeeping are the CPU restatement (oracle/spt_ref.py; the HIP path is checked against it,
bit-exact, by tests/test_gpu_cache.py::test_spt_cache_view_batches_match_restatement) and the per-view gradient is
the oracle's rasterizer backward.  The test checks that both ranks hold identical resident sets and that the
exchanged gradients are bitwise equal to one process running both views on that resident set and averaging.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hlgs_core import synthetic as S

NAMES = ("xyz", "f_dc", "opacity", "scaling", "rotation", "f_rest")
SHAPES = {"xyz": (3,), "f_dc": (1, 3), "opacity": (1,), "scaling": (3,), "rotation": (4,), "f_rest": (15, 3)}
W, H = 160, 120


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene(sky=4, n=4000, seed=11):
    from hlgs_core import spt
    cam0 = S.make_camera(256, 192)
    h = S.make_dynamic_hierarchy(S.make_gaussians(n, 0, cam0, seed=seed), skybox_points=sky, seed=seed)
    nodes = torch.tensor(h["nodes"])
    nodes[:, 3] = torch.where(nodes[:, 2] == 2, nodes[:, 3], torch.zeros_like(nodes[:, 3]))
    b = spt.build_hierarchical_spt(nodes, torch.tensor(h["means3D"]), torch.log(torch.tensor(h["scales"])), sky, 3.0,
                                   0.02, 20)
    b = {k: (v.numpy() if v is not None else None) for k, v in b.items()}
    G = nodes.shape[0]
    storage = {k: np.asarray(h["means3D"], np.float32).copy() if k == "xyz" else None for k in NAMES}
    rng = np.random.default_rng(seed)
    for k in NAMES:
        if storage[k] is None:
            storage[k] = rng.normal(0, 0.3, size=(G,) + SHAPES[k]).astype(np.float32)
    storage["scaling"] = np.log(np.asarray(h["scales"], np.float32)).astype(np.float32)
    return b, storage


def _cameras():
    return [S.make_camera(W, H, T=np.array([0.05, 0.0, 0.4])),
            S.make_camera(W, H, T=np.array([-0.3, 0.05, 0.9]))]


def _resident(b, sky, fpt, campos):
    """Union cut + bookkeeping of a batch of views (the restatement), from an empty cache: the resident rows."""
    from hlgs_core import spt
    from oracle import oracle as O
    from oracle import spt_ref as SR
    planes = np.stack([spt.extract_frustum_planes(torch.as_tensor(f)).numpy() for f in fpt])
    coarse = SR.upper_tree_cut(b["upper_tree_nodes"], b["upper_tree_xyz"], b["bounding_sphere_radii"],
                               b["min_distance_squared"], planes, campos, 1.0, True, True)
    cut_fn = lambda i, d: O.spt_cut(b["SPT_gaussian_indices"], b["SPT_starts"], b["SPT_max"],  # noqa: E731
                                    b["SPT_min"], i, d, compat=True)
    r = SR.cache_pass(b["upper_tree_nodes"], b["upper_tree_xyz"], coarse, campos, 1.0, np.zeros(0, np.int32),
                      np.zeros(0, np.float32), np.zeros(0, np.int32), np.arange(sky, dtype=np.int32), 0, sky, 0.9,
                      0.05, cut_fn)
    return r["render_indices"]


def _view_grads(storage, rows, cam, seed):
    """The rank's own view over the resident rows: the oracle's rasterizer forward + backward (activated
    parameters, SH degree 3), gradients per parameter table in NAMES order."""
    from oracle import oracle as O
    xyz = storage["xyz"][rows]
    sh = np.concatenate([storage["f_dc"][rows], storage["f_rest"][rows]], 1)
    rot = storage["rotation"][rows]
    sc = dict(means3D=xyz, shs=sh, sh_degree=3, scales=np.exp(storage["scaling"][rows]).astype(np.float32),
              rotations=(rot / np.linalg.norm(rot, axis=1, keepdims=True)).astype(np.float32),
              opacities=(1 / (1 + np.exp(-storage["opacity"][rows]))).astype(np.float32))
    g, gd = S.upstream_grads(W, H, seed=seed)
    fr = O.forward(sc, S.cam_numpy(cam), do_depth=True)
    gr = O.backward(fr, sc, g, gd)
    dsh = gr["dsh"].reshape(len(rows), 16, 3)
    return [gr["dmean3D"].reshape(-1, 3), dsh[:, :1], gr["dopacity"].reshape(-1, 1), gr["dscale"].reshape(-1, 3),
            gr["drot"].reshape(-1, 4), dsh[:, 1:]]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hlgs_core.dp import FlatGradExchange
    from hlgs_core.spt_cache import gather_views
    sky = 4
    b, storage = _scene(sky)
    cam = _cameras()[rank]
    fpt, campos = gather_views(cam["projmatrix"], cam["campos"])
    rows = _resident(b, sky, fpt.numpy(), campos.numpy())
    grads = _view_grads(storage, rows, cam, seed=20 + rank)
    params = [torch.zeros(g.shape, requires_grad=True) for g in grads]
    for p, g in zip(params, grads):
        p.grad = torch.tensor(np.ascontiguousarray(g))
    ex = FlatGradExchange(params, bucket_bytes=8192)
    ex.allreduce()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), rows=rows, views=fpt.numpy(),
             **{f"g{i}": p.grad.numpy() for i, p in enumerate(params)})
    ex.close()
    dist.destroy_process_group()


def test_config5_view_dp_gloo(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r0, r1 = np.load(tmp_path / "r0.npz"), np.load(tmp_path / "r1.npz")
    np.testing.assert_array_equal(r0["rows"], r1["rows"])  # the same resident set, in the same order
    np.testing.assert_array_equal(r0["views"], r1["views"])
    sky = 4
    b, storage = _scene(sky)
    cams = _cameras()
    fpt = np.stack([c["projmatrix"].numpy() for c in cams])
    campos = np.stack([c["campos"].numpy().reshape(-1)[:3] for c in cams])
    rows = _resident(b, sky, fpt, campos)
    np.testing.assert_array_equal(rows, r0["rows"])
    # the union holds at least the rows each view's own cut would
    for c in cams:
        own = _resident(b, sky, c["projmatrix"].numpy()[None], c["campos"].numpy().reshape(1, -1)[:, :3])
        assert len(rows) >= len(own)
    assert len(rows) > 100
    g0 = _view_grads(storage, rows, cams[0], seed=20)
    g1 = _view_grads(storage, rows, cams[1], seed=21)
    for i, (a, c) in enumerate(zip(g0, g1)):
        want = ((a.astype(np.float32) + c.astype(np.float32)).astype(np.float32) * np.float32(0.5)).astype(np.float32)
        for r in (r0, r1):
            np.testing.assert_array_equal(r[f"g{i}"], want, err_msg=f"gradient table {i}")
        assert np.abs(want).max() > 0
