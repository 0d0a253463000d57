"""View-data-parallel gradient exchange on CPU with gloo, world_size 2 (the N>1 path of bench.py).

Each rank computes gradients of its own view; after FlatGradExchange.allreduce every rank must hold the
mean of all ranks' gradients, bitwise identical across ranks.  Gradients come from the oracle (one view
per rank), exactly the quantities the GPU ranks exchange."""
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_grads(rank, world):
    from hlgs_core import synthetic as S
    from oracle import oracle as O
    cam = S.ring_camera(64, 48, rank, world)
    sc = S.make_gaussians(300, 1, S.make_camera(64, 48), seed=0)
    fr = O.forward(sc, S.cam_numpy(cam))
    g = O.backward(fr, sc, *S.upstream_grads(64, 48, seed=1 + rank))
    return [g["dmean3D"], g["dscale"], g["drot"], g["dopacity"], g["dsh"]]


def _worker(rank, world, port, out_dir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hlgs_core.dp import FlatGradExchange
    grads = _rank_grads(rank, world)
    params = [torch.zeros(g.shape, requires_grad=True) for g in grads]
    for p, g in zip(params, grads):
        p.grad = torch.tensor(g)
    FlatGradExchange(params, bucket_bytes=4096).allreduce()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), *[p.grad.numpy() for p in params])
    dist.destroy_process_group()


def test_view_dp_allreduce_gloo(tmp_path):
    world = 2
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    r0, r1 = np.load(tmp_path / "r0.npz"), np.load(tmp_path / "r1.npz")
    sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
    expect = [(a + b) / 2 for a, b in zip(_rank_grads(0, world), _rank_grads(1, world))]
    for k, e in zip(r0.files, expect):
        np.testing.assert_array_equal(r0[k], r1[k])
        np.testing.assert_allclose(r0[k], e, rtol=1e-6, atol=1e-7)
