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
    ex = FlatGradExchange(params, bucket_bytes=4096)
    ex.allreduce()
    assert ex.last_collectives > 1  # packed gradients: bucketed, pack and transfer pipelined
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


def _direct_worker(rank, world, port, out_dir):
    """The rasterizer backward's direct path: gradients written into the exchange's flat buffer (direct_grad),
    adopted by autograd as .grad, all-reduced without packing; a second backward on top of a set .grad must
    accumulate into fresh memory (no aliasing)."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hlgs_core.dp import FlatGradExchange, direct_grad
    grads = [torch.tensor(g) for g in _rank_grads(rank, world)]
    params = [torch.zeros(g.shape, requires_grad=True) for g in grads]

    class Render(torch.autograd.Function):  # stands in for _RasterizeGaussians: grads land where direct_grad says
        @staticmethod
        def forward(ctx, scale, *ps):
            ctx.ps, ctx.scale = ps, scale
            return sum((p * 0).sum() for p in ps)

        @staticmethod
        def backward(ctx, _):
            outs = []
            for p, g in zip(ctx.ps, grads):
                d = direct_grad(p)
                d = torch.empty_like(g) if d is None else d
                d.copy_(g * ctx.scale)
                outs.append(d)
            return (None,) + tuple(outs)

    ex = FlatGradExchange(params, bucket_bytes=4096)
    Render.apply(1.0, *params).backward()
    lo, hi = ex.flat.data_ptr(), ex.flat.data_ptr() + 4 * ex.flat.numel()
    aliased = all(lo <= p.grad.data_ptr() < hi for p in params)
    Render.apply(1.0, *params).backward()  # .grad set: accumulate, 2 x local gradient
    doubled = all(torch.equal(p.grad, 2 * g) for p, g in zip(params, grads))
    ex.allreduce()  # ends the round: the flat buffer may be handed out again
    for p in params:
        p.grad = None
    # two renders of the same parameters in one autograd pass: both backwards run before AccumulateGrad, so the
    # buffer must be handed out once only (else the engine sums the buffer with itself)
    (Render.apply(1.0, *params) + Render.apply(2.0, *params)).backward()
    twice = all(torch.equal(p.grad, 3 * g) for p, g in zip(params, grads))
    ex.allreduce()
    for p in params:
        p.grad = None
    Render.apply(1.0, *params).backward()
    ex.allreduce()
    assert ex.last_collectives == 1  # gradients already in the flat buffer: one collective over all of it
    ex.close()
    np.savez(os.path.join(out_dir, f"d{rank}.npz"), *[p.grad.numpy() for p in params],
             flags=np.array([aliased, doubled, twice]))
    dist.destroy_process_group()


def test_view_dp_direct_gradients_gloo(tmp_path):
    world = 2
    port = _free_port()
    mp.spawn(_direct_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    r0, r1 = np.load(tmp_path / "d0.npz"), np.load(tmp_path / "d1.npz")
    assert r0["flags"].all() and r1["flags"].all()
    sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
    expect = [(a + b) / 2 for a, b in zip(_rank_grads(0, world), _rank_grads(1, world))]
    for k, e in zip([f for f in r0.files if f != "flags"], expect):
        np.testing.assert_array_equal(r0[k], r1[k])
        np.testing.assert_allclose(r0[k], e, rtol=1e-6, atol=1e-7)


def _split_worker(rank, world, port, out_dir):
    """Early/late split of the exchange (the SH backward's outputs -- dmean3D, dsh -- arrive late): the collectives
    over the early runs go first, then the late ones; the result must be bitwise the single collective's."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hlgs_core.dp import FlatGradExchange, direct_grad
    grads = [torch.tensor(g) for g in _rank_grads(rank, world)]  # means3D, scales, rotations, opacities, shs
    params = [torch.zeros(g.shape, requires_grad=True) for g in grads]
    late_set = {0, 4}

    class Render(torch.autograd.Function):
        @staticmethod
        def forward(ctx, split, *ps):
            ctx.ps, ctx.split = ps, split
            return sum((p * 0).sum() for p in ps)

        @staticmethod
        def backward(ctx, _):
            outs = []
            for i, (p, g) in enumerate(zip(ctx.ps, grads)):
                d = direct_grad(p, late=ctx.split and i in late_set)
                d.copy_(g)
                outs.append(d)
            return (None,) + tuple(outs)

    ex = FlatGradExchange(params)
    res, ncoll = [], []
    for split in (True, False):
        for p in params:
            p.grad = None
        Render.apply(split, *params).backward()
        ex.allreduce()
        ncoll.append(ex.last_collectives)
        res.append([p.grad.clone() for p in params])
    ex.close()
    same = all(torch.equal(a, b) for a, b in zip(*res))
    np.savez(os.path.join(out_dir, f"s{rank}.npz"), *[t.numpy() for t in res[0]],
             flags=np.array([same, ncoll == [3, 1]]))
    dist.destroy_process_group()


def test_view_dp_early_late_split_gloo(tmp_path):
    world = 2
    port = _free_port()
    mp.spawn(_split_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    r0, r1 = np.load(tmp_path / "s0.npz"), np.load(tmp_path / "s1.npz")
    assert r0["flags"].all() and r1["flags"].all()
    sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
    expect = [(a + b) / 2 for a, b in zip(_rank_grads(0, world), _rank_grads(1, world))]
    for k, e in zip([f for f in r0.files if f != "flags"], expect):
        np.testing.assert_array_equal(r0[k], r1[k])
        np.testing.assert_allclose(r0[k], e, rtol=1e-6, atol=1e-7)
