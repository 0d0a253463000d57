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


def _sh_basis_np(dirs, ncoef):
    """Real SH basis of the reference's colour (utils/sh_utils.py constants, forward.cu:20-67) at unit directions
    (N, 3), degrees up to 3: (N, ncoef).  Test restatement of what hlgs_sh_grad_from_colour evaluates."""
    C0, C1 = 0.28209479177387814, 0.4886025119029199
    C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
    C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
          1.445305721320277, -0.5900435899266435]
    x, y, z = dirs[:, 0], dirs[:, 1], dirs[:, 2]
    xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
    b = [np.full_like(x, C0), -C1 * y, C1 * z, -C1 * x,
         C2[0] * xy, C2[1] * yz, C2[2] * (2 * zz - xx - yy), C2[3] * xz, C2[4] * (xx - yy),
         C3[0] * y * (3 * xx - yy), C3[1] * xy * z, C3[2] * y * (4 * zz - xx - yy),
         C3[3] * z * (2 * zz - 3 * xx - 3 * yy), C3[4] * x * (4 * zz - xx - yy), C3[5] * z * (xx - yy),
         C3[6] * x * (xx - 3 * yy)]
    return np.stack(b[:ncoef], 1)


def _rank_colour_grads(rank, world):
    """The rank's dL/dRGB with the SH clamp mask applied (what the factored backward hands the exchange), its camera
    centre, and the oracle's full gradients of the same view."""
    from hlgs_core import synthetic as S
    from oracle import oracle as O
    cam = S.ring_camera(64, 48, rank, world)
    sc = S.make_gaussians(300, 1, S.make_camera(64, 48), seed=0)
    fr = O.forward(sc, S.cam_numpy(cam))
    g = O.backward(fr, sc, *S.upstream_grads(64, 48, seed=1 + rank))
    cl = fr.clamped[:, None] >> np.arange(3)[None, :] & 1
    drgb = np.where((cl == 0) & (fr.radii[:, None] > 0), g["dcolor"], 0.0).astype(np.float32)
    return drgb, S.cam_numpy(cam)["campos"].astype(np.float32), g


def _factor_worker(rank, world, port, out_dir):
    """Colour-factored exchange plumbing over gloo: the SH leaf leaves the flat buffer, each rank's [campos | dL/dRGB]
    row is all-gathered and the SH gradient rebuilt from the rows in rank order (the HIP rebuild,
    hlgs_sh_grad_from_colour, is checked on the GPU by tests/test_gpu_dp.py; here a numpy restatement stands in)."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hlgs_core import dp
    from hlgs_core.dp import FlatGradExchange, colour_factor
    drgb, campos, g = _rank_colour_grads(rank, world)
    grads = [torch.tensor(g[k]) for k in ("dmean3D", "dscale", "drot", "dopacity")]
    params = [torch.zeros(x.shape, requires_grad=True) for x in grads]
    means = torch.tensor(_rank_means())
    shs = torch.zeros(g["dsh"].shape, requires_grad=True)

    def rebuild(cf, V):
        P = cf.means.shape[0]
        rows = cf.gathered.numpy()
        m = cf.means.detach().numpy().astype(np.float64)
        acc = np.zeros((P, 4, 3))
        for v in range(V):
            d = m - rows[v, :3].astype(np.float64)
            acc += _sh_basis_np(d / np.linalg.norm(d, axis=1, keepdims=True), 4)[:, :, None] * \
                rows[v, 4:].reshape(P, 1, 3)
        cf.sh_buf.copy_(torch.tensor(acc / V, dtype=torch.float32))
    dp.rebuild_sh = rebuild

    ex = FlatGradExchange(params + [shs], colour_factor=dict(means=means, sh=shs))
    assert all(p is not shs for p in ex.params)  # the SH leaf is not all-reduced
    fac = colour_factor(shs)
    fac[0].copy_(torch.tensor(drgb))
    fac[3](torch.tensor(campos), 1, 0)
    for p, x in zip(params, grads):
        p.grad = x.clone()
    shs.grad = fac[1]  # what autograd does with the view the backward returns
    ex.allreduce()
    ok = shs.grad.data_ptr() == ex.cf.sh_buf.data_ptr() and not ex.cf.written
    ex.close()
    np.savez(os.path.join(out_dir, f"f{rank}.npz"), *[p.grad.numpy() for p in params], shs.grad.numpy(),
             flags=np.array([ok]))
    dist.destroy_process_group()


def _rank_means():
    from hlgs_core import synthetic as S
    return S.make_gaussians(300, 1, S.make_camera(64, 48), seed=0)["means3D"]


def test_view_dp_colour_factored_sh_gloo(tmp_path):
    world = 2
    port = _free_port()
    mp.spawn(_factor_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    r0, r1 = np.load(tmp_path / "f0.npz"), np.load(tmp_path / "f1.npz")
    assert r0["flags"].all() and r1["flags"].all()
    sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
    g0, g1 = _rank_colour_grads(0, world)[2], _rank_colour_grads(1, world)[2]
    expect = [(g0[k] + g1[k]) / 2 for k in ("dmean3D", "dscale", "drot", "dopacity", "dsh")]
    files = [f for f in r0.files if f != "flags"]
    for k, e in zip(files, expect):
        np.testing.assert_array_equal(r0[k], r1[k])
        np.testing.assert_allclose(r0[k], e, rtol=1e-5, atol=1e-7)
