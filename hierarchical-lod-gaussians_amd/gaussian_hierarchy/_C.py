"""`gaussian_hierarchy._C` LOD entry points on MI355X.

Signatures follow submodules/gaussianhierarchy/torch/torch_interface.h:36-95 as bound in ext.cpp:15-27:

    expand_to_size(nodes, boxes, size, viewpoint, viewdir, render_indices, parent_indices,
                   nodes_for_render_indices) -> int
    expand_to_size_dynamic(nodes, positions, scales, size, viewpoint, viewdir, render_indices,
                           parent_indices, nodes_for_render_indices) -> int
    get_interpolation_weights(indices, size, nodes, boxes, viewpoint, viewdir, ts, num_kids) -> None
    get_interpolation_weights_dynamic(indices, size, nodes, positions, scales, viewpoint, viewdir, ts,
                                      num_kids) -> None
    get_spt_cut_cuda(number_of_SPTs, gaussian_indices, SPT_starts, SPT_max, SPT_min, SPT_indices,
                     SPT_distances) -> (cut, counts_prefix)
    get_morton_indices(xyz, min, max, codes) -> None          (codes: int64, written in place)
    load_hierarchy(filename) -> (pos, shs (P,16,3), alpha (P,1), log-scales, rotations, nodes (N,7), boxes (N,2,4))
    load_dynamic_hierarchy(filename) -> (pos, shs (P,(deg+1)^2,3), alpha (P,1), log-scales, rotations, nodes (P,6))
    write_hierarchy(filename, pos, shs, opacities, log_scales, rotations, nodes, boxes) -> None
    write_dynamic_hierarchy(filename, pos, shs, opacities, log_scales, rotations, nodes, SH_degree) -> None
    expand_to_target(nodes, target) -> int32 indices

The file functions run in libhlgs.so's host code (no Eigen) and return CPU tensors, as the reference does.

Output buffers are caller-allocated, full-size and written in place; only the first `count` entries are
valid (render_hierarchy.py:36-40, 68-69).  The reference reads `viewdir` on the host for
expand_to_size[_dynamic] and both `viewpoint` and `viewdir` on the host for the weights
(torch_interface.cpp:163-164, 188-189, 216-217, 240-241); this binding accepts either device, copying
the three floats where the kernels need them.
"""
import ctypes as C

import torch

from hlgs_core import _lib as L


def _host3(t):
    v = t.detach().reshape(-1)[:3].to("cpu", torch.float32)
    return L.f3(v.tolist())


def _i32(t):
    if t.dtype != torch.int32:
        raise RuntimeError("expected an int32 tensor")
    return t.contiguous()


def _f32(t):
    return t.contiguous().float()


def _scratch(nbytes, dev):
    return torch.empty((int(nbytes),), dtype=torch.uint8, device=dev)


def _writable(t, name):
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous (it is written in place)")
    return t


def expand_to_size_dynamic(nodes, positions, scales, size, viewpoint, viewdir, render_indices, parent_indices,
                           nodes_for_render_indices):
    lib = L.load()
    nd, pos, sc = _i32(nodes), _f32(positions), _f32(scales)
    L.require_gpu(nd, pos, sc, render_indices)
    N = nd.size(0)
    vp = viewpoint.detach().reshape(-1)[:3].to(device=nd.device, dtype=torch.float32).contiguous()
    count = C.c_int(0)
    scratch = _scratch(lib.hlgs_lod_scratch_size(N), nd.device)
    L.check(lib.hlgs_expand_to_size_dynamic(N, float(size), L.ptr(nd), L.ptr(pos), L.ptr(sc), L.ptr(vp),
                                            _host3(viewdir), L.ptr(_writable(render_indices, "render_indices")),
                                            L.ptr(_writable(parent_indices, "parent_indices")),
                                            L.ptr(_writable(nodes_for_render_indices, "nodes_for_render_indices")),
                                            L.ptr(scratch), C.byref(count), L.stream()))
    return int(count.value)


def get_interpolation_weights_dynamic(indices, size, nodes, positions, scales, viewpoint, viewdir, ts, num_kids):
    lib = L.load()
    ix, nd, pos, sc = _i32(indices), _i32(nodes), _f32(positions), _f32(scales)
    L.require_gpu(ix, nd, pos, sc, ts)
    L.check(lib.hlgs_get_interpolation_weights_dynamic(ix.size(0), L.ptr(ix), float(size), L.ptr(nd), L.ptr(pos),
                                                       L.ptr(sc), _host3(viewpoint), _host3(viewdir),
                                                       L.ptr(_writable(ts, "ts")), L.ptr(_writable(num_kids, "num_kids")),
                                                       L.stream()))


def expand_to_size(nodes, boxes, size, viewpoint, viewdir, render_indices, parent_indices, nodes_for_render_indices):
    lib = L.load()
    nd, bx = _i32(nodes), _f32(boxes)
    L.require_gpu(nd, bx, render_indices)
    N = nd.size(0)
    vp = viewpoint.detach().reshape(-1)[:3].to(device=nd.device, dtype=torch.float32).contiguous()
    count = C.c_int(0)
    scratch = _scratch(lib.hlgs_lod_scratch_size(N), nd.device)
    L.check(lib.hlgs_expand_to_size(N, float(size), L.ptr(nd), L.ptr(bx), L.ptr(vp), _host3(viewdir),
                                    L.ptr(_writable(render_indices, "render_indices")),
                                    L.ptr(_writable(parent_indices, "parent_indices")),
                                    L.ptr(_writable(nodes_for_render_indices, "nodes_for_render_indices")),
                                    L.ptr(scratch), C.byref(count), L.stream()))
    return int(count.value)


def get_interpolation_weights(indices, size, nodes, boxes, viewpoint, viewdir, ts, num_kids):
    lib = L.load()
    ix, nd, bx = _i32(indices), _i32(nodes), _f32(boxes)
    L.require_gpu(ix, nd, bx, ts)
    L.check(lib.hlgs_get_interpolation_weights(ix.size(0), L.ptr(ix), float(size), L.ptr(nd), L.ptr(bx),
                                               _host3(viewpoint), _host3(viewdir), L.ptr(_writable(ts, "ts")),
                                               L.ptr(_writable(num_kids, "num_kids")), L.stream()))


def get_spt_cut_cuda(number_of_SPTs, gaussian_indices, SPT_starts, SPT_max, SPT_min, SPT_indices, SPT_distances,
                     compat=True):
    """SPT cut (runtime_switching.cu:878-994).  compat=True reproduces the reference exactly, including its
    interval-boundary attribution and the dropping of Gaussian index 0; compat=False
    gives the intended semantics of scene/gaussian_model.py:163-181."""
    lib = L.load()
    s = int(number_of_SPTs)
    gi, st, mx, mn = _i32(gaussian_indices), _i32(SPT_starts), _f32(SPT_max), _f32(SPT_min)
    si, sd = _i32(SPT_indices), _f32(SPT_distances)
    L.require_gpu(gi, st, mx, mn, si, sd)
    dev = gi.device
    counts_prefix = torch.zeros((s,), dtype=torch.int32, device=dev)
    if s == 0:
        return torch.zeros((0,), dtype=torch.int32, device=dev), counts_prefix
    scratch = _scratch(lib.hlgs_spt_scratch_size(s), dev)
    ncand = C.c_int(0)
    stream = L.stream()
    L.check(lib.hlgs_spt_cut_prepare(s, L.ptr(st), L.ptr(mx), L.ptr(si), L.ptr(sd), L.ptr(scratch), C.byref(ncand),
                                     stream))
    n = int(ncand.value)
    work = _scratch(lib.hlgs_spt_work_size(n), dev)
    cut = torch.empty((max(n, 1),), dtype=torch.int32, device=dev)
    count = C.c_int(0)
    L.check(lib.hlgs_spt_cut_finish(s, mx.size(0), n, L.ptr(gi), L.ptr(st), L.ptr(mn), L.ptr(si), L.ptr(sd),
                                    int(bool(compat)), L.ptr(scratch), L.ptr(work), L.ptr(cut), L.ptr(counts_prefix),
                                    C.byref(count), stream))
    return cut[:int(count.value)].clone(), counts_prefix


def lod_interp_forward(S, ridx, pidx, w, means, scales, rots, opac, shs):
    lib = L.load()
    n = int(ridx.size(0))
    dev = means.device
    M3 = int(shs[0].numel()) if (shs is not None and shs.numel()) else 0
    f32 = dict(dtype=torch.float32, device=dev)
    out_m = torch.empty((S + n, 3), **f32)
    out_s = torch.empty((S + n, 3), **f32)
    out_r = torch.empty((S + n, 4), **f32)
    out_o = torch.empty((S + n, 1), **f32)
    out_sh = torch.empty((S + n,) + tuple(shs.shape[1:]), **f32) if M3 else None
    L.check(lib.hlgs_lod_interp_forward(int(S), n, M3, L.ptr(ridx), L.ptr(pidx), L.ptr(w), L.ptr(means),
                                        L.ptr(scales), L.ptr(rots), L.ptr(opac), L.ptr(shs) if M3 else None,
                                        L.ptr(out_m), L.ptr(out_s), L.ptr(out_r), L.ptr(out_o),
                                        L.ptr(out_sh) if M3 else None, L.stream()))
    return out_m, out_s, out_r, out_o, out_sh


def lod_interp_backward(S, ridx, pidx, w, rots, P, g_m, g_s, g_r, g_o, g_sh, sh_shape):
    lib = L.load()
    n = int(ridx.size(0))
    dev = rots.device
    f32 = dict(dtype=torch.float32, device=dev)
    d_m = torch.empty((P, 3), **f32)  # written completely by the kernel
    d_s = torch.empty((P, 3), **f32)
    d_r = torch.empty((P, 4), **f32)
    d_o = torch.empty((P, 1), **f32)
    M3 = 0
    d_sh = None
    if sh_shape is not None:
        d_sh = torch.empty((P,) + tuple(sh_shape[1:]), **f32)
        M3 = int(d_sh[0].numel()) if P else 0
    scratch = _scratch(lib.hlgs_lod_interp_scratch_size(int(P), n), dev)
    L.check(lib.hlgs_lod_interp_backward(int(P), int(S), n, M3, L.ptr(ridx), L.ptr(pidx), L.ptr(w), L.ptr(rots),
                                         L.ptr(g_m), L.ptr(g_s), L.ptr(g_r), L.ptr(g_o),
                                         L.ptr(g_sh) if M3 else None, L.ptr(d_m), L.ptr(d_s), L.ptr(d_r), L.ptr(d_o),
                                         L.ptr(d_sh) if M3 else None, L.ptr(scratch), L.stream()))
    return d_m, d_s, d_r, d_o, d_sh


def get_morton_indices(xyz, min, max, codes):  # noqa: A002  (the reference's parameter names)
    """Morton code per position inside the [min, max] box, written into the int64 tensor `codes`
    (morton.cu:9-58)."""
    lib = L.load()
    p = _f32(xyz)
    mn = min.detach().reshape(-1)[:3].to(device=p.device, dtype=torch.float32).contiguous()
    mx = max.detach().reshape(-1)[:3].to(device=p.device, dtype=torch.float32).contiguous()
    if codes.dtype != torch.int64 or not codes.is_contiguous():
        raise RuntimeError("codes must be a contiguous int64 tensor")
    L.require_gpu(p, mn, mx, codes)
    L.check(lib.hlgs_morton_codes(p.size(0), L.ptr(p), L.ptr(mn), L.ptr(mx), L.ptr(codes), L.stream()))


def _info(filename, dynamic):
    info = L.HierInfo()
    L.check(L.load().hlgs_hier_info_read(str(filename).encode(), int(dynamic), C.byref(info)))
    return info


def _host_f32(t, *shape):
    return t.detach().to("cpu", torch.float32).contiguous().reshape(*shape)


def load_hierarchy(filename):
    """LoadHierarchy (torch_interface.cpp:9-40): full or binary16 .hier -> CPU tensors
    (pos (P,3), shs (P,16,3), alpha (P,1), log-scales (P,3), rotations (P,4), nodes (N,7) int32, boxes (N,2,4))."""
    info = _info(filename, False)
    P, N = info.G, info.N
    f = lambda *sh: torch.empty(sh, dtype=torch.float32)  # noqa: E731
    pos, shs, alpha, scales, rot, boxes = f(P, 3), f(P, 16, 3), f(P, 1), f(P, 3), f(P, 4), f(N, 2, 4)
    nodes = torch.empty((N, 7), dtype=torch.int32)
    L.check(L.load().hlgs_hier_load(str(filename).encode(), L.ptr(pos), L.ptr(rot), L.ptr(scales), L.ptr(alpha),
                                    L.ptr(shs), L.ptr(nodes), L.ptr(boxes)))
    return pos, shs, alpha, scales, rot, nodes, boxes


def load_dynamic_hierarchy(filename):
    """LoadDynamicHierarchy (torch_interface.cpp:43-74): .dhier -> CPU tensors (pos (P,3), shs (P,(deg+1)^2,3),
    alpha (P,1), log-scales (P,3), rotations (P,4), nodes (P,6) int32 HierarchyNode rows)."""
    info = _info(filename, True)
    P = info.G
    f = lambda *sh: torch.empty(sh, dtype=torch.float32)  # noqa: E731
    pos, shs, alpha, scales, rot = f(P, 3), f(P, (info.sh_degree + 1) ** 2, 3), f(P, 1), f(P, 3), f(P, 4)
    nodes = torch.empty((P, 6), dtype=torch.int32)
    L.check(L.load().hlgs_dhier_load(str(filename).encode(), L.ptr(pos), L.ptr(rot), L.ptr(scales), L.ptr(alpha),
                                     L.ptr(shs), L.ptr(nodes)))
    return pos, shs, alpha, scales, rot, nodes


def write_hierarchy(filename, pos, shs, opacities, log_scales, rotations, nodes, boxes):
    """WriteHierarchy (torch_interface.cpp:77-104): the binary16 .hier layout (the reference writer's default)."""
    P, N = pos.size(0), nodes.size(0)
    a = [_host_f32(pos, P, 3), _host_f32(shs, P, 48), _host_f32(opacities, P), _host_f32(log_scales, P, 3),
         _host_f32(rotations, P, 4)]
    nd = nodes.detach().to("cpu", torch.int32).contiguous().reshape(N, 7)
    bx = _host_f32(boxes, N, 8)
    L.check(L.load().hlgs_hier_write(str(filename).encode(), P, N, *[L.ptr(x) for x in a], L.ptr(nd), L.ptr(bx), 1))


def write_dynamic_hierarchy(filename, pos, shs, opacities, log_scales, rotations, nodes, SH_degree):
    """WriteDynamicHierarchy (torch_interface.cpp:107-133): the first (deg+1)^2 x 3 floats of every SH row of
    the contiguous `shs` are written (hierarchy_writer.cpp:133-150 writes that many bytes from its start)."""
    P, N = pos.size(0), nodes.size(0)
    deg = int(SH_degree)
    flat = shs.detach().to("cpu", torch.float32).contiguous().reshape(-1)
    need = P * 3 * (deg + 1) ** 2
    if flat.numel() < need:
        raise RuntimeError("shs holds fewer coefficients than SH_degree needs")
    a = [_host_f32(pos, P, 3), flat[:need].contiguous(), _host_f32(opacities, P), _host_f32(log_scales, P, 3),
         _host_f32(rotations, P, 4)]
    nd = nodes.detach().to("cpu", torch.int32).contiguous().reshape(N, 6)
    L.check(L.load().hlgs_dhier_write(str(filename).encode(), P, N, *[L.ptr(x) for x in a], L.ptr(nd), deg))


def expand_to_target(nodes, target):
    """ExpandToTarget (torch_interface.cpp:136-146): Gaussian indices of the static hierarchy cut at depth
    `target` (traversal.cpp:15-39) as a CPU int32 tensor."""
    lib = L.load()
    nd = nodes.detach().to("cpu", torch.int32).contiguous()
    N = nd.size(0)
    count = C.c_int(0)
    L.check(lib.hlgs_expand_to_target(N, L.ptr(nd), int(target), None, 0, C.byref(count)))
    out = torch.empty((count.value,), dtype=torch.int32)
    L.check(lib.hlgs_expand_to_target(N, L.ptr(nd), int(target), L.ptr(out), count.value, C.byref(count)))
    return out
