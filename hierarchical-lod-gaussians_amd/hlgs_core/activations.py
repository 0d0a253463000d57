"""The parameter activations of the training step on the HIP path (libhlgs.so, csrc/act.hip).

    activate(opacity_raw, scaling_raw, rotation_raw) -> (opacity, scales, rotations)

is GaussianModel.get_opacity / get_scaling / get_rotation (scene/gaussian_model.py:44-56: sigmoid, exp,
torch.nn.functional.normalize) over every resident row in one kernel, and their backward in one more; torch runs
them as about ten elementwise and reduction kernels per step (train_post.py's render of the cached rows).
"""
import torch

from hlgs_core import _lib as L


class _Activate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, op_raw, sc_raw, rot_raw):
        n = op_raw.shape[0]
        if sc_raw.shape != (n, 3) or rot_raw.shape != (n, 4) or op_raw.numel() != n:
            raise RuntimeError("activate: expected opacity (n, 1), scaling (n, 3) and rotation (n, 4) rows")
        o_r, s_r, r_r = (t.detach().contiguous().float() for t in (op_raw, sc_raw, rot_raw))
        L.require_gpu(o_r, s_r, r_r)
        op, sc, rot = torch.empty_like(o_r), torch.empty_like(s_r), torch.empty_like(r_r)
        L.check(L.load().hlgs_activate_forward(n, L.ptr(o_r), L.ptr(s_r), L.ptr(r_r), L.ptr(op), L.ptr(sc),
                                               L.ptr(rot), L.stream()))
        ctx.save_for_backward(op, sc, r_r)
        ctx.set_materialize_grads(False)
        return op.view(op_raw.shape), sc, rot

    @staticmethod
    def backward(ctx, g_op, g_sc, g_rot):
        op, sc, r_r = ctx.saved_tensors
        n = r_r.shape[0]
        g = [None if t is None else t.contiguous().float() for t in (g_op, g_sc, g_rot)]
        d = [None if t is None else torch.empty_like(s) for t, s in zip(g, (op, sc, r_r))]
        L.check(L.load().hlgs_activate_backward(n, L.ptr(op), L.ptr(sc), L.ptr(r_r), *(L.ptr(t) for t in g),
                                                *(L.ptr(t) for t in d), L.stream()))
        if d[0] is not None:
            d[0] = d[0].view(op.shape)
        return tuple(d)


def activate(opacity_raw, scaling_raw, rotation_raw):
    """(sigmoid(opacity_raw), exp(scaling_raw), normalize(rotation_raw)) in one HIP pass, differentiable."""
    return _Activate.apply(opacity_raw, scaling_raw, rotation_raw)
