"""View-data-parallel gradient exchange.

Each rank holds a full replica of the Gaussian parameters and renders its own training view; the only
collective is one all-reduce of the Gaussian gradients (RCCL over xGMI with backend "nccl", gloo on
CPU).  Gradients are packed into one flat fp32 buffer so RCCL moves a few large messages instead of
one per parameter tensor, then averaged (the reference trains one view per step; G views per step is
an effective batch of G).
"""
import weakref

import torch
import torch.distributed as dist


_AVG_OK = [True]  # ReduceOp.AVG accepted by the backend (flips once if it is not)

# Parameters whose gradient the rasterizer backward may write straight into an exchange's flat buffer:
# data_ptr -> (weakref to the parameter, weakref to its exchange, index in the exchange).  Weak references, so a
# parameter replaced by densification or by the SPT cache (new tensors every step) does not keep its old storage or
# the exchange's flat buffer alive; an exchange that is garbage-collected drops its own entries.  The view is made
# per call: autograd adopts a returned gradient only while nothing else holds a reference to that tensor.
_DIRECT = {}


def _drop_entries(keys, token):
    for k in keys:
        e = _DIRECT.get(k)
        if e is not None and e[3] == token:
            del _DIRECT[k]


def direct_grad(t, late=False):
    """Destination for the gradient of input tensor `t`, or None.

    Used by the rasterizer backward (diff_gaussian_rasterization._C, alt_gaussian_rasterization._C): when `t` is a
    parameter registered by a FlatGradExchange(direct=True) and its .grad is unset, the backward writes the
    gradient into the exchange's flat buffer, autograd adopts that tensor as .grad (it steals a fresh leaf
    gradient instead of copying it), and the all-reduce finds it already packed.  With .grad set (accumulation)
    a fresh tensor is returned as usual, so an in-place `.grad +=` never aliases its own input.

    The view is handed out at most once per exchange round (until allreduce() / unpack() / release()): two
    rasterizer backwards of one autograd pass both see .grad unset, because AccumulateGrad runs only after both
    finish; the second one gets None, so autograd sums two distinct tensors instead of the buffer with itself.

    late: the backward completes this output on its late stream (the SH backward, see late_stream_for)."""
    e = _DIRECT.get(t.data_ptr()) if t is not None and t.numel() else None
    if e is None:
        return None
    p, ex = e[0](), e[1]()
    if p is None or ex is None:
        _DIRECT.pop(t.data_ptr(), None)
        return None
    i = e[2]
    if ex.adopted[i] and p.grad is None:
        # the view handed out in an earlier backward was adopted as .grad and then dropped (set to None) without
        # allreduce() / unpack() / release(): that round was abandoned, so this backward starts a new one
        ex._stale_round()
    if ex.claimed[i]:
        # a second gradient for this parameter in one autograd pass (e.g. two renders of the same leaves): autograd
        # sums it with the view on the current stream, so the late kernels writing the view must be done first
        ex.join()
        return None
    if p.grad is not None or p.shape != t.shape or p.dtype != t.dtype or ex.flat.device != t.device:
        return None
    ex.claimed[i] = True
    ex.late[i] = bool(late)
    v = ex.flat[ex.offsets[i]:ex.offsets[i] + ex.numels[i]].view_as(p)
    _VIEWS[v.data_ptr()] = weakref.ref(ex)
    return v


def _adopt_hook(exref, i):
    """Post-accumulate-grad hook: records that parameter i's .grad is the exchange's view (so a later backward that
    finds .grad reset to None knows the round was abandoned, see direct_grad)."""
    def hook(p):
        ex = exref()
        if ex is not None and ex.claimed[i] and p.grad is not None and \
                p.grad.data_ptr() == ex.flat.data_ptr() + 4 * ex.offsets[i]:
            ex.adopted[i] = True
    return hook


# data_ptr of a view direct_grad handed out -> weak reference to its exchange (late_stream_for's lookup)
_VIEWS = {}


def late_stream_for(*views):
    """The stream on which the rasterizer backward may run its late kernels (hlgs_rasterize_backward_split), or None.

    Only when every late output (non-empty views: dmean3D, dsh, ddc) is a direct_grad view of one exchange built with
    overlap=True: then autograd's only consumer of those tensors is AccumulateGrad adopting them (no kernel), and the
    exchange joins the late stream before its collective over them (FlatGradExchange.allreduce / join)."""
    exs = set()
    for v in views:
        if v is None or v.numel() == 0:
            continue
        r = _VIEWS.get(v.data_ptr())
        ex = r() if r is not None else None
        if ex is None or ex.late_stream is None or not ex.flat.data_ptr() <= v.data_ptr() < ex.flat.data_ptr() + \
                4 * ex.flat.numel():
            return None
        exs.add(id(ex))
        one = ex
    return one.late_stream if len(exs) == 1 else None


def note_late_work(stream, tensors):
    """After a split backward: the exchange whose late stream this is joins it before reading the late gradients;
    every tensor the late kernels touch is kept from reuse by the caching allocator until they finish."""
    for t in tensors:
        if isinstance(t, torch.Tensor) and t.is_cuda and t.numel():
            t.record_stream(stream)
    ev = torch.cuda.Event()
    ev.record(stream)
    for r in list(_VIEWS.values()):
        ex = r()
        if ex is not None and ex.late_stream is stream:
            ex.pending = ev


class FlatGradExchange:
    """Pack -> all-reduce -> hand back, for a fixed list of parameter tensors.

    When the rasterizer backward has written the gradients straight into the flat buffer (direct_grad), there is
    nothing to pack and one collective covers the whole buffer.  Otherwise the buffer is cut into buckets; each
    bucket's all-reduce is launched (async) as soon as its slice is packed, so packing bucket k+1 overlaps the
    transfer of bucket k.  RCCL averages in the collective
    (ReduceOp.AVG), and afterwards every parameter's .grad is a view into the reduced buffer -- no unpack copy
    and no separate scaling pass.  64 MB buckets keep each ring well above its bandwidth knee on xGMI while
    leaving several buckets to pipeline for a 1M-Gaussian model (236 MB of fp32 gradients).
    """

    def __init__(self, params, bucket_bytes=64 << 20, average=True, group=None, direct=True, overlap=False):
        self.params = list(params)
        self.numels = [p.numel() for p in self.params]
        self.offsets = []
        off = 0
        for n in self.numels:
            self.offsets.append(off)
            off += n
        total = off
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.flat = torch.empty(total, dtype=torch.float32, device=dev)
        self.average = average
        self.group = group
        per = max(1, bucket_bytes // 4)
        self.buckets = [(s, min(s + per, total)) for s in range(0, total, per)]
        self.direct = []
        self.claimed = [False] * len(self.params)
        self.late = [False] * len(self.params)
        self.adopted = [False] * len(self.params)  # a handed-out view became .grad (post-accumulate hook)
        # overlap (opt-in): the rasterizer backward runs its SH backward on late_stream (hlgs_rasterize_backward_split),
        # so the collective over the gradients that are final before it (opacity, scale, rotation) starts while it
        # runs.  Then means3D / shs / dc .grad are complete on the current stream only after allreduce(), join() or
        # release(); code that reads them in between (clipping, NaN checks, densification statistics) calls join()
        # first.  A second gradient into those leaves from another rasterizer call in the same backward is ordered
        # by direct_grad (it joins); one from any other loss term is not, so overlap=True requires that the
        # rasterizer be the only consumer of means3D / shs / dc in the loss.
        self.late_stream = torch.cuda.Stream(device=dev) if (overlap and direct and dev.type == "cuda") else None
        self.pending = None  # event on late_stream after the last split backward
        self._token = object()
        self._hooks = []
        self._warned = False
        if direct:
            me = weakref.ref(self)
            for i, p in enumerate(self.params):
                if p.is_contiguous() and p.dtype == torch.float32:
                    _DIRECT[p.data_ptr()] = (weakref.ref(p), me, i, self._token)
                    self.direct.append(p.data_ptr())
                    if p.requires_grad and hasattr(p, "register_post_accumulate_grad_hook"):
                        self._hooks.append(p.register_post_accumulate_grad_hook(_adopt_hook(me, i)))
        self._finalizer = weakref.finalize(self, _drop_entries, list(self.direct), self._token)

    def close(self):
        """Stop offering the flat buffer to the rasterizer backward.  Rebuild the exchange (and close the old one)
        whenever the parameter tensors are replaced: entries are keyed by storage address."""
        self._finalizer()
        self.direct = []
        for h in self._hooks:
            h.remove()
        self._hooks = []

    def _stale_round(self):
        if not self._warned:
            import warnings
            warnings.warn("FlatGradExchange: gradients were reset without allreduce()/unpack()/release(); starting a "
                          "new exchange round (call release() after a backward whose gradients are not exchanged)",
                          RuntimeWarning, stacklevel=3)
            self._warned = True
        self.release()

    def join(self):
        """Order the current stream after the late kernels of the last split backward (the gradients they complete
        -- dmean3D, dsh, ddc -- are readable on the current stream afterwards).  allreduce() joins by itself."""
        if self.pending is not None:
            torch.cuda.current_stream(self.flat.device).wait_event(self.pending)
            self.pending = None

    def release(self):
        """End the exchange round without a collective: the flat buffer may be handed out again."""
        self.join()
        self.claimed = [False] * len(self.params)
        self.late = [False] * len(self.params)
        self.adopted = [False] * len(self.params)

    def _pack_range(self, a, b):
        for p, off, n in zip(self.params, self.offsets, self.numels):
            lo, hi = max(a, off), min(b, off + n)
            if lo >= hi:
                continue
            dst = self.flat[lo:hi]
            if p.grad is None:
                dst.zero_()
            else:
                src = p.grad.reshape(-1)[lo - off:hi - off]
                if src.data_ptr() != dst.data_ptr():
                    dst.copy_(src)

    def pack(self):
        self._pack_range(0, self.flat.numel())

    def unpack(self):
        for p, off, n in zip(self.params, self.offsets, self.numels):
            p.grad = self.flat[off:off + n].view_as(p)
        self.release()

    def allreduce(self):
        """All-reduce every parameter's .grad across the process group (mean if average, else sum)."""
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            self.release()
            return
        world = dist.get_world_size(self.group)
        native_avg = self.average and dist.get_backend(self.group) == "nccl" and _AVG_OK[0]
        works = []
        # gradients the backward already wrote into the flat buffer need no packing, so there is nothing for the
        # buckets to overlap with: one collective over the whole buffer saves the per-call startup of the others
        base = self.flat.data_ptr()
        in_place = all(p.grad is not None and p.grad.data_ptr() == base + 4 * off
                       for p, off in zip(self.params, self.offsets))
        split = in_place and any(self.late) and not all(self.late)
        if split:
            # the early gradients' runs first (their backward is done on this stream), then the join, then the late
            # runs: elementwise the same reduction as one collective over the whole buffer
            runs = []
            for i, (off, n) in enumerate(zip(self.offsets, self.numels)):
                if runs and runs[-1][2] == self.late[i] and runs[-1][1] == off:
                    runs[-1][1] = off + n
                else:
                    runs.append([off, off + n, self.late[i]])
            spans = [(a, b) for a, b, lt in runs if not lt] + [None] + [(a, b) for a, b, lt in runs if lt]
        else:
            self.join()
            spans = [(0, self.flat.numel())] if in_place else self.buckets
        self.last_collectives = sum(1 for sp in spans if sp is not None)
        for sp in spans:
            if sp is None:
                self.join()
                continue
            a, b = sp
            self._pack_range(a, b)
            if native_avg:
                try:
                    works.append(dist.all_reduce(self.flat[a:b], op=dist.ReduceOp.AVG, group=self.group,
                                                 async_op=True))
                    continue
                except (RuntimeError, ValueError):  # a collective library without averaging: sum, scale below
                    if works:  # the op is rejected at its first use, before any collective went out
                        raise
                    _AVG_OK[0] = native_avg = False
            works.append(dist.all_reduce(self.flat[a:b], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        for w in works:
            w.wait()
        if self.average and not native_avg:
            self.flat.mul_(1.0 / world)
        self.unpack()
