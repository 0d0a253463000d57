"""View-data-parallel gradient exchange.

Each rank holds a full replica of the Gaussian parameters and renders its own training view; the only
collective is one all-reduce of the Gaussian gradients (RCCL over xGMI with backend "nccl", gloo on
CPU).  Gradients are packed into one flat fp32 buffer so RCCL moves a few large messages instead of
one per parameter tensor, then averaged (the reference trains one view per step; G views per step is
an effective batch of G).

Colour-factored SH exchange (colour_factor=...).  One view's SH gradient is an outer product per Gaussian,
dL/dsh[c] = basis_c(view direction) * dL/dRGB (computeColorFromSH backward, backward.cu:23-142), so a rank does not
need the other ranks' (D+1)^2 x 3 SH rows, only their 3-float colour gradients and camera centres: the SH parameters
leave the all-reduce, the rasterizer backward writes dL/dRGB into the exchange (hlgs_grads.drgb), one all-gather moves
those rows, and every rank rebuilds the averaged SH gradient with hlgs_sh_grad_from_colour -- the same products,
summed in rank order, identical on every rank.  At SH degree 3 a Gaussian's exchange drops from 59 all-reduced floats
(2 (N-1)/N x 236 bytes over each GPU's links) to 11 all-reduced plus 3 gathered per rank.
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


class _ColourFactor:
    """Per-exchange state of the colour-factored SH gradient: this rank's row [campos x, y, z, pad | dL/dRGB P x 3],
    the gathered rows of all ranks, and the buffers the rebuilt SH (and alt-variant dc) gradients live in."""

    def __init__(self, means, sh, dc, world, dev):
        self.means, self.sh, self.dc = means, sh, dc
        P = means.shape[0]
        self.row = P * 3 + 4
        self.mine = torch.zeros(self.row, dtype=torch.float32, device=dev)
        self.gathered = torch.empty((max(1, world), self.row), dtype=torch.float32, device=dev)
        self.sh_buf = torch.empty(sh.shape, dtype=torch.float32, device=dev)
        self.dc_buf = torch.empty(dc.shape, dtype=torch.float32, device=dev) if dc is not None else None
        self.written = False  # a backward wrote this round's row
        self.D = 0
        self.variant = 0


# SH parameter data_ptr -> (weak ref to the parameter, weak ref to its exchange)
_FACTOR = {}


def colour_factor(sh, dc=None):
    """For the rasterizer backward: (drgb view P x 3, dsh destination, ddc destination or None, record) when `sh` is the
    SH parameter of a colour-factored exchange whose round has not produced its row yet, else None.  The backward writes
    dL/dRGB into drgb (hlgs_grads.drgb) instead of dsh / ddc and calls record(campos, degree, variant); the returned
    dsh / ddc views become the leaves' .grad and are filled by the exchange's allreduce()."""
    e = _FACTOR.get(sh.data_ptr()) if sh is not None and sh.numel() else None
    if e is None:
        return None
    p, ex = e[0](), e[1]()
    if p is None or ex is None or ex.cf is None:
        _FACTOR.pop(sh.data_ptr(), None)
        return None
    cf = ex.cf
    if cf.written or p.grad is not None or p.shape != sh.shape or (dc is not None) != (cf.dc is not None) or \
            (dc is not None and cf.dc.grad is not None):
        return None
    P = cf.means.shape[0]
    if sh.shape[0] != P or (dc is not None and dc.shape[0] != P):
        return None

    def record(campos, degree, variant):
        cf.mine[:3].copy_(campos.reshape(-1)[:3])
        cf.D, cf.variant, cf.written = int(degree), int(variant), True
    # fresh views per call, so autograd adopts them as .grad (it steals a gradient nothing else references)
    return (cf.mine[4:].view(P, 3), cf.sh_buf.view(cf.sh.shape), cf.dc_buf.view(cf.dc.shape) if dc is not None else None,
            record)


def _check_factored(cf):
    """The rebuilt gradient reaches the leaves only if their .grad is the exchange's buffer (autograd adopted the views
    colour_factor handed out): a second gradient into those leaves in the same backward (another rasterizer call, another
    loss term) makes autograd sum into a new tensor, which the factored exchange cannot complete."""
    for t, buf in ((cf.sh, cf.sh_buf), (cf.dc, cf.dc_buf)):
        if t is not None and (t.grad is None or t.grad.data_ptr() != buf.data_ptr()):
            raise RuntimeError("FlatGradExchange(colour_factor=...): the SH leaves received a gradient besides the "
                               "factored rasterizer backward in this step; use the plain exchange for such losses")


def rebuild_sh(cf, world):
    """hlgs_sh_grad_from_colour over the gathered rows (rank order), averaged: fills cf.sh_buf / cf.dc_buf."""
    from hlgs_core import _lib as L
    lib = L.load()
    L.require_gpu(cf.gathered, cf.means, cf.sh_buf)
    P = cf.means.shape[0]
    M = cf.sh.shape[1] if cf.sh.dim() > 1 else 0
    base = cf.gathered.data_ptr()
    L.check(lib.hlgs_sh_grad_from_colour(P, world, cf.D, M, cf.variant, L.ptr(cf.means.detach().contiguous()), base,
                                         base + 16, cf.row, 1.0 / world, L.ptr(cf.sh_buf),
                                         L.ptr(cf.dc_buf) if cf.dc_buf is not None else None, L.stream()))


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

    def __init__(self, params, bucket_bytes=64 << 20, average=True, group=None, direct=True, overlap=False,
                 colour_factor=None):
        # colour_factor = dict(means=<means3D leaf>, sh=<SH leaf (P, M, 3)>, dc=<the alt variant's dc leaf> or None):
        # the SH leaves leave the flat buffer and are exchanged as colour gradients (module docstring); needs averaging
        self.cf = None
        params = list(params)
        if colour_factor is not None:
            sh, dc = colour_factor["sh"], colour_factor.get("dc")
            assert average, "the colour-factored SH exchange averages"
            world = dist.get_world_size(group) if dist.is_initialized() else 1
            self.cf = _ColourFactor(colour_factor["means"], sh, dc, world, sh.device)
            params = [p for p in params if p is not sh and p is not dc]
            _FACTOR[sh.data_ptr()] = (weakref.ref(sh), weakref.ref(self))
        self.params = params
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

    def link_bytes(self, world):
        """(all-reduced bytes, bytes all-gathered per rank, bytes each GPU moves over its links per exchange for a ring
        of `world` ranks: 2 (N-1)/N of the all-reduced buffer plus (N-1) gathered rows)."""
        ar = 4 * self.flat.numel()
        ag = 4 * self.cf.row if self.cf is not None else 0
        return ar, ag, int(2 * (world - 1) / world * ar + (world - 1) * ag)

    def close(self):
        """Stop offering the flat buffer to the rasterizer backward.  Rebuild the exchange (and close the old one)
        whenever the parameter tensors are replaced: entries are keyed by storage address."""
        if self.cf is not None:
            e = _FACTOR.get(self.cf.sh.data_ptr())
            if e is not None and e[1]() is self:
                del _FACTOR[self.cf.sh.data_ptr()]
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
        if self.cf is not None:
            self.cf.written = False

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
            if self.cf is not None and self.cf.written:
                _check_factored(self.cf)
                self.join()  # the SH backward may still be writing this rank's row on the late stream
                self.cf.gathered[0].copy_(self.cf.mine)
                rebuild_sh(self.cf, 1)
            elif self.cf is not None:
                self._warn_unfactored()
            self.release()
            return
        world = dist.get_world_size(self.group)
        cf = self.cf
        cf_work = []

        def start_gather():
            """The rows of all ranks, gathered while the flat buffer is reduced; called once the late stream (which
            writes this rank's row with the SH backward) is joined."""
            if cf is None or not cf.written or cf_work:
                return
            if cf.gathered.shape[0] != world:  # sized at construction, possibly before init_process_group
                cf.gathered = torch.empty((world, cf.row), dtype=torch.float32, device=cf.mine.device)
            if cf.mine.is_cuda and dist.get_backend(self.group) != "nccl":
                # gloo has no all_gather of device tensors (one-GPU rehearsals): each rank's row in its own slot
                # of a zeroed buffer, summed -- the same rows, twice the bytes
                me = dist.get_rank(self.group)
                cf.gathered.zero_()
                cf.gathered[me].copy_(cf.mine)
                cf_work.append(dist.all_reduce(cf.gathered, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
            elif dist.get_backend(self.group) == "nccl":  # RCCL writes the rows straight into the [world, row] buffer
                cf_work.append(dist.all_gather_into_tensor(cf.gathered, cf.mine, group=self.group, async_op=True))
            else:
                cf_work.append(dist.all_gather(list(cf.gathered.unbind(0)), cf.mine, group=self.group, async_op=True))

        if cf is not None:
            if cf.written:
                _check_factored(cf)
            else:  # the backward did not factor (no rasterizer call saw the exchange): plain averaged all-reduce
                self._warn_unfactored()
                self.join()
                for t in (cf.sh, cf.dc):
                    if t is not None and t.grad is not None:
                        dist.all_reduce(t.grad, op=dist.ReduceOp.SUM, group=self.group)
                        t.grad.mul_(1.0 / world)
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
            start_gather()
            spans = [(0, self.flat.numel())] if in_place else self.buckets
        self.last_collectives = sum(1 for sp in spans if sp is not None) + (1 if cf is not None and cf.written else 0)
        for sp in spans:
            if sp is None:
                self.join()
                start_gather()
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
        self.join()
        start_gather()  # (split spans with no late run: nothing joined above)
        if cf_work:
            cf_work[0].wait()
            rebuild_sh(cf, world)
        self.unpack()

    def _warn_unfactored(self):
        """Warns (once) when the SH leaves hold a gradient that did not come through the factored backward.
        A colour-factored exchange whose round produced no colour row: the SH leaves' gradient came from elsewhere
        (e.g. a fresh torch.cat of dc and rest each step, which the exchange cannot recognise), so it is exchanged by a
        plain all-reduce -- correct, but without the factored exchange's bandwidth saving."""
        if any(t is not None and t.grad is not None for t in (self.cf.sh, self.cf.dc)) and \
                not getattr(self, "_warned_unfactored", False):
            import warnings
            warnings.warn("FlatGradExchange(colour_factor=...): no rasterizer backward wrote a colour row this round; "
                          "the SH gradient is exchanged by a plain all-reduce (pass the SH parameter leaf itself to the "
                          "rasterizer to factor it)", RuntimeWarning, stacklevel=3)
            self._warned_unfactored = True
