"""View-data-parallel gradient exchange.

Each rank holds a full replica of the Gaussian parameters and renders its own training view; the only
collective is one all-reduce of the Gaussian gradients (RCCL over xGMI with backend "nccl", gloo on
CPU).  Gradients are packed into one flat fp32 buffer so RCCL moves a few large messages instead of
one per parameter tensor, then averaged (the reference trains one view per step; G views per step is
an effective batch of G).
"""
import torch
import torch.distributed as dist


class FlatGradExchange:
    """Pack -> all-reduce -> unpack for a fixed list of parameter tensors.

    bucket_bytes splits the flat buffer so the all-reduce of bucket k can overlap the packing of bucket
    k+1 (async_op); 256 MB buckets keep each RCCL ring well above its bandwidth knee on xGMI.
    """

    def __init__(self, params, bucket_bytes=256 << 20, average=True, group=None):
        self.params = list(params)
        self.numels = [p.numel() for p in self.params]
        total = sum(self.numels)
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.flat = torch.empty(total, dtype=torch.float32, device=dev)
        self.average = average
        self.group = group
        per = max(1, bucket_bytes // 4)
        self.buckets = [(s, min(s + per, total)) for s in range(0, total, per)] or [(0, 0)]

    def pack(self):
        off = 0
        for p, n in zip(self.params, self.numels):
            g = p.grad if p.grad is not None else torch.zeros_like(p)
            self.flat[off:off + n].copy_(g.reshape(-1))
            off += n

    def unpack(self):
        off = 0
        for p, n in zip(self.params, self.numels):
            if p.grad is None:
                p.grad = torch.empty_like(p)
            p.grad.copy_(self.flat[off:off + n].view_as(p))
            off += n

    def allreduce(self):
        """All-reduce every parameter's .grad across the process group (sum, then /world if average)."""
        if not dist.is_initialized() or dist.get_world_size() == 1:
            return
        self.pack()
        works = [dist.all_reduce(self.flat[a:b], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                 for a, b in self.buckets if b > a]
        for w in works:
            w.wait()
        if self.average:
            self.flat.mul_(1.0 / dist.get_world_size(self.group))
        self.unpack()
