#!/usr/bin/env python3
"""One-GPU smoke test of FlatGradExchange's RCCL path (backend "nccl", world size 1): ReduceOp.AVG is accepted by
RCCL, buckets pipeline, and .grad ends up as views of the reduced buffer with the packed values.  The exchange
skips a world of 1, so the size check is patched to run the collective path anyway."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hierarchical-lod-gaussians_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from hlgs_core import dp  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
params = [torch.randn(1000, 3, device="cuda", requires_grad=True), torch.randn(1000, 16, 3, device="cuda",
                                                                            requires_grad=True)]
grads = [torch.randn_like(p) for p in params]
for p, g in zip(params, grads):
    p.grad = g.clone()
ex = dp.FlatGradExchange(params, bucket_bytes=20000)
real = dist.get_world_size
dist.get_world_size = lambda group=None: 2 if group is None else real(group)
try:
    ex.allreduce()
finally:
    dist.get_world_size = real
torch.cuda.synchronize()
for p, g in zip(params, grads):
    assert torch.equal(p.grad, g), "reduced gradient differs"
    assert p.grad.data_ptr() >= ex.flat.data_ptr(), "grad is not a view of the flat buffer"
print("ok: AVG accepted" if dp._AVG_OK[0] else "ok: AVG rejected, SUM fallback", len(ex.buckets), "buckets")
dist.destroy_process_group()
