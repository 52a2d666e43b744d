"""Batch data parallelism for the paired step: one process per GPU, torch.distributed over
RCCL ("nccl" backend on ROCm) / gloo on CPU.

The reference is single-device (models/model.py:24); SURVEY.md §8(e) adds batch DP: every
rank holds identical G/D replicas, sees B/world images, and the two exchange points of the
step are all-reduces of the D gradients (before Adam(D), models/model.py:632-633) and of the
G gradients (before Adam(G), :645-646).  Each rank scales its loss gradient by 1/world, so a
SUM all-reduce yields exactly the gradient of the global-batch mean loss with no extra pass.

Gradients live in one flat buffer per model (p.grad are views into it), so each exchange is a
single large collective -- on xGMI a ring all-reduce is per-link bound and one 47 MB (G) or
11 MB (D) message per step is the cheapest shape.
"""
import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


class FlatGrads:
    """Allocates one contiguous gradient buffer for `params` and points every p.grad at its
    slice (views stay valid as long as nobody sets p.grad = None)."""

    def __init__(self, params):
        self.params = [p for p in params]
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.views = []
        off = 0
        for p in self.params:
            v = self.flat[off:off + p.numel()].view_as(p)
            self.views.append(v)
            off += p.numel()
        self.attach()

    def attach(self):
        for p, v in zip(self.params, self.views):
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                p.grad = v
        return self

    def allreduce_sum(self, group=None):
        """In-place SUM across ranks (callers pre-scale by 1/world)."""
        ws, _ = world()
        if ws > 1:
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)


def broadcast_params(module, src=0, group=None):
    """Make every rank start from rank `src`'s weights (identical anyway under seed 47)."""
    ws, _ = world()
    if ws > 1:
        for p in module.parameters():
            dist.broadcast(p.data, src=src, group=group)


def shard_batch(x, rank, world_size):
    """Contiguous equal shard of a global batch (DistributedSampler-equivalent for tiles)."""
    n = x.shape[0]
    if n % world_size:
        raise ValueError(f"global batch {n} not divisible by world size {world_size}")
    per = n // world_size
    return x[rank * per:(rank + 1) * per]
