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


_force = False


def set_force_collectives(on):
    """Issue the gradient all-reduces even in a one-rank process group (they are then identities).  The
    only way to execute the RCCL path -- ProcessGroupNCCL's stream beside the backward kernels, the
    bucket hand-offs, the waits before Adam -- on a box with one GPU (`bench.py --rccl-world1`,
    tests/test_gpu_rccl.py).  Returns the previous setting."""
    global _force
    prev, _force = _force, bool(on)
    return prev


def collectives_on():
    """True when the step's gradient exchanges run: more than one rank, or a forced one-rank group."""
    ws, _ = world()
    return ws > 1 or (_force and dist.is_available() and dist.is_initialized())


class FlatGrads:
    """Allocates one contiguous gradient buffer for `params` and points every p.grad at its
    slice (views stay valid as long as nobody sets p.grad = None).

    `params` is a list of tensors, or a {name: tensor} dict together with `buckets`: lists of
    names in the order the backward finishes them.  The buffer is laid out bucket by bucket, so
    each bucket is one contiguous slice and can be all-reduced as soon as the backward has
    written it (`ready`), overlapping RCCL with the rest of the backward: ProcessGroupNCCL runs
    the collective on its own stream after the current one, so the kernels queued after it
    proceed in parallel; `finish` makes the current stream wait for all of them (before Adam)."""

    def __init__(self, params, buckets=None):
        if isinstance(params, dict):
            named = params
            order = buckets if buckets is not None else [list(named)]
            listed = [n for b in order for n in b]
            if sorted(listed) != sorted(named):
                raise ValueError("buckets must list every parameter exactly once")
            self.params = [named[n] for n in listed]
            sizes = [sum(named[n].numel() for n in b) for b in order]
            self.bucket_names = [tuple(b) for b in order]
        else:
            self.params = [p for p in params]
            sizes = [sum(p.numel() for p in self.params)]
            self.bucket_names = [None]
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.views = []
        off = 0
        for p in self.params:
            v = self.flat[off:off + p.numel()].view_as(p)
            self.views.append(v)
            off += p.numel()
        self.buckets = []
        off = 0
        for sz in sizes:
            self.buckets.append(self.flat[off:off + sz])
            off += sz
        self._pending, self._handles, self._group = [], [], None
        self.attach()

    def attach(self):
        for p, v in zip(self.params, self.views):
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                p.grad = v
        return self

    def allreduce_sum(self, group=None):
        """In-place SUM across ranks (callers pre-scale by 1/world)."""
        if collectives_on():
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)

    # ---- bucketed, overlapped SUM all-reduce
    def begin(self, group=None):
        self._group = group
        self._pending = list(range(len(self.buckets)))
        self._handles = []

    def ready(self, bucket):
        """The backward has finished every gradient of `bucket` (index, or the name of one of its
        parameters' bucket key): start its all-reduce asynchronously."""
        i = bucket if isinstance(bucket, int) else self.bucket_index(bucket)
        if i not in self._pending:
            return
        self._pending.remove(i)
        if collectives_on():
            self._handles.append(dist.all_reduce(self.buckets[i], op=dist.ReduceOp.SUM, group=self._group,
                                                 async_op=True))

    def bucket_index(self, key):
        for i, names in enumerate(self.bucket_names):
            if names is not None and any(n == key or n.startswith(key + ".") for n in names):
                return i
        raise KeyError(key)

    def finish(self):
        """Start whatever was never marked ready, then wait for every bucket's all-reduce."""
        for i in list(self._pending):
            self.ready(i)
        for h in self._handles:
            h.wait()
        self._handles = []


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
