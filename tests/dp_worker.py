"""One rank of the data-parallel parity test (tests/test_gpu_dp.py launches two of these; not a
pytest module).  Runs `iters` fused training iterations of the chosen step on this rank's shard of
a seeded global batch, with torch.distributed (gloo on HIP tensors: both ranks share the one GPU of
the test box) driving the step's bucketed gradient all-reduce, and saves the per-iteration losses
and the final parameters.

  python tests/dp_worker.py OUT KIND GLOBAL_BATCH RES ITERS     (env RANK, WORLD_SIZE, MASTER_PORT)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flood-prediction-gan_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def global_batch(kind, n, res):
    g = torch.Generator().manual_seed(2024)
    x = torch.rand((n, 9, res, res), generator=g) * 2 - 1
    y = torch.rand((n, 3, res, res), generator=g) * 2 - 1
    return x, y


def nets(m, kind):
    if kind == "paired":
        return {"generator": m.generator, "discriminator": m.discriminator}
    return {n: getattr(m, n) for n in ("pre_to_post_generator", "post_to_pre_generator", "pre_discriminator",
                                       "post_discriminator")}


def grads(m, kind):
    """the (all-reduced) gradients the last iteration's optimiser steps used"""
    return {f"{net}/{k}": p.grad.detach().cpu().clone() for net, mod in nets(m, kind).items()
            for k, p in mod.named_parameters()}


def make_model(kind):
    from floodgan.model import Model
    name = {"paired": "PairedAttention", "attentiongan": "AttentionGAN", "cyclegan": "CycleGAN"}[kind]
    return Model(model=name, num_epochs=2, topography="all")


def run(m, kind, x, y, iters):
    step = m.step_fn if kind == "paired" else m.cycle_step_fn
    return [step(x.cuda(), y.cuda()).cpu() for _ in range(iters)]


def optimizers(m):
    return {"optimizer_generator": m.optimizer_generator, "optimizer_discriminator": m.optimizer_discriminator}


def _cpu(o):
    if isinstance(o, torch.Tensor):
        return o.detach().cpu().clone()
    if isinstance(o, dict):
        return {k: _cpu(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return type(o)(_cpu(v) for v in o)
    return o


def snapshot(m, kind):
    """the full training state before an iteration: every network's parameters and both optimisers' state
    dicts (torch.optim.Adam format; empty before the first step)"""
    state = {f"{net}/{k}": v.detach().cpu().clone() for net, mod in nets(m, kind).items()
             for k, v in mod.state_dict().items()}
    return {"state": state, "optim": {k: _cpu(o.state_dict()) for k, o in optimizers(m).items()}}


def load_snapshot(m, kind, snap):
    """continue from another run's state (teacher forcing, tests only)"""
    with torch.no_grad():
        for net, mod in nets(m, kind).items():
            mod.load_state_dict({k: snap["state"][f"{net}/{k}"] for k in mod.state_dict()})
    for k, o in optimizers(m).items():
        if snap["optim"][k]["state"]:
            o.load_state_dict(snap["optim"][k])


def main():
    out, kind, n, res, iters = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if os.environ.get("FLOODGAN_CONV_MATH"):
        from floodgan import _lib
        _lib.load()             # applies FLOODGAN_CONV_MATH
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{os.environ['MASTER_PORT']}", rank=rank,
                            world_size=world)
    from floodgan.parallel import broadcast_params, shard_batch
    m = make_model(kind)
    for net in nets(m, kind).values():
        broadcast_params(net)
    x, y = global_batch(kind, n, res)
    xs, ys = shard_batch(x, rank, world), shard_batch(y, rank, world)
    if kind != "paired":
        import random
        for pool in (m.cycle_step_fn.pre_pool, m.cycle_step_fn.post_pool):
            pool.rng = random.Random(5)
    step = m.step_fn if kind == "paired" else m.cycle_step_fn
    record = os.environ.get("FG_RECORD_DECISIONS") == "1"
    if record:                     # the activation decisions of this rank's passes (teacher forcing, test only)
        step.record_decisions = True
    # per iteration: the state it started from (rank 0; the replicas are identical, checked at the end), the
    # all-reduced gradients its optimiser steps used, and this rank's activation / L1-sign decisions
    losses, its = [], []
    for _ in range(iters):
        pre = snapshot(m, kind) if rank == 0 else None
        losses += run(m, kind, xs, ys, 1)
        its.append({"pre": pre, "grads": grads(m, kind) if rank == 0 else None,
                    "decisions": _cpu(step.decisions) if record else None})
    torch.cuda.synchronize()
    state = {f"{net}/{k}": v.detach().cpu() for net, mod in nets(m, kind).items() for k, v in mod.state_dict().items()}
    out_d = {"losses": torch.stack(losses), "state": state, "iters": its}
    torch.save(out_d, f"{out}.rank{rank}")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
