"""Batch data parallelism (floodgan/parallel.py) on the CPU with the gloo backend, world size 2:
per-rank gradients of the local-shard loss scaled by 1/world, summed by FlatGrads.allreduce_sum,
equal the single-process gradient of the global-batch mean loss."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _loss(G, D, x, y):
    from oracle import paired_attention as O
    fake, _ = O.generator_forward(G, x)
    pred = O.discriminator_forward(D, torch.cat((x, fake), 1))
    return F.mse_loss(pred, torch.ones_like(pred)) + 100 * F.mse_loss(fake, y)


def _worker(rank, world, port, out, bucketed=False):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "flood-prediction-gan_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    from floodgan.parallel import FlatGrads, broadcast_params, shard_batch, world as W
    from oracle import paired_attention as O
    assert W() == (world, rank)
    torch.manual_seed(123 + rank)                  # deliberately different local init ...
    Gp, Dp = O.init_params(seed=47 if rank == 0 else 48)
    mod = torch.nn.Module()
    for k, v in list(Gp.items()) + [("D." + k, v) for k, v in Dp.items()]:
        mod.register_parameter(k.replace(".", "_"), torch.nn.Parameter(v.clone()))
    broadcast_params(mod)                          # ... made identical by the broadcast
    params = list(mod.parameters())
    ng = len(Gp)
    G = dict(zip(Gp.keys(), params[:ng]))
    D = dict(zip(Dp.keys(), params[ng:]))
    if bucketed:
        # the fused step's layout: G buckets in backward-completion order, then D's, each
        # all-reduced asynchronously as soon as it is "ready" (here: in completion order after
        # the whole backward, the overlap itself is a timing matter)
        from floodgan import executor as X
        named = dict(list(zip(Gp.keys(), params[:len(Gp)])) + [("D." + k, p) for k, p in zip(Dp.keys(), params[len(Gp):])])
        buckets = X.gen_bucket_names() + [["D." + n for n in b] for b in X.disc_bucket_names()]
        fg = FlatGrads(named, buckets)
    else:
        fg = FlatGrads(params)
    fg.flat.zero_()
    g = torch.Generator().manual_seed(99)
    x = torch.rand(4, 9, 32, 32, generator=g) * 2 - 1
    y = torch.rand(4, 3, 32, 32, generator=g) * 2 - 1
    loss = _loss(G, D, shard_batch(x, rank, world), shard_batch(y, rank, world)) / world
    loss.backward()
    if bucketed:
        fg.begin()
        for i in range(len(fg.buckets)):
            fg.ready(i)
        fg.finish()
        flat = torch.cat([p.grad.flatten() for p in params])      # back in parameter order
    else:
        fg.allreduce_sum()
        flat = fg.flat.clone()
    if rank == 0:
        torch.save((flat, [p.detach().clone() for p in params]), out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("bucketed", [False, True])
def test_gloo_world2_allreduce_matches_full_batch(tmp_path, bucketed):
    ctx = mp.get_context("spawn")
    out = str(tmp_path / "rank0.pt")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, out, bucketed)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    flat, params = torch.load(out, weights_only=True)
    # single process, full batch, rank-0 weights
    from oracle import paired_attention as O
    Gp, Dp = O.init_params(seed=47)
    ps = [torch.nn.Parameter(v.clone()) for v in list(Gp.values()) + list(Dp.values())]
    for a, b in zip(ps, params):
        assert torch.equal(a.detach(), b)
    ng = len(Gp)
    G = dict(zip(Gp.keys(), ps[:ng]))
    D = dict(zip(Dp.keys(), ps[ng:]))
    g = torch.Generator().manual_seed(99)
    x = torch.rand(4, 9, 32, 32, generator=g) * 2 - 1
    y = torch.rand(4, 3, 32, 32, generator=g) * 2 - 1
    _loss(G, D, x, y).backward()
    ref = torch.cat([p.grad.flatten() for p in ps])
    rel = float((flat - ref).norm() / ref.norm())
    assert rel < 1e-5, rel


def test_shard_batch_rejects_uneven():
    from floodgan.parallel import shard_batch
    with pytest.raises(ValueError):
        shard_batch(torch.zeros(5, 1), 0, 2)
