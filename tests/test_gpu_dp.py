"""Batch data parallelism of the REAL training steps (floodgan.parallel): two
ranks, each a separate process holding its own replica on the one GPU of the test box, gloo on HIP
tensors carrying the steps' bucketed asynchronous SUM all-reduces (the same FlatGrads / ready()
path RCCL takes on an 8-GPU node).  Each rank trains on half of a global batch; every iteration must
equal one process training on the whole batch from the same state: the per-rank losses average to the
single-process losses (equal shards, mean losses), the all-reduced gradients equal its gradients, and the
updates meet the U criterion (decided elements move the same way and agree; tests/test_gpu_northstar.py).
The production (f16x3) path is also pinned iteration by iteration against the fp64 oracle.

What this pins: the 1/world pre-scaling folded into the loss gradients (model.py PairedStep,
cycle.py CycleStep), the bucket layout and the ready() order of the executors' backward, and the
asynchronous all-reduces racing the remaining backward kernels.

Both sides run the exact-fp32 conv math (FLOODGAN_CONV_MATH=fp32): every output element's
accumulation order is then independent of the batch it sits in, so each rank's per-sample forward is
bit-identical to the single process's and the only difference left is the order in which the
all-reduce adds the two shards' gradient partial sums.  (Under f16x3 the per-tensor operand scale of a
half batch can differ from the whole batch's by a power of two: rounding-level differences that flip
ReLU kinks -- the same chaos the single-device tests handle by teacher-forcing decisions.)"""
import os
import socket
import subprocess
import sys

import pytest
import torch

from oracle import paired_attention as O
from test_gpu_northstar import KINK, _update_agreement, u_compare, u_summary
from test_gpu_parity import DEV, NTOL, nrel

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import dp_worker as W  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(tmp_path, kind, n, res, iters, **env_extra):
    """two dp_worker ranks (gloo on HIP tensors); their saved records"""
    out = str(tmp_path / "dp")
    port = _free_port()
    env = dict(os.environ, WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="2",
               FG_RECORD_DECISIONS="1")
    env.pop("FLOODGAN_CONV_MATH", None)
    env.update(env_extra)
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dp_worker.py"), out, kind, str(n), str(res),
                               str(iters)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r))) for r in range(2)]
    try:
        rcs = [p.wait(timeout=240) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0], rcs
    ranks = [torch.load(f"{out}.rank{r}", weights_only=True) for r in range(2)]
    for k, v in ranks[0]["state"].items():
        assert torch.equal(v, ranks[1]["state"][k]), k              # the replicas stay identical
    return ranks


def _merge(a, b):
    """the two ranks' decisions of one iteration as one global batch (rank 0 holds the first half)"""
    if isinstance(a, dict):
        return {k: _merge(a[k], b[k]) for k in a}
    if isinstance(a, list):
        return [_merge(x, y) for x, y in zip(a, b)]
    return torch.cat((a, b), 0)


def _count_diff(a, b):
    if isinstance(a, dict):
        return sum(_count_diff(a[k], b[k]) for k in a)
    if isinstance(a, list):
        return sum(_count_diff(x, y) for x, y in zip(a, b))
    return int((a.cpu() != b.cpu()).sum())


def _flip_positions(a, b):
    """{(network, D pass or None): [forward positions of the layers whose decisions differ]} of a paired step's
    decision records (PairedStep.decisions): G's ReLU layers, D's LeakyReLU layers per pass (0 fake / 1 real of the
    D step, 2 the G step), the L1 signs"""
    pos_g = {"conv1": 0, "conv2": 1, "conv3": 2, **{f"block{i}": 3 + i for i in range(9)}}
    out = {}
    for net, passes in a.items():
        for pi, (da, db) in enumerate(zip(passes, b[net])):
            for k in da:
                if _count_diff(da[k], db[k]):
                    pos = (pos_g.get(k, 12 if k.startswith("deconv1") else 13) if net == "G" else
                           {"model.0": 0, "model.2": 1, "model.5": 2, "model.8": 3}.get(k, 0))
                    out.setdefault((net, pi if net == "D" else None), []).append(pos)
    return out


def _param_position(net, k):
    """forward position of a parameter's layer in the numbering of _flip_positions (a conv that consumes a decided
    activation sits half a step after it: its weight gradient reads the activation)"""
    layer = k.rsplit(".", 1)[0]
    if net == "discriminator":
        return {"model.0": 0, "model.2": 1, "model.5": 2, "model.8": 3, "model.11": 4}[layer]
    if layer.startswith("resnet_blocks."):
        i, conv = layer.split(".")[1:3]
        return 3 + int(i) - 0.5 + (0.5 if conv == "conv1" else 1.0)
    return {"conv1": 0, "conv2": 1, "conv3": 2}.get(layer, 12 + (layer[7] == "2") + 2 * (layer[7] == "3") - 0.5)


def _flip_reach(flips, net, k):
    """True when a differing decision lies downstream of parameter k: its gradient then legitimately carries the
    flip (one unit of backward flow passed or blocked, ~1/sqrt(elements) of the gradient: the 1e-3 envelope);
    every other tensor keeps the 1e-5 bound.  A flip in D's G-step pass or in the L1 signs reaches all of G; a flip in
    a D-step pass reaches D's layers up to the one that reads the activation."""
    q = _param_position(net, k)
    if net == "generator":
        if flips.get(("D", 2)) or flips.get(("L1", None)):
            return True
        return any(q <= d + 0.5 for d in flips.get(("G", None), []))
    return any(q <= d + 1 for pi in (0, 1) for d in flips.get(("D", pi), []))


def _post_state(ranks, it):
    """the two-rank state after iteration `it`"""
    its = ranks[0]["iters"]
    return its[it + 1]["pre"]["state"] if it + 1 < len(its) else ranks[0]["state"]


@pytest.mark.parametrize("kind,n,res", [("paired", 4, 64), ("attentiongan", 2, 32)])
def test_two_rank_step_equals_single_rank(kind, n, res, tmp_path, report):
    """Two ranks (exact-fp32 conv math) train two iterations on halves of a global batch.  For EACH iteration a
    single process is loaded with the state the two ranks started it from (every network, both Adam states) and
    runs the same iteration on the whole batch; in the paired step it also continues its G half on the two-rank
    discriminator after Adam(D) (PairedStep.d_after), as the oracle comparisons do.  Asserted per iteration:
      * the all-reduced gradients equal the single-process gradients: 1e-5 norm-relative (IN-cancelled biases
        excluded), widened to 1e-3 only for the tensors a differing activation / L1-sign decision
        lies downstream of (counted and positioned; every tensor above 1e-5 is reported);
      * the losses: the two ranks' mean equals the single process's to 1e-5;
      * the update (U criterion, tests/test_gpu_northstar.py): every element whose first moment is decided --
        |m| above 10x the gradient's disagreement -- moves the same way (fraction 1.0) and the decided updates
        agree to 1e-3; the undecided fraction is reported.
    A DP defect -- a missing or doubled bucket, a stale replica, the 1/world scale applied twice -- moves the
    gradients by O(1) and fails the first bound; rounding-level gradient noise that Adam's normalisation
    amplifies only touches undecided elements."""
    from floodgan import _lib as L
    iters = 2
    ranks = _launch(tmp_path, kind, n, res, iters, FLOODGAN_CONV_MATH="fp32")
    x, y = W.global_batch(kind, n, res)
    skip_g, skip_d = O.cancelled_biases()
    prev = L.get_conv_math()
    L.set_conv_math("fp32")
    try:
        for it in range(iters):
            rec = ranks[0]["iters"][it]
            post = _post_state(ranks, it)
            m = W.make_model(kind)
            if kind != "paired":
                import random
                for pool in (m.cycle_step_fn.pre_pool, m.cycle_step_fn.post_pool):
                    pool.rng = random.Random(5)
            W.load_snapshot(m, kind, rec["pre"])
            step = m.step_fn if kind == "paired" else m.cycle_step_fn
            step.record_decisions = True
            if kind == "paired":
                step.d_after = {k: post[f"discriminator/{k}"].to(DEV) for k, _ in m.discriminator.named_parameters()}
            single = W.run(m, kind, x, y, 1)[0].double()
            merged = _merge(rec["decisions"], ranks[1]["iters"][it]["decisions"])
            flips = _count_diff(merged, step.decisions)
            reach = _flip_positions(merged, step.decisions) if kind == "paired" else None
            mean = (ranks[0]["losses"][it].double() + ranks[1]["losses"][it].double()) / 2
            lrel = float(((mean - single).abs() / single.abs()).max())
            opt_state = {}
            for o in (m.optimizer_generator, m.optimizer_discriminator):
                opt_state.update(o.state)
            rows, bad, over = [], [], []
            for net, mod in W.nets(m, kind).items():
                skip = skip_g if "generator" in net else skip_d
                for k, p in mod.named_parameters():
                    if k in skip:
                        continue
                    key = f"{net}/{k}"
                    ge = nrel(rec["grads"][key], p.grad)
                    # the paired discriminator's own Adam(D) result (its parameters now hold d_after)
                    p_single = step.d_after_own[k] if kind == "paired" and net == "discriminator" else p
                    agree, uerr, frac, perr = _update_agreement(rec["pre"]["state"][key], post[key], p_single,
                                                                rec["grads"][key], p.grad, opt_state[p]["exp_avg"])
                    rows.append((net, k, ge, agree, uerr, frac, perr))
                    # 1e-5 unless a differing decision downstream of this tensor explains more (paired: by layer;
                    # the cycle step's records are not positioned, so any flip there widens its networks' bounds)
                    reached = flips > 0 and (reach is None or _flip_reach(reach, net, k))
                    if ge > 1e-5:
                        over.append((net, k, ge, reached))
                    if ge > (1e-3 if reached else 1e-5) or agree < 1.0 or uerr > NTOL:
                        bad.append(rows[-1])
            report("dp_two_rank_vs_single_continuation", kind=kind, n=n, res=res, it=it, decisions_differing=flips,
                   loss_rel=lrel, **u_summary(rows), bad=bad, over_1e5=over,
                   flip_layers={f"{a}{'' if b is None else b}": v for (a, b), v in (reach or {}).items()})
            assert flips <= 8, (it, flips)
            assert not bad, (it, bad)
            assert lrel < 1e-5, (it, mean, single)
            del m
    finally:
        L.set_conv_math(prev)


def test_two_rank_paired_f16x3_vs_fp64(tmp_path, report):
    """The production DP path: the default f16x3 conv math, two ranks each on half of a global batch of 4
    (64x64), bucketed asynchronous SUM all-reduces, two iterations.  For each iteration the fp64 oracle
    continues from the state the ranks started it from (both networks, both Adam states), with the two ranks'
    activation and L1-sign decisions teacher-forced and, for the G half, the two-rank discriminator after
    Adam(D) (models/model.py:611-651, updates at :633 and :646).  Asserted per iteration: the all-reduced G / D
    gradients vs fp64 to 1e-4 (P2), every differing decision at its kink, and the U criterion on the updates
    (decided elements: direction 1.0, update 1e-3)."""
    n, res, iters = 4, 64, 2
    ranks = _launch(tmp_path, "paired", n, res, iters)
    x, y = W.global_batch("paired", n, res)
    for it in range(iters):
        rec = ranks[0]["iters"][it]
        pre, post = rec["pre"], _post_state(ranks, it)
        dec = O.ActDecisions(_merge(rec["decisions"], ranks[1]["iters"][it]["decisions"]))
        split = lambda st, net: {k.split("/", 1)[1]: v for k, v in st.items() if k.startswith(net + "/")}  # noqa: E731
        g0, d0 = split(pre["state"], "generator"), split(pre["state"], "discriminator")
        lr = pre["optim"]["optimizer_generator"]["param_groups"][0]["lr"]
        st = O.PairedStepOracle(dtype=torch.float64, lr=lr)
        st.load_state(g0, d0, pre["optim"]["optimizer_generator"] if it else None,
                      pre["optim"]["optimizer_discriminator"] if it else None)
        orec = {}
        st.step(x, y, record=orec, d_after=split(post, "discriminator"), decisions=dec)
        rows, bad = u_compare(st, orec, {"G": g0, "D": d0},
                              {"G": split(post, "generator"), "D": split(post, "discriminator")},
                              {"G": split(rec["grads"], "generator"), "D": split(rec["grads"], "discriminator")})
        report("dp_two_rank_f16x3_vs_fp64", n=n, res=res, it=it, **u_summary(rows),
               decisions_differing=sum(c for _, _, c, _ in dec.log), worst_kink=dec.worst(), bad=bad)
        assert dec.worst() < KINK, (it, dec.worst())
        assert not bad, (it, bad)
