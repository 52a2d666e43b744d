"""Pix2Pix on the HIP path vs the CPU oracle (oracle/pix2pix.py, pinned to the
reference's own train_paired by tests/test_oracle_pix2pix_golden.py), at 256x256 -- the U-Net-256's
smallest input.

  P1  the generator output (training mode: batch statistics, the drawn Dropout masks), the
      discriminator outputs of the D step's fused fake / real pass (two BatchNorm groups) and every
      BatchNorm running statistic they update, vs the fp32 oracle.
  U   two training iterations of the fused step, teacher-forced: before each, the fp64 oracle takes the
      HIP state (parameters, BatchNorm buffers, both Adam states), the HIP Dropout masks, the HIP
      activation decisions and, for the G half, the HIP discriminator after Adam(D).  Every G / D
      gradient within 1e-4, every differing decision at its kink, every decided element's update in the
      same direction and the decided updates within 1e-3 (tests/test_gpu_northstar.py's criterion).
  P3  the Model's own train_paired over two epochs vs the reference's golden losses and outputs, within
      the reference algorithm's own envelope under 1e-6 input noise.
"""
import copy

import numpy as np
import pytest
import torch

from oracle import paired_attention as O
from oracle import pix2pix as OP
from test_gpu_northstar import KINK, _update_agreement
from test_gpu_parity import DEV, NTOL, nrel
from test_oracle_pix2pix_golden import CASES, load_gold, probe_sample, synth_inputs

pytestmark = pytest.mark.gpu

R = 256


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.set_num_threads(min(16, max(1, len(__import__("os").sched_getaffinity(0)))))


def _model(case="all_bs2", **kw):
    """case: a tests/test_oracle_pix2pix_golden.CASES key -- topography="all" (9-ch input) or, for BASELINE.json
    configs[0], topography=None (3-ch RGB input)"""
    from floodgan.model import Model
    return Model(model="Pix2Pix", num_epochs=2, topography="all" if CASES[case][2] == 9 else None, **kw)


def _state(mod):
    return ({k: v.detach().cpu() for k, v in mod.named_parameters()},
            {k: v.detach().cpu().clone() for k, v in mod.named_buffers()})


@pytest.mark.parametrize("case", sorted(CASES))
def test_p1_forward_and_running_stats(case, report):
    from floodgan import executor as X
    from floodgan import pix2pix as P2P
    _, n, c = CASES[case]
    m = _model(case)
    (x, y), _ = synth_inputs(N=n, C=c)
    (gp, gb), (dp, db) = _state(m.generator), _state(m.discriminator)
    torch.manual_seed(5)
    masks = P2P.draw_dropout_masks(n, R, R)
    xd, yd = x.to(DEV), y.to(DEV)
    G, D = m.generator, m.discriminator
    fake, _ = P2P.gen_forward(G.param_dict(), G.buffer_dict(), xd, masks=masks, save=False)
    pred, _ = P2P.disc_forward(D.param_dict(), D.buffer_dict(), X.disc_pack([(xd, fake), (xd, yd)], c + 3), groups=2,
                               save=False)
    torch.cuda.synchronize()
    with torch.no_grad():
        gb_r, db_r = copy.deepcopy(gb), copy.deepcopy(db)
        fake_r = OP.generator_forward(gp, gb_r, x, masks=dict(masks))
        pf = OP.discriminator_forward(dp, db_r, torch.cat((x, fake_r), 1))
        pr = OP.discriminator_forward(dp, db_r, torch.cat((x, y), 1))
    e = dict(g_out=nrel(fake, fake_r), d_fake=nrel(pred[:n], pf), d_real=nrel(pred[n:], pr))
    run = [(k, nrel(v, gb_r[k])) for k, v in G.named_buffers() if v.is_floating_point()]
    run += [(k, nrel(v, db_r[k])) for k, v in D.named_buffers() if v.is_floating_point()]
    report("pix2pix_p1_256", case=case, **e, worst_running_stat=max(run, key=lambda t: t[1]))
    assert max(e.values()) < 1e-4, e
    assert max(r for _, r in run) < 1e-5, max(run, key=lambda t: t[1])
    # one BatchNorm call per generator layer, two (fake, real) per discriminator layer
    assert all(int(v) == 1 for k, v in G.named_buffers() if k.endswith("num_batches_tracked"))
    assert all(int(v) == 2 for k, v in D.named_buffers() if k.endswith("num_batches_tracked"))


@pytest.mark.parametrize("case", sorted(CASES))
def test_update_teacher_forced(case, report):
    """Two fused iterations at 256x256 on the golden inputs (batch 2 with topography="all"; batch 1 with
    the 3-ch RGB input of BASELINE.json configs[0]), each checked against the fp64 oracle continuing from
    the HIP state with the HIP masks and decisions."""
    from floodgan import pix2pix as P2P
    _, n, c = CASES[case]
    m = _model(case)
    G, D = m.generator, m.discriminator
    step = m.step_fn
    step.record_decisions = True
    for it, (x, y) in enumerate(synth_inputs(N=n, C=c)):
        lr = 2e-4 if it == 0 else 1e-4
        for opt in (m.optimizer_generator, m.optimizer_discriminator):
            for grp in opt.param_groups:
                grp["lr"] = lr
        (g0, gb0), (d0, db0) = _state(G), _state(D)
        st = OP.Pix2PixStepOracle(dtype=torch.float64, lr=lr, c_in=c)
        st.load_state(g0, gb0, d0, db0, m.optimizer_generator.state_dict() if it else None,
                      m.optimizer_discriminator.state_dict() if it else None)
        torch.manual_seed(it + 1)
        step(x.to(DEV), y.to(DEV))
        torch.cuda.synchronize()
        rec = {}
        dec = O.ActDecisions(step.decisions)
        masks = {k: v.cpu() for k, v in P2P.dropout_masks(step.last_masks, n, R, R).items()}
        st.step(x, y, record=rec, masks=masks, decisions=dec,
                d_after={k: v.detach().cpu() for k, v in D.named_parameters()})
        rows, bad = [], []
        for net, mod, P0, grads, opt_ref in (("G", G, g0, rec["g_grads"], st.opt_g), ("D", D, d0, rec["d_grads"],
                                                                                     st.opt_d)):
            params_ref = st.G if net == "G" else rec["d_after_own"]
            order = list(st.G if net == "G" else st.D)
            for k, p in mod.named_parameters():
                ge = nrel(p.grad, grads[k])
                m_ref = opt_ref.state[opt_ref.param_groups[0]["params"][order.index(k)]]["exp_avg"]
                agree, uerr, frac, perr = _update_agreement(P0[k], p, params_ref[k], p.grad, grads[k], m_ref)
                rows.append((net, k, ge, agree, uerr, frac, perr))
                if ge > 1e-4 or agree < 1.0 or uerr > NTOL:
                    bad.append(rows[-1])
        run = [(k, nrel(v, st.GB[k])) for k, v in G.named_buffers() if v.is_floating_point()]
        report("pix2pix_update_teacher_forced", case=case, R=R, it=it, worst_grad=max(rows, key=lambda r: r[2])[1:3],
               min_agree=min(r[3] for r in rows), worst_update=max(rows, key=lambda r: r[4])[1:5:3],
               min_decided=min(r[5] for r in rows), decisions_differing=sum(r[2] for r in dec.log),
               worst_kink=dec.worst(), worst_running_stat_G=max(run, key=lambda t: t[1]), bad=bad)
        assert dec.worst() < KINK, dec.worst()
        assert not bad, bad
        assert max(r for _, r in run) < 1e-5


def _reference_envelope(gold, case, sigma=1e-6, trials=2):
    """how far the reference algorithm (fp32 oracle) itself lands from the golden run when its inputs
    carry `sigma` relative noise: per iteration (G probe, D probe, losses)"""
    from test_oracle_pix2pix_golden import probe
    _, n, c = CASES[case]
    batches = synth_inputs(N=n, C=c)
    x0, y0 = batches[0]
    env = [[0.0, 0.0, 0.0], [0.0, 0.0, 0.0]]
    for trial in range(1, trials + 1):
        st = OP.Pix2PixStepOracle(c_in=c)
        for it, (x, y) in enumerate(batches):
            st.set_lr(float(gold[f"it{it}_lr"][0]))
            noise = torch.randn(x.shape, generator=torch.Generator().manual_seed(trial * 10 + it))
            torch.manual_seed(it + 1)
            ls = np.array(st.step(x * (1 + sigma * noise), y))
            g, d = probe(((st.G, st.GB), (st.D, st.DB)), x0, y0)
            e = (nrel(torch.from_numpy(g[2:]), torch.from_numpy(gold[f"it{it}_g_out"][2:])),
                 nrel(torch.from_numpy(d), torch.from_numpy(gold[f"it{it}_d_out"])),
                 float((np.abs(ls - gold[f"it{it}_losses"]) / np.abs(gold[f"it{it}_losses"])).max()))
            env[it] = [max(a, b) for a, b in zip(env[it], e)]
    return env


@pytest.mark.parametrize("case", sorted(CASES))
def test_train_paired_vs_reference_golden(case, report):
    """Model("Pix2Pix").train_paired over the golden's two epochs (one batch each; torch.manual_seed(epoch)
    fixes the Dropout masks exactly as in the reference) vs the reference's recorded losses and its
    training-mode G / D probes after each epoch."""
    gold = load_gold(case)
    env = _reference_envelope(gold, case)
    _, n, c = CASES[case]
    batches = synth_inputs(N=n, C=c)
    x0, y0 = (t.to(DEV) for t in batches[0])
    recorded = []

    class _Loader:
        def __init__(self):
            self.epoch = 0

        def __iter__(self):
            x, y = batches[self.epoch]
            self.epoch += 1
            return iter([(x, y, ["synthetic"] * n)])

    m = _model(case, train_loader=_Loader())
    m.generator.dropout_rng = "host"          # the reference's CPU draws, mask for mask
    orig = m.save_results

    def _record(epoch, losses, t0):
        with torch.no_grad(), torch.random.fork_rng(devices=[]):
            torch.manual_seed(99)
            g = copy.deepcopy(m.generator)(x0)           # the copy keeps dropout_rng = "host"
            d = copy.deepcopy(m.discriminator)(torch.cat((x0, y0), 1))
        recorded.append(([losses[k][-1] for k in ("losses_discriminator_real", "losses_discriminator_synthetic",
                                                  "losses_generator_synthetic", "l1_losses_generator_synthetic")],
                         probe_sample(g.cpu()), d.cpu().numpy()))
        orig(epoch, losses, t0)

    m.save_results = _record
    m.train_paired()
    for it, (losses, g, d) in enumerate(recorded):
        ref = gold[f"it{it}_losses"].copy()
        ref[3] *= 100
        lrel = np.abs(np.array(losses) - ref) / np.abs(ref)
        e_g = nrel(torch.from_numpy(g[2:]), torch.from_numpy(gold[f"it{it}_g_out"][2:]))
        e_d = nrel(torch.from_numpy(d), torch.from_numpy(gold[f"it{it}_d_out"]))
        report("pix2pix_train_vs_reference_golden", case=case, it=it, loss_rel=lrel.tolist(), g_probe=e_g, d_probe=e_d,
               reference_envelope=env[it])
        if it == 0:       # P1: the D losses and the L1 term are evaluated before any update
            assert lrel[[0, 1, 3]].max() < 1e-4, lrel
        assert lrel.max() < max(NTOL, 2 * env[it][2]), (lrel, env[it])
        assert e_g < max(NTOL, 2 * env[it][0]), (e_g, env[it])
        assert e_d < max(NTOL, 2 * env[it][1]), (e_d, env[it])


def test_modules_autograd_and_eval_mode():
    """The drop-in modules through autograd (nn.MSELoss on D(cat(x, G(x)))) equal the executor step's
    gradients, and .eval() uses the running statistics with Dropout off (vs the oracle restated with
    F.batch_norm(training=False))."""
    import torch.nn.functional as F
    m = _model()
    G, D = m.generator, m.discriminator
    (x, y), _ = synth_inputs()
    xd = x[:1].to(DEV)
    G.eval()
    with torch.no_grad():
        out = G(xd)
    gp, gb = _state(G)
    P = {k: v.double() for k, v in gp.items()}
    B = {k: (v.double() if v.is_floating_point() else v) for k, v in gb.items()}
    ref = OP.generator_forward(P, B, x[:1].double(), training=False)
    assert nrel(out, ref) < 1e-4
    G.train()
    torch.manual_seed(3)
    fake = G(xd)
    pred = D(torch.cat((xd, fake), 1))
    F.mse_loss(pred, torch.ones_like(pred)).backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in G.parameters())
    assert all(p.grad is not None for p in D.parameters())


@pytest.mark.parametrize("seed,pre,shapes,p", [
    (47, 0, [(8, 512, 8, 8), (8, 512, 16, 16), (8, 512, 32, 32)], 0.5),   # Pix2Pix 512^2 batch 8: 69 chunks
    (5, 3, [(2, 512, 4, 4), (2, 512, 8, 8), (2, 512, 16, 16)], 0.5),     # 256^2 batch 2: one chunk
    (9, 623, [(1, 7, 3), (79872,), (79873,), (5,)], 0.3),                  # odd sizes across chunk boundaries
    (0, 624, [(10_500_000,)], 0.5),                                        # past the committed jump table
])
def test_device_torch_stream_bit_exact(seed, pre, shapes, p):
    """floodgan.torch_rng (csrc/mt19937.hip): the device-generated masks equal torch's CPU draws
    torch.empty(shape).bernoulli_(p) -- the reference's nn.Dropout (models/model_architectures.py:52) -- element for
    element, from the same generator state, and commit() leaves torch's generator exactly where those CPU draws
    leave it."""
    from floodgan import torch_rng
    torch.manual_seed(seed)
    if pre:
        torch.randint(0, 2 ** 31, (pre,), dtype=torch.int64)
    state = torch.get_rng_state()
    outs, commit = torch_rng.draw(shapes, p, DEV)
    commit()
    after = torch.get_rng_state()
    torch.set_rng_state(state)
    ref = [torch.empty(s).bernoulli_(p) for s in shapes]
    for o, r in zip(outs, ref):
        assert o.shape == r.shape
        assert torch.equal(o.cpu(), r), int((o.cpu() != r).sum())
    assert torch.equal(after, torch.get_rng_state())


def test_step_host_dropout_is_torch_stream(report):
    """Pix2PixStep with dropout_rng = "host": the masks of each iteration are torch's CPU draws (levels 7, 6, 5, as
    the reference's forward draws them) and, after the step, torch's generator stands where the CPU draws leave it
    -- two iterations in a row at 256x256, batch 2."""
    from floodgan import pix2pix as P2P
    m = _model()
    m.generator.dropout_rng = "host"
    (x, y), _ = synth_inputs(N=2, C=9)
    torch.manual_seed(123)
    for it in range(2):
        state = torch.get_rng_state()
        m.step_fn(x.to(DEV), y.to(DEV)).cpu()
        after = torch.get_rng_state()
        torch.set_rng_state(state)
        ref = P2P.draw_dropout_masks(2, R, R)
        for k, v in ref.items():
            assert torch.equal(m.step_fn.last_masks[k].cpu(), v), (it, k)
        assert torch.equal(after, torch.get_rng_state()), it
