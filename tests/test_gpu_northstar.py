"""Parity at the north-star configuration (BASELINE.json configs[1]: PairedAttention, 512x512,
topography=all) and the pinned-update criterion, against the CPU oracle (oracle/paired_attention.py,
pinned to the reference's own train_paired by tests/test_oracle_golden.py).

  P1  everything computed before the first update (G output, attention mask, D outputs, the D
      losses and the L1 term) vs the fp32 oracle: norm-relative <= 1e-5.
  P2  every G and D gradient under a smooth loss vs the fp64 oracle: <= 1e-4, with the oracle's
      ReLU / LeakyReLU decisions teacher-forced to the HIP path's (oracle.ActDecisions); every
      decision that differs must sit within rounding of the kink (|pre-activation| <= 1e-4 of the
      layer's rms).  Without this, one flipped element moves a whole network's gradients by
      ~1/sqrt(pixels x channels): at 512x512 the ~30 rounding-level flips put ANY two fp32
      evaluations (the reference's CPU run included) ~2e-3 apart.
  U   the optimiser update itself, teacher-forced: the oracle continues from the HIP state
      (parameters + Adam moments) and, for the G half, from the HIP discriminator after Adam(D)
      (models/model.py:633, :646).  Every element whose first moment is decided well above the
      gradient's rounding-level disagreement must move in the same direction (fraction 1.0) and the
      update of the decided elements agrees to 1e-3 norm-relative; undecided elements (|m| within
      10x the gradient noise: IN-cancelled biases, flipped ReLU kinks) are reported, not asserted.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import attention_cycle as OC
from oracle import paired_attention as O
from test_gpu_parity import DEV, KTOL, NTOL, buf_from, nchw, nrel

pytestmark = pytest.mark.gpu

R = 512


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from floodgan import _lib as L
    L.check(L.load().fg_device_ok(), "device_ok")
    torch.set_num_threads(min(16, max(1, len(__import__("os").sched_getaffinity(0)))))


def _model(**kw):
    from floodgan.model import Model
    return Model(model="PairedAttention", num_epochs=2, topography=kw.pop("topography", "all"), **kw)


def _inputs(n, c=9, res=R, seed=1234):
    g = torch.Generator().manual_seed(seed)
    return torch.rand((n, c, res, res), generator=g) * 2 - 1, torch.rand((n, 3, res, res), generator=g) * 2 - 1


# ---------------------------------------------------------------------------------------------- P1

def test_p1_forward_and_losses_512(report):
    """512x512, batch 2: G output, attention mask, D(real), D(synthetic) at the seed-47 weights and the
    three pre-update losses of the fused training step (models/model.py:615-631, :643) vs the fp32 oracle."""
    x, y = _inputs(2)
    Gp, Dp = O.init_params()
    with torch.no_grad():
        fake_r, mask_r = O.generator_forward(Gp, x)
        dr_r = O.discriminator_forward(Dp, torch.cat((x, y), 1))
        df_r = O.discriminator_forward(Dp, torch.cat((x, fake_r), 1))
    ref = np.array([float(F.mse_loss(dr_r, torch.ones_like(dr_r))), float(F.mse_loss(df_r, torch.zeros_like(df_r))),
                    100 * float(F.l1_loss(fake_r, y))])
    m = _model()
    xd, yd = x.to(DEV), y.to(DEV)
    with torch.no_grad():
        out = m.generator(xd)
        mask = m.generator.last_attention_mask
        dr = m.discriminator(torch.cat((xd, yd), 1))
        df = m.discriminator(torch.cat((xd, out), 1))
    e = dict(g_out=nrel(out, fake_r), mask=nrel(mask, mask_r), d_real=nrel(dr, dr_r), d_synthetic=nrel(df, df_r))
    losses = m.step_fn(xd, yd).cpu().numpy().astype(np.float64)
    lrel = np.abs(losses[[0, 1, 3]] - ref) / np.abs(ref)
    report("p1_512_vs_oracle_fp32", R=R, batch=2, loss_rel=lrel.tolist(), **e)
    assert max(e.values()) < KTOL, e
    assert lrel.max() < KTOL, lrel


# ---------------------------------------------------------------------------------------------- P2

def _worst(pairs):
    return max(pairs, key=lambda t: t[1])


KINK = 1e-4    # largest |pre-activation| / rms at which the HIP and fp64 decisions may differ


def hip_smooth_grads(m, x, y):
    """Executor-level forward + backward of MSE(D(cat(x, G(x))), 1) + 100*MSE(G(x), y) (the G step's
    loss with the L1 term made smooth) through libfloodgan: (G grads, D grads, activation decisions)."""
    from floodgan import executor as X
    gp, dp = m.generator.param_dict(), m.discriminator.param_dict()
    C = x.shape[1]
    fake, _, S = X.gen_forward(gp, x, save=True)
    pred, dS = X.disc_forward(dp, X.disc_pack([(x, fake)], C + 3), save=True)
    g_pred = (2.0 / pred.numel()) * (pred - 1)
    g_fake = ((200.0 / fake.numel()) * (fake - y)).contiguous()
    gD = X.disc_backward(dp, dS, g_pred.contiguous(), param_grads=True, input_grad=g_fake, input_grad_channels=(C, 3),
                         input_grad_accumulate=True)
    gG = X.gen_backward(gp, S, g_fake)
    dec = {"G": [X.gen_act_decisions(S)], "D": [X.disc_act_decisions(dS)]}
    torch.cuda.synchronize()
    return {k: v.clone() for k, v in gG.items()}, {k: v.clone() for k, v in gD.items()}, dec


def oracle_smooth_grads(Gp, Dp, x, y, dec):
    """the same loss on the fp64 oracle with the HIP decisions teacher-forced"""
    Gd = {k: v.double().requires_grad_(True) for k, v in Gp.items()}
    Dd = {k: v.double().requires_grad_(True) for k, v in Dp.items()}
    fake_r, _ = O.generator_forward(Gd, x.double(), O._forced(dec, "G"))
    pr = O.discriminator_forward(Dd, torch.cat((x.double(), fake_r), 1), O._forced(dec, "D"))
    (F.mse_loss(pr, torch.ones_like(pr)) + 100 * F.mse_loss(fake_r, y.double())).backward()
    return {k: v.grad for k, v in Gd.items()}, {k: v.grad for k, v in Dd.items()}


def compare_smooth_grads(m, x, y, c_in=9):
    gG, gD, masks = hip_smooth_grads(m, x.to(DEV), y.to(DEV))
    dec = O.ActDecisions(masks)
    Gp, Dp = O.init_params(c_in=c_in)
    rG, rD = oracle_smooth_grads(Gp, Dp, x, y, dec)
    skip_g, skip_d = O.cancelled_biases()
    eg = _worst([(k, nrel(v, rG[k])) for k, v in gG.items() if k not in skip_g])
    ed = _worst([(k, nrel(v, rD[k])) for k, v in gD.items() if k not in skip_d])
    flips = sum(n for _, _, n, _ in dec.log)
    return eg, ed, flips, dec.worst()


def test_p2_gradients_512(report):
    """512x512, batch 1: every G and D gradient of the smooth loss vs the fp64 oracle with the HIP
    activation decisions teacher-forced (IN-cancelled biases excluded: their gradients are pure
    rounding noise); every differing decision within rounding of its kink."""
    x, y = _inputs(1, seed=99)
    eg, ed, flips, kink = compare_smooth_grads(_model(), x, y)
    report("p2_512_grads_vs_fp64", R=R, worst_G=eg, worst_D=ed, decisions_differing=flips, worst_kink=kink)
    assert eg[1] < 1e-4 and ed[1] < 1e-4, (eg, ed)
    assert kink < KINK, kink


# ---------------------------------------------------------------------------------------------- batch 8

def test_bs8_per_sample_equals_bs1_512(report):
    """The bench's own shape (batch 8 at 512x512: the resblock convs' persistent workgroups stream two
    tiles each, the tile-crossing path of conv_fwd_f3).  InstanceNorm is per sample, so each sample's
    G output / mask / D output at batch 8 equals a batch-1 run of that sample; two samples are also
    checked against the fp32 oracle, and the fused step's pre-update losses at batch 8 equal the torch
    losses (models/model.py:626-631, :643) of the validated module outputs."""
    x, y = _inputs(8, seed=7)
    m = _model()
    xd, yd = x.to(DEV), y.to(DEV)
    with torch.no_grad():
        out8 = m.generator(xd)
        mask8 = m.generator.last_attention_mask.clone()
        dr8 = m.discriminator(torch.cat((xd, yd), 1))
        df8 = m.discriminator(torch.cat((xd, out8), 1))
        errs = []
        for i in (0, 3, 7):
            o1 = m.generator(xd[i:i + 1])
            k1 = m.generator.last_attention_mask
            d1 = m.discriminator(torch.cat((xd[i:i + 1], yd[i:i + 1]), 1))
            errs.append((i, nrel(out8[i:i + 1], o1), nrel(mask8[i:i + 1], k1), nrel(dr8[i:i + 1], d1)))
    Gp, Dp = O.init_params()
    oerr = []
    with torch.no_grad():
        for i in (0, 7):
            fr, mr = O.generator_forward(Gp, x[i:i + 1])
            oerr.append((i, nrel(out8[i:i + 1], fr), nrel(mask8[i:i + 1], mr)))
    ref = np.array([float(F.mse_loss(dr8, torch.ones_like(dr8))), float(F.mse_loss(df8, torch.zeros_like(df8))),
                    100 * float(F.l1_loss(out8, yd))])
    losses = m.step_fn(xd, yd).cpu().numpy().astype(np.float64)
    lrel = np.abs(losses[[0, 1, 3]] - ref) / np.abs(ref)
    report("bs8_512_per_sample", per_sample_vs_bs1=errs, vs_oracle=oerr, step_loss_rel=lrel.tolist(),
           losses=losses.tolist())
    assert max(max(e[1:]) for e in errs) < KTOL, errs
    assert max(max(e[1:]) for e in oerr) < KTOL, oerr
    assert lrel.max() < KTOL, lrel
    assert np.isfinite(losses).all()


def _separable_grads(m, xs, ys, c1, c2, weights=None, g_only=False):
    """HIP executor gradients of L = sum_i w_i [c1 * sum (D(cat(x_i, G(x_i))) - 1)^2 + c2 * sum (G(x_i) - y_i)^2]
    with FIXED scales c1, c2 (not the batch means) and per-sample weights w (default 1): the loss is a sum over
    samples, so its gradients at batch B are the sum of the batch-1 gradients of each sample (InstanceNorm and
    the PatchGAN are per sample).  g_only: the generator term alone (no discriminator).  Returns (G grads,
    D grads, activation decisions {"G": [...], "D": [...]}), cloned."""
    from floodgan import executor as X
    gp, dp = m.generator.param_dict(), m.discriminator.param_dict()
    N, C = xs.shape[0], xs.shape[1]
    w = torch.ones(N, device=xs.device) if weights is None else weights.to(xs.device)
    fake, _, S = X.gen_forward(gp, xs, save=True)
    g_fake = (c2 * w.view(-1, 1, 1, 1) * (fake - ys)).contiguous()
    gD, dec = {}, {"G": [X.gen_act_decisions(S)]}
    if not g_only:
        pred, dS = X.disc_forward(dp, X.disc_pack([(xs, fake)], C + 3), save=True)
        gD = X.disc_backward(dp, dS, (c1 * w.view(-1, 1, 1, 1) * (pred - 1)).contiguous(), param_grads=True,
                             input_grad=g_fake, input_grad_channels=(C, 3), input_grad_accumulate=True)
        dec["D"] = [X.disc_act_decisions(dS)]
        del dS
    gG = X.gen_backward(gp, S, g_fake)
    torch.cuda.synchronize()
    return {k: v.clone() for k, v in gG.items()}, {k: v.clone() for k, v in gD.items()}, dec


C1_512, C2_512 = 2.0 / (62 * 62), 200.0 / (3 * R * R)     # the batch-1 mean scales of compare_smooth_grads


def test_bs8_generator_backward_equals_sum_of_bs1_512(report):
    """The generator backward at the bench's batch 8 (512x512: the resblock weight gradients' split reductions
    over M = 131072 rows, conv_wgrad_f3_kernel<256,0>; the batch-8 input-gradient tile streams) under a
    per-sample-separable smooth loss on G's output: every weight gradient equals the sum of the eight batch-1
    HIP runs to 1e-5 (IN-cancelled biases excluded) when both evaluations take the same
    activation decisions.  They usually do -- the forward reads the same per-sample values -- but where the
    f16x3 operand scale (a power of two from the BATCH absmax) differs between the batch-8 and the batch-1
    evaluation of a tensor, rounding-level differences can flip a ReLU sitting at its kink, and one flip moves
    a whole network's gradients by ~1e-4 (P2); the tolerance is then the flip envelope, 3e-3, and the flips
    are reported.  The exact pin of the batch-8 backward is test_bs8_backward_vs_fp64_512 (teacher-forced)."""
    x, y = _inputs(8, seed=17)
    m = _model()
    xd, yd = x.to(DEV), y.to(DEV)
    g8, _, dec8 = _separable_grads(m, xd, yd, C1_512, C2_512, g_only=True)
    gs, flips = None, 0
    for i in range(8):
        g1, _, dec1 = _separable_grads(m, xd[i:i + 1], yd[i:i + 1], C1_512, C2_512, g_only=True)
        gs = g1 if gs is None else {k: gs[k] + v for k, v in g1.items()}
        for k, v in dec1["G"][0].items():
            flips += int((v[0] != dec8["G"][0][k][i]).sum())
        del g1, dec1
    skip_g, _ = O.cancelled_biases()
    eg = _worst([(k, nrel(v, gs[k])) for k, v in g8.items() if k not in skip_g])
    report("bs8_512_G_backward_vs_sum_bs1", worst_G=eg, decisions_differing_bs8_vs_bs1=flips)
    assert flips <= 200, flips
    assert eg[1] < (1e-5 if flips == 0 else 3e-3), (eg, flips)


def test_bs8_backward_vs_fp64_512(report):
    """The whole smooth G + D loss at batch 8, 512x512 (the D pass on 8 images, D's input gradient into G, the
    G backward) with per-sample weights that keep samples 0 and 5: the batch-8 HIP gradients of every G and
    D parameter equal the fp64 oracle's (the sum of its two batch-1 runs, each with the HIP batch-8 decisions
    of that sample teacher-forced) to 1e-4, every differing decision within rounding of its kink (P2's
    criterion at the bench's shape: the batch-8 kernels, their split reductions and tile streams)."""
    keep = (0, 5)
    x, y = _inputs(8, seed=23)
    m = _model()
    w = torch.zeros(8)
    w[list(keep)] = 1.0
    g8, d8, dec8 = _separable_grads(m, x.to(DEV), y.to(DEV), C1_512, C2_512, weights=w)
    Gp, Dp = O.init_params()
    rG, rD, flips, kink = None, None, 0, 0.0
    for i in keep:
        dec = O.ActDecisions({net: [{k: v[i:i + 1] for k, v in dec8[net][0].items()}] for net in ("G", "D")})
        gG, gD = oracle_smooth_grads(Gp, Dp, x[i:i + 1], y[i:i + 1], dec)
        rG = gG if rG is None else {k: rG[k] + v for k, v in gG.items()}
        rD = gD if rD is None else {k: rD[k] + v for k, v in gD.items()}
        flips += sum(n for _, _, n, _ in dec.log)
        kink = max(kink, dec.worst())
    skip_g, skip_d = O.cancelled_biases()
    eg = _worst([(k, nrel(v, rG[k])) for k, v in g8.items() if k not in skip_g])
    ed = _worst([(k, nrel(v, rD[k])) for k, v in d8.items() if k not in skip_d])
    report("bs8_512_backward_vs_fp64", samples=list(keep), worst_G=eg, worst_D=ed, decisions_differing=flips,
           worst_kink=kink)
    assert eg[1] < 1e-4 and ed[1] < 1e-4, (eg, ed)
    assert kink < KINK, kink


# ---------------------------------------------------------------------------------------------- U

BETA1 = 0.5


def _update_agreement(p0, p_hip, p_ref, g_hip, g_ref, m_ref):
    """(fraction of decided elements whose update direction agrees, norm-relative update error over
    the decided elements, fraction decided, norm-relative error of the whole updated tensor)"""
    p0, p_hip, p_ref, g_hip, g_ref = (t.detach() for t in (p0, p_hip, p_ref, g_hip, g_ref))
    d_hip = (p_hip.double().cpu() - p0.double().cpu()).flatten()
    d_ref = (p_ref.double().cpu() - p0.double().cpu()).flatten()
    dg = (g_hip.double().cpu() - g_ref.double().cpu()).flatten()
    sigma = float(dg.pow(2).mean().sqrt())
    # m_new = beta1*m_old + (1 - beta1)*g with m_old shared, so the direction of an element's update can
    # only differ if (1 - beta1)*|dg_e| >= |m_e|: decided = |m| above 10x that (and 10x the tensor's rms)
    dec = m_ref.double().cpu().flatten().abs() > 10 * (1 - BETA1) * torch.clamp(dg.abs(), min=sigma) + 1e-30
    # and an update the fp32 parameter can hold: |dp| below ~2 ulp of p rounds away in the HIP state
    dec &= d_ref.abs() > p0.double().cpu().flatten().abs() * 2.0 ** -22
    n = int(dec.sum())
    if n == 0:
        return 1.0, 0.0, 0.0, nrel(p_hip, p_ref)
    agree = float((torch.sign(d_hip[dec]) == torch.sign(d_ref[dec])).double().mean())
    err = float((d_hip[dec] - d_ref[dec]).norm() / max(float(d_ref[dec].norm()), 1e-30))
    return agree, err, n / d_ref.numel(), nrel(p_hip, p_ref)


def u_compare(st, rec, P0, P_hip, g_hip):
    """The U criterion for one iteration of a run against the fp64 oracle `st` that continued from the same
    state (PairedStepOracle after step(..., record=rec, d_after=the run's D after Adam(D), decisions=...)).
    P0 / P_hip / g_hip: {"G": {name: tensor}, "D": {...}} -- the run's parameters before and after the
    iteration and the gradients its optimiser steps used.  Returns (rows, bad): per parameter (net, name,
    gradient error, direction agreement of the decided elements, decided-update error, decided fraction,
    whole-tensor error); bad = rows past the bounds (gradient 1e-4, agreement 1.0, decided update 1e-3).
    IN-cancelled biases are skipped (their gradients are rounding noise).  D's last bias gradient
    is a plain sum of the prediction residuals whose terms cancel (mean(pred_fake) + mean(pred_real - 1)): its error
    is measured against the sum's mass (mean |pred_fake| + mean |pred_real - 1|, rec["d_sum_mass"]) when that
    exceeds the sum -- the forward-error bound of a sum -- not against the cancelled result, and then to 1e-5 (a few
    ulp of the forward's rounding); both measures are kept in `sums` {name: (mass-relative,
    plain)}."""
    skip_g, skip_d = O.cancelled_biases()
    mass = rec.get("d_sum_mass", {})
    rows, bad = [], []
    sums = rec.setdefault("sum_errors", {})
    for net, grads, skip, opt_ref, params_ref, order in (
            ("G", rec["g_grads"], skip_g, st.opt_g, st.G, list(st.G)),
            ("D", rec["d_grads"], skip_d, st.opt_d, rec["d_after_own"], list(st.D))):
        for k in order:
            if k in skip:
                continue
            ge = nrel(g_hip[net][k], grads[k])
            gtol = 1e-4
            if net == "D" and k in mass:
                ref = grads[k].detach().double().cpu()
                den = max(float(ref.norm()), mass[k] * ref.numel() ** 0.5, 1e-30)
                plain = ge
                ge = float((g_hip[net][k].detach().double().cpu() - ref).norm()) / den
                sums[k] = (ge, plain)
                gtol = 1e-5
            m_ref = opt_ref.state[opt_ref.param_groups[0]["params"][order.index(k)]]["exp_avg"]
            agree, uerr, frac, perr = _update_agreement(P0[net][k], P_hip[net][k], params_ref[k], g_hip[net][k],
                                                        grads[k], m_ref)
            rows.append((net, k, ge, agree, uerr, frac, perr))
            if ge > gtol or agree < 1.0 or uerr > NTOL:
                bad.append(rows[-1])
    return rows, bad


def u_summary(rows):
    return dict(worst_grad=max(rows, key=lambda r: r[2])[1:3], min_agree=min(r[3] for r in rows),
                worst_update=max(rows, key=lambda r: r[4])[1:5:3], min_decided=min(r[5] for r in rows),
                worst_param_rel=max(rows, key=lambda r: r[6])[1:7:5])


def _teacher_forced_iterations(m, batches, report, name, **tags):
    """Run the fused step over `batches` [(x, y, lr)], one iteration each.  Before each, the fp64 oracle is
    loaded with the HIP state (G, D, both Adam states) and runs the same iteration with the HIP path's
    activation decisions and, for the G half, the HIP discriminator after Adam(D).  Asserted per iteration:
    every G and D gradient within 1e-4, every differing decision at its kink, every decided element's update
    direction agrees and the decided updates agree to 1e-3 (models/model.py:633, :646)."""
    G, D = m.generator, m.discriminator
    m.step_fn.record_decisions = True
    for it, (x, y, lr) in enumerate(batches):
        for opt in (m.optimizer_generator, m.optimizer_discriminator):
            for grp in opt.param_groups:
                grp["lr"] = lr
        g0 = {k: v.detach().clone() for k, v in G.named_parameters()}
        d0 = {k: v.detach().clone() for k, v in D.named_parameters()}
        st = O.PairedStepOracle(dtype=torch.float64, lr=lr, c_in=x.shape[1])
        st.load_state(g0, d0, m.optimizer_generator.state_dict() if it else None,
                      m.optimizer_discriminator.state_dict() if it else None)
        losses = m.step_fn(x.to(DEV), y.to(DEV))
        torch.cuda.synchronize()
        rec = {}
        dec = O.ActDecisions(m.step_fn.decisions)
        ref_losses = st.step(x, y, record=rec, d_after={k: v.detach().cpu() for k, v in D.named_parameters()},
                             decisions=dec)
        rows, bad = u_compare(st, rec, {"G": g0, "D": d0}, {"G": dict(G.named_parameters()),
                                                             "D": dict(D.named_parameters())},
                              {"G": {k: p.grad for k, p in G.named_parameters()},
                               "D": {k: p.grad for k, p in D.named_parameters()}})
        hl = losses.cpu().double().numpy()
        rl = np.array([float(v) for v in ref_losses])
        rl[3] *= 100
        lrel = float(np.max(np.abs(hl - rl) / np.abs(rl)))
        report(name, it=it, **tags, **u_summary(rows), decisions_differing=sum(r[2] for r in dec.log),
               worst_kink=dec.worst(), loss_rel=lrel, bad=bad, sum_errors_mass_plain=rec.get("sum_errors"))
        assert np.isfinite(hl).all(), (it, hl)
        assert dec.worst() < KINK, (it, dec.worst())
        assert not bad, (it, bad)
        # the losses the HIP loop logged vs the oracle's teacher-forced ones (the G loss sees the HIP Adam(D))
        assert lrel < 1e-4, (it, hl, rl)


@pytest.mark.parametrize("R_", [32, 64])
def test_update_teacher_forced_vs_golden_inputs(golden, R_, report):
    """Two iterations on the reference's golden inputs and learning rates (_teacher_forced_iterations)."""
    g = golden(R_)
    batches = [(torch.from_numpy(g[f"x{it}"]), torch.from_numpy(g[f"y{it}"]), float(g[f"it{it}_lr"][0]))
               for it in range(2)]
    _teacher_forced_iterations(_model(), batches, report, "update_teacher_forced", R=R_)


@pytest.mark.parametrize("R_,bs", [(64, 2), (128, 8)])
def test_update_teacher_forced_10_iterations(R_, bs, report):
    """Ten consecutive iterations of the bench's code path (default switches: f16x3 math, pack cache with the
    batched re-pack after each Adam step, pre-split operands and the block copies, the fused statistics
    epilogues) on fresh synthetic batches, each checked against the fp64 oracle continuing from the HIP state
    (_teacher_forced_iterations): the f16x3 scale slots, pack caches and pre-split flags carried across
    iterations must keep every gradient and update within the criterion (VERDICT r3 item 2;
    models/model.py:611-651)."""
    m = _model()
    lr = m.optimizer_generator.param_groups[0]["lr"]
    batches = [_inputs(bs, res=R_, seed=500 + it) + (lr,) for it in range(10)]
    _teacher_forced_iterations(m, batches, report, "update_teacher_forced_10it", R=R_, bs=bs)


def test_update_teacher_forced_512(report):
    """The U criterion at the bench resolution (512x512, batch 2, default switches: f16x3, pack cache, pre-split
    operands, fused statistics): two consecutive iterations, each checked against the fp64 oracle continuing from
    the HIP state with the HIP decisions teacher-forced (_teacher_forced_iterations; models/model.py:611-651,
    updates at :633 and :646).  The second iteration runs on the packs, scale slots and Adam moments the first
    one left behind."""
    m = _model()
    lr = m.optimizer_generator.param_groups[0]["lr"]
    batches = [_inputs(2, seed=600 + it) + (lr,) for it in range(2)]
    _teacher_forced_iterations(m, batches, report, "update_teacher_forced_512", R=R, bs=2)


def test_check_scales_bench_loop_25_steps(report):
    """FLOODGAN_CHECK_SCALES on the bench's shape (512x512, batch 8) for 25 consecutive steps: before every f16x3
    launch each operand is re-measured against the absmax slot the launch scales it by, every cached weight
    pack and split copy is rebuilt and compared bit for bit (ops.check_scale); any stale slot raises.  The loss
    trajectory stays finite."""
    from floodgan import ops
    prev = ops.CHECK_SCALES
    ops.CHECK_SCALES = True
    ops.SCALE_CHECKS.clear()
    try:
        m = _model()
        x, y = _inputs(8, seed=77)
        x, y = x.to(DEV), y.to(DEV)
        losses = [m.step_fn(x, y).cpu() for _ in range(25)]
    finally:
        ops.CHECK_SCALES = prev
    counts = dict(ops.SCALE_CHECKS)
    report("check_scales_bench_loop", steps=25, checks=counts, first=losses[0].tolist(), last=losses[-1].tolist())
    assert all(torch.isfinite(v).all() for v in losses)
    assert counts.get("fp32", 0) > 0 and counts.get("presplit", 0) > 0 and counts.get("pack", 0) > 0, counts
    assert counts.get("split_copy", 0) > 0, counts


def test_f16x3_tracks_exact_fp32_30_steps_512(report):
    """The headline's conv math (f16x3) against the exact-fp32 MFMA math over 30 consecutive training steps at
    512x512, batch 2, from the same seed-47 initialisation and the same batches (4 distinct, cycled), with no teacher
    forcing: the per-step losses and every parameter's total update (p_30 - p_0).  A GAN trajectory amplifies any
    rounding difference (flipped ReLU / L1 kinks, Adam-normalised small gradients), so the yardstick is how far two
    fp32-grade evaluations drift apart on the same trajectory: the exact-fp32 run against (a) the bf16x6 math
    (fp32-equivalent split bf16 products) and (b) itself with the inputs perturbed by one ulp.  f16x3 must stay
    within 3x the larger control.  (The IN-cancelled conv biases, whose updates are Adam-normalised rounding noise
    in any evaluation, are reported apart.)"""
    from floodgan import _lib as L
    steps = 30
    batches = [tuple(t.to(DEV) for t in _inputs(2, seed=900 + b)) for b in range(4)]
    g = torch.Generator(device="cpu").manual_seed(3)
    ulp = [tuple(t * (1 + torch.where(torch.rand(t.shape, generator=g) < 0.5, -1.0, 1.0).to(DEV) * 2.0 ** -23)
                 for t in bt) for bt in batches]
    skip_g, skip_d = O.cancelled_biases()
    runs = {}
    prev = L.get_conv_math()
    try:
        for arm, math, data in (("f16x3", "f16x3", batches), ("fp32", "fp32", batches), ("bf16x6", "bf16x6", batches),
                                ("fp32_ulp", "fp32", ulp)):
            L.set_conv_math(math)
            m = _model()
            nets = {"generator": m.generator, "discriminator": m.discriminator}
            p0 = {f"{n}/{k}": p.detach().double().clone() for n, mod in nets.items() for k, p in mod.named_parameters()}
            losses = torch.stack([m.step_fn(*data[s % 4]).cpu().double() for s in range(steps)])
            upd = {f"{n}/{k}": p.detach().double() - p0[f"{n}/{k}"] for n, mod in nets.items()
                   for k, p in mod.named_parameters()}
            runs[arm] = (losses, upd)
    finally:
        L.set_conv_math(prev)
    l32, u32 = runs["fp32"]
    out = {}
    for arm in ("f16x3", "bf16x6", "fp32_ulp"):
        la, ua = runs[arm]
        lrel = ((la - l32).abs() / l32.abs()).max(dim=1).values
        rows = {}
        for key in u32:
            net, k = key.split("/", 1)
            rows[key] = (nrel(ua[key], u32[key]), k in (skip_g if net == "generator" else skip_d))
        kept = {k: v for k, (v, c) in rows.items() if not c}
        worst_key = max(kept, key=kept.get)
        out[arm] = dict(loss_rel_max=float(lrel.max()), loss_rel_per_step=[float(v) for v in lrel],
                        update_rel_median=float(np.median(list(kept.values()))), update_rel_worst=kept[worst_key],
                        worst_tensor=worst_key,
                        cancelled_update_rel_median=float(np.median([v for v, c in rows.values() if c])))
        print(arm, {k: v for k, v in out[arm].items() if k != "loss_rel_per_step"})
    report("f16x3_vs_fp32_30_steps_512", steps=steps, batch=2, arms=out)
    for arm in out:
        assert np.isfinite(out[arm]["loss_rel_max"])
    ctrl = {k: max(out["bf16x6"][k], out["fp32_ulp"][k]) for k in ("loss_rel_max", "update_rel_median", "update_rel_worst")}
    for k, v in ctrl.items():
        assert out["f16x3"][k] <= 3 * v, (k, out["f16x3"][k], v)


# ---------------------------------------------------------------------------------------------- topography

@pytest.mark.parametrize("c_in,topo", [(3, None), (4, "dem"), (6, "map")])
def test_topography_variants_step(c_in, topo, report):
    """The reference's other input stacks (models/model.py:78: None -> 3, dem/flow/river -> 4, map -> 6
    generator channels; the paired D takes c_in + 3): seed-47 init bit-identical to the oracle's, P1
    losses of one fused step, and P2 gradients (decisions teacher-forced) vs fp64 at 32x32."""
    Rr = 32
    m = _model(topography=topo)
    assert m.generator.conv1.weight.shape[1] == c_in and m.discriminator.model[0].weight.shape[1] == c_in + 3
    Gp, Dp = O.init_params(c_in=c_in)
    for k, v in m.generator.named_parameters():
        assert torch.equal(v.detach().cpu(), Gp[k]), k
    x, y = _inputs(2, c=c_in, res=Rr, seed=c_in)
    eg, ed, flips, kink = compare_smooth_grads(m, x, y, c_in)
    ref = np.array(O.PairedStepOracle(c_in=c_in).step(x, y))
    ref[3] *= 100
    losses = m.step_fn(x.to(DEV), y.to(DEV)).cpu().numpy().astype(np.float64)
    lrel = np.abs(losses - ref) / np.abs(ref)
    report("topography_variant", c_in=c_in, worst_G=eg, worst_D=ed, decisions_differing=flips, worst_kink=kink,
           loss_rel=lrel.tolist())
    assert eg[1] < 1e-4 and ed[1] < 1e-4 and kink < KINK, (eg, ed, kink)
    assert lrel[[0, 1, 3]].max() < KTOL, lrel


# ---------------------------------------------------------------------------------------------- cycle @ 512

@pytest.mark.parametrize("model", ["attentiongan", "cyclegan"])
def test_cycle_p1_losses_512(model, report):
    """BASELINE configs[3]/[4] resolution: the eight iteration-0 losses of CycleStep at 512x512,
    batch 1 (all evaluated before any parameter update: the D losses use pre-update D weights and the
    synthetic images of the pre-update generators) vs the fp32 oracle's forwards (models/model.py:685-737)."""
    from floodgan.model import Model
    g = torch.Generator().manual_seed(31)
    x = torch.rand((1, 9, R, R), generator=g) * 2 - 1
    y = torch.rand((1, 3, R, R), generator=g) * 2 - 1
    P = OC.init_cycle_params(model=model)
    gen = OC.cyclegan_generator_forward if model == "cyclegan" else (lambda p, t: O.generator_forward(p, t)[0])
    D = O.discriminator_forward
    cond = x[:, 3:]
    with torch.no_grad():
        post_real = torch.cat((y, cond), 1)
        sp = torch.cat((gen(P["pre_to_post"], x), cond), 1)
        spre = torch.cat((gen(P["post_to_pre"], post_real), cond), 1)
        rp = gen(P["pre_to_post"], spre)
        rq = gen(P["post_to_pre"], sp)

        def mse(p, t):
            return float(F.mse_loss(p, torch.full_like(p, t)))
        ref = np.array([mse(D(P["post_d"], sp), 1), mse(D(P["pre_d"], spre), 1), 10 * float(F.l1_loss(rq, x[:, :3])),
                        10 * float(F.l1_loss(rp, y)), mse(D(P["pre_d"], x), 1), mse(D(P["post_d"], post_real), 1),
                        mse(D(P["pre_d"], spre), 0), mse(D(P["post_d"], sp), 0)])
    m = Model(model=model, num_epochs=2, topography="all")
    losses = m.cycle_step_fn(x.to(DEV), y.to(DEV)).cpu().numpy().astype(np.float64)
    lrel = np.abs(losses - ref) / np.abs(ref)
    report("cycle_p1_512", model=model, loss_rel=lrel.tolist())
    assert lrel.max() < KTOL, lrel


@pytest.mark.parametrize("model", ["attentiongan", "cyclegan"])
def test_cycle_generator_input_gradient_512(model, report):
    """The cycle path's generator input gradient and weight gradients at 512x512 (smooth loss) vs fp64,
    the generator's ReLU decisions teacher-forced (see P2)."""
    from floodgan import executor as X
    from floodgan.model import Model
    g = torch.Generator().manual_seed(41)
    x = torch.rand((1, 9, R, R), generator=g) * 2 - 1
    y = torch.rand((1, 3, R, R), generator=g) * 2 - 1
    m = Model(model=model, num_epochs=2, topography="all")
    gp = m.pre_to_post_generator.param_dict()
    xd, yd = x.to(DEV), y.to(DEV)
    out, _, S = X.gen_forward(gp, xd, save=True)
    gx = torch.empty_like(xd)
    gG = X.gen_backward(gp, S, ((2.0 / out.numel()) * (out - yd)).contiguous(), input_grad=gx)
    dec = O.ActDecisions({"G": [X.gen_act_decisions(S)]})
    del S
    P = OC.init_cycle_params(model=model)
    names = m.pre_to_post_generator.param_dict()
    ref_names = dict(zip(names, P["pre_to_post"]))      # executor name -> reference state_dict name
    Gd = {k: v.double().requires_grad_(True) for k, v in P["pre_to_post"].items()}
    xr = x.double().requires_grad_(True)
    f = O._forced(dec, "G")
    out_r = OC.cyclegan_generator_forward(Gd, xr, f) if model == "cyclegan" else O.generator_forward(Gd, xr, f)[0]
    F.mse_loss(out_r, y.double()).backward()
    skip = OC.cyclegan_cancelled_biases() if model == "cyclegan" else O.cancelled_biases()[0]
    eg = _worst([(k, nrel(gG[k], Gd[ref_names[k]].grad)) for k in gG if ref_names[k] not in skip])
    e_x = nrel(gx, xr.grad)
    report("cycle_input_grad_512", model=model, input_grad=e_x, worst_G=eg,
           decisions_differing=sum(n for _, _, n, _ in dec.log), worst_kink=dec.worst())
    assert e_x < 1e-4 and eg[1] < 1e-4, (e_x, eg)
    assert dec.worst() < KINK, dec.worst()


# ---------------------------------------------------------------------------------------------- kernels

@pytest.mark.parametrize("cap", [2, 3, 4, 7, 8])
@pytest.mark.parametrize("cfg,case", [(4, (256, 256, 3, 1, 1, "reflect", 20)), (6, (256, 128, 3, 1, 1, "reflect", 19)),
                                      (9, (128, 64, 3, 1, 1, "constant", 21)), (7, (128, 64, 3, 1, 1, "constant", 21)),
                                      (7, (32, 64, 7, 1, 3, "constant", 23)), (1, (128, 256, 4, 2, 1, "constant", 22))])
def test_conv_f3_tile_stream(cfg, case, cap):
    """conv_fwd_f3 with at most `cap` persistent workgroups: every workgroup streams many tiles back to
    back (next tile's k-stages issued during the current tile's last stages and epilogue, setup_issue()
    mid-stream, ragged last tiles) -- the path the bench's 512x512 batch-8 resblock convs take.  With 4 or 8
    workgroups the 4-phase launch also takes the phase-interleaved, round-rotated tile order."""
    from floodgan import _lib as L, ops, plans as PL
    from floodgan.plans import Buf
    cin, cout, k, s, p, mode, H = case
    prev = L.get_conv_math()
    L.set_conv_math("f16x3")
    try:
        L.set_f3_tile(cfg)
        L.load().fg_set_f3_persistent(cap)
        torch.manual_seed(cap + cfg)
        x = torch.randn(3, cin, H, H, dtype=torch.float64)
        w = torch.randn(cout, cin, k, k, dtype=torch.float64) * 0.05
        b = torch.randn(cout, dtype=torch.float64)
        xin = F.pad(x, (p,) * 4, mode=mode) if p else x
        y = F.conv2d(xin, w, b, stride=s)
        X = buf_from(x, p, mode)
        wd = w.float().to(DEV)
        mm = PL.wmap_conv_fwd(wd.shape, X.c)
        Ho = PL.out_size(H, k, s, p)
        Y = Buf.empty(3, Ho, Ho, cout, 0, DEV)
        ops.conv([PL.conv_problem(X, p, k, s, ops.pack_weight(wd, mm), mm, Y, bias=b.float().to(DEV))])
        torch.cuda.synchronize()
        assert nrel(nchw(Y), y) < KTOL
        # a 4-problem launch (ConvTranspose2d phases) crossing problem boundaries mid-stream
        if cin >= 128 and s == 1:
            wt = torch.randn(cin, cout // 2, 3, 3, dtype=torch.float64) * 0.05
            yt = F.conv_transpose2d(x, wt, None, stride=2, padding=1, output_padding=1)
            XT = buf_from(x, 1, "constant")
            wtd = wt.float().to(DEV)
            maps = PL.phase_maps(wtd.shape, 3, 1, XT.c)
            YT = Buf.empty(3, 2 * H, 2 * H, cout // 2, 0, DEV)
            ops.conv(PL.phase_problems(XT, wtd.shape, 3, 1, YT, [ops.pack_weight(wtd, q) for q, _, _ in maps], maps))
            torch.cuda.synchronize()
            assert nrel(nchw(YT), yt) < KTOL
    finally:
        L.set_f3_tile(-1)
        L.load().fg_set_f3_persistent(1)
        L.set_conv_math(prev)


def _log_uniform(shape, lo=-12, hi=0, seed=0):
    g = torch.Generator().manual_seed(seed)
    mag = 10 ** (torch.rand(shape, generator=g, dtype=torch.float64) * (hi - lo) + lo)
    sign = torch.where(torch.rand(shape, generator=g) < 0.5, -1.0, 1.0).double()
    return mag * sign


@pytest.mark.parametrize("case", ["log_uniform", "sample_disparity"])
def test_f16x3_dynamic_range(case, report):
    """f16x3 (per-tensor power-of-two scale, two fp16 pieces) on operands with a heavy dynamic range
    vs fp64 and vs the exact-fp32 MFMA path: 'log_uniform' -- activations and gradients log-uniform
    over 1e-12..1 within one tensor; 'sample_disparity' -- one image of the batch 1e-5 x smaller than
    the other (its elements sit 2^-17 below the tensor's scale)."""
    from floodgan import _lib as L, ops, plans as PL
    from floodgan.plans import Buf
    cin, cout, H = 256, 256, 12
    if case == "log_uniform":
        x = _log_uniform((2, cin, H, H), seed=1)
        gy = _log_uniform((2, cout, H, H), seed=2)
    else:
        torch.manual_seed(3)
        x = torch.randn(2, cin, H, H, dtype=torch.float64)
        x[1] *= 1e-5
        gy = torch.randn(2, cout, H, H, dtype=torch.float64)
        gy[0] *= 1e-5
    torch.manual_seed(4)
    w = torch.randn(cout, cin, 3, 3, dtype=torch.float64) * 0.05
    y_ref = F.conv2d(F.pad(x, (1,) * 4, mode="reflect"), w)
    gw_ref = torch.nn.grad.conv2d_weight(F.pad(x, (1,) * 4, mode="reflect"), w.shape, gy)
    prev = L.get_conv_math()
    res = {}
    try:
        for math in ("fp32", "f16x3"):
            L.set_conv_math(math)
            X = buf_from(x, 1, "reflect")
            wd = w.float().to(DEV)
            mm = PL.wmap_conv_fwd(wd.shape, X.c)
            Y = Buf.empty(2, H, H, cout, 0, DEV)
            ops.conv([PL.conv_problem(X, 1, 3, 1, ops.pack_weight(wd, mm), mm, Y)])
            GY = buf_from(gy, 0, "constant")
            dw = torch.empty(wd.shape, dtype=torch.float32, device=DEV)
            ops.wgrad(PL.wgrad_conv(GY, X, 1, 3, 1, cout), PL.wmap_wgrad(wd.shape, True, X.c, 3), dw)
            torch.cuda.synchronize()
            yo = nchw(Y)
            res[math] = dict(fwd=nrel(yo, y_ref), fwd_per_image=[nrel(yo[i], y_ref[i]) for i in range(2)],
                             wgrad=nrel(dw, gw_ref))
    finally:
        L.set_conv_math(prev)
    report("f16x3_dynamic_range", case=case, **res)
    f3, f32 = res["f16x3"], res["fp32"]
    assert f3["fwd"] < KTOL and f3["wgrad"] < KTOL, res
    # per image: no worse than 1e-5, or than 4x the exact-fp32 path where that is itself above it
    for a, b in zip(f3["fwd_per_image"], f32["fwd_per_image"]):
        assert a < max(KTOL, 4 * b), res


def test_fused_attention_head(report):
    """The attention head's 1x1 conv fused into its input's norm passes (fg_in_apply_head: the logits formed by the
    apply pass, the activation not written; fg_in_bwd_head: the 64-channel input gradient w^T g_logits formed inside
    the norm backward, and the head's weight / bias gradients from the activation recomputed in its statistics pass)
    against the separate conv1x1 forward / input-gradient / weight-gradient kernels, one iteration of the fused step
    (64x64, batch 2) from the same weights: bit-identical losses, attention mask and every gradient except the head's
    own weight and bias (a different summation order: within 1e-6)."""
    from floodgan import executor as X
    x, y = _inputs(2, res=64, seed=11)
    out = []
    prev = X.FUSED_HEAD
    try:
        for fused in (False, True):
            X.FUSED_HEAD = fused
            m = _model()
            ls = m.step_fn(x.to(DEV), y.to(DEV)).cpu()
            torch.cuda.synchronize()
            out.append((ls, {k: p.grad.detach().cpu().clone() for k, p in m.generator.named_parameters()},
                        {k: p.grad.detach().cpu().clone() for k, p in m.discriminator.named_parameters()},
                        m.step_fn.last_mask.detach().cpu().clone()))
    finally:
        X.FUSED_HEAD = prev
    head = {"deconv3_attention.weight", "deconv3_attention.bias"}
    assert torch.equal(out[0][0], out[1][0]), (out[0][0], out[1][0])
    assert torch.equal(out[0][3], out[1][3])
    assert all(torch.equal(out[0][1][k], out[1][1][k]) for k in out[0][1] if k not in head)
    assert all(torch.equal(out[0][2][k], out[1][2][k]) for k in out[0][2])
    errs = {k: nrel(out[1][1][k], out[0][1][k]) for k in head}
    report("fused_attention_head", head_grad_rel=errs)
    assert max(errs.values()) < 1e-6, errs


def test_fused_step_deterministic():
    """Run-to-run determinism of the fused step (every reduction in a fixed order, no atomics in the sums):
    two fresh models trained two iterations on the same batches give bit-identical losses and parameters."""
    x, y = _inputs(2, res=64, seed=3)
    out = []
    for _ in range(2):
        m = _model()
        ls = [m.step_fn(x.to(DEV), y.to(DEV)).cpu() for _ in range(2)]
        torch.cuda.synchronize()
        out.append((torch.stack(ls), [p.detach().cpu().clone() for p in m.generator.parameters()],
                    [p.detach().cpu().clone() for p in m.discriminator.parameters()]))
    assert torch.equal(out[0][0], out[1][0])
    assert all(torch.equal(a, b) for a, b in zip(out[0][1], out[1][1]))
    assert all(torch.equal(a, b) for a, b in zip(out[0][2], out[1][2]))
