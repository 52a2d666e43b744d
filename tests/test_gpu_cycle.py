"""GPU parity of the AttentionGAN cycle path -- the generator input
gradient, the fused-cat generator input, the reflect-pad adjoint into NCHW, and the CycleStep
iteration -- against the CPU oracle (oracle/attention_cycle.py, pinned to the reference's own
train_cycle by tests/test_oracle_cycle_golden.py) and torch-CPU fp64.  Tolerances as in
test_gpu_parity.py: kernels 1e-5, networks / step 1e-3 (north star)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import attention_cycle as OC
from oracle import paired_attention as O
from test_gpu_parity import DEV, KTOL, NTOL, _fold_cpu, _worst, buf_from, nrel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from floodgan import _lib as L
    L.check(L.load().fg_device_ok(), "device_ok")


def test_tail_input_gradient():
    """fg_tail_bwd's g_x: d(output10)/d(input[:, :3]) = attention10 (models/model_architectures.py:251)."""
    from floodgan import ops
    from floodgan.plans import Buf
    torch.manual_seed(5)
    N, H = 2, 16
    cl = torch.randn(N, 27, H, H, dtype=torch.float64)
    al = torch.randn(N, 10, H, H, dtype=torch.float64)
    x = torch.randn(N, 9, H, H, dtype=torch.float64, requires_grad=True)
    a = torch.softmax(al, 1)
    out = sum(torch.tanh(cl[:, 3 * i:3 * i + 3]) * a[:, i:i + 1] for i in range(9)) + x[:, :3] * a[:, 9:10]
    g = torch.randn_like(out)
    (gx_ref,) = torch.autograd.grad(out, x, g)
    gx = torch.full((N, 9, H, H), 7.0, device=DEV)
    ops.tail_bwd(buf_from(cl, 0, "constant", 32), buf_from(al, 0, "constant", 16), x.detach().float().to(DEV),
                 g.float().to(DEV), Buf.empty(N, H, H, 32, 6, DEV), Buf.empty(N, H, H, 16, 0, DEV), gx=gx)
    torch.cuda.synchronize()
    assert nrel(gx[:, :3], gx_ref[:, :3]) < KTOL
    assert float((gx[:, 3:] - 7.0).abs().max()) == 0.0          # channels >= 3 untouched


@pytest.mark.parametrize("p,c,acc", [(3, 9, 3), (1, 4, 0), (3, 12, 0)])
def test_unfold_nchw(p, c, acc):
    from floodgan import ops
    from floodgan.plans import Buf
    torch.manual_seed(6)
    N, H, W = 2, 13, 17
    gpad = torch.randn(N, c, H + 2 * p, W + 2 * p)
    ref = _fold_cpu(gpad.double(), p)
    G = buf_from(gpad, 0, "constant", c_alloc=(c + 3) // 4 * 4)
    G = Buf(G.t, N, H + 2 * p, W + 2 * p, G.c, 0)
    base = torch.randn(N, c, H, W)
    dst = base.to(DEV).permute(0, 2, 3, 1).contiguous().permute(0, 3, 1, 2)   # non-contiguous NCHW view
    ops.unfold_nchw(G, p, c, dst, acc_channels=acc)
    torch.cuda.synchronize()
    ref = ref.float()
    ref[:, :acc] += base[:, :acc]
    assert nrel(dst, ref) < KTOL


def test_generator_x_extra_equals_cat():
    """gen_forward(x, x_extra=cond) == gen_forward(cat(x, cond)) (the fused cat of :682-689)."""
    from floodgan import executor as X
    from floodgan.model import Model
    torch.manual_seed(8)
    m = Model(model="AttentionGAN", num_epochs=2, topography="all")
    P = m.pre_to_post_generator.param_dict()
    img = torch.rand(2, 3, 32, 32, device=DEV) * 2 - 1
    cond = torch.rand(2, 6, 32, 32, device=DEV) * 2 - 1
    with torch.no_grad():
        a, ma, _ = X.gen_forward(P, img, save=False, x_extra=cond)
        b, mb, _ = X.gen_forward(P, torch.cat((img, cond), 1), save=False)
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(ma, mb)


def _gen_fwd(model, P, x):
    return OC.cyclegan_generator_forward(P, x) if model == "cyclegan" else O.generator_forward(P, x)[0]


def _skip_g(model):
    return OC.cyclegan_cancelled_biases() if model == "cyclegan" else O.cancelled_biases()[0]


@pytest.mark.parametrize("model", ["attentiongan", "cyclegan"])
def test_generator_input_gradient_vs_fp64(model, report):
    """The cycle path's new backward: d loss / d input through the drop-in generator (autograd over
    the fused node) vs the fp64 oracle; a smooth loss so no kink decides the sign."""
    from floodgan.model import Model
    R = 32
    torch.manual_seed(12)
    x = torch.rand(2, 9, R, R) * 2 - 1
    y = torch.rand(2, 3, R, R) * 2 - 1
    m = Model(model=model, num_epochs=2, topography="all")
    P = OC.init_cycle_params(model=model)
    Gd = {k: v.double().requires_grad_(True) for k, v in P["pre_to_post"].items()}
    xr = x.double().requires_grad_(True)
    out_r = _gen_fwd(model, Gd, xr)
    F.mse_loss(out_r, y.double()).backward()
    xd = x.to(DEV).requires_grad_(True)
    out = m.pre_to_post_generator(xd)
    F.mse_loss(out, y.to(DEV)).backward()
    e_x = nrel(xd.grad, xr.grad)
    skip_g = _skip_g(model)
    eg = [(k, nrel(p.grad, Gd[k].grad)) for k, p in m.pre_to_post_generator.named_parameters() if k not in skip_g]
    report("cycle_generator_input_grad_vs_fp64", model=model, R=R, input_grad=e_x, worst_G=_worst(eg))
    assert e_x < 1e-4 and _worst(eg)[1] < 1e-4, (e_x, _worst(eg))


def _cycle_model(identity, model="attentiongan", topography="all"):
    from floodgan.model import Model
    return Model(model=model, num_epochs=2, topography=topography, add_identity_loss=identity)


CASES = [("attentiongan", False), ("attentiongan", True), ("cyclegan", False)]
# topography=None (models/model.py:682-689: no conditions cat, 3-channel generators and discriminators)
CASES_TOPO = [(m, i, "all") for m, i in CASES] + [("attentiongan", True, None), ("cyclegan", False, None)]


@pytest.mark.parametrize("model,identity,topography", CASES_TOPO)
def test_cycle_step_gradients_vs_fp64(model, identity, topography, report):
    """First CycleStep iteration: every G and D gradient vs the fp64 oracle iteration (all of them are
    computed before any parameter update) with every network pass's ReLU / LeakyReLU decisions
    teacher-forced to the HIP path's (oracle.ActDecisions; each differing decision must sit within
    rounding of its kink), and all iteration-0 losses."""
    torch.manual_seed(13)
    R = 32
    c_in = 9 if topography else 3
    x = torch.rand(2, c_in, R, R) * 2 - 1
    y = torch.rand(2, 3, R, R) * 2 - 1
    m = _cycle_model(identity, model, topography)
    m.cycle_step_fn.record_decisions = True
    losses = m.cycle_step_fn(x.to(DEV), y.to(DEV)).cpu().numpy().astype(np.float64)
    dec = O.ActDecisions(m.cycle_step_fn.decisions)
    st = OC.CycleStepOracle(identity=identity, dtype=torch.float64, model=model, c_in=c_in)
    rec = {}
    ref_losses = np.array(st.step(x, y, record=rec, decisions=dec))
    assert not any(dec.queues.values()), "every recorded pass consumed"
    lrel = np.abs(losses - ref_losses) / np.abs(ref_losses)
    skip_g, skip_d = _skip_g(model), O.cancelled_biases()[1]
    errs = {}
    for net, mod, skip in (("pre_to_post", m.pre_to_post_generator, skip_g),
                           ("post_to_pre", m.post_to_pre_generator, skip_g),
                           ("pre_d", m.pre_discriminator, skip_d), ("post_d", m.post_discriminator, skip_d)):
        ref = rec["g_grads" if "_to_" in net else "d_grads"][net]
        errs[net] = _worst([(k, nrel(p.grad, ref[k])) for k, p in mod.named_parameters() if k not in skip])
    report("cycle_step_grads_vs_fp64", model=model, R=R, identity=identity, topography=topography,
           loss_rel=lrel.tolist(), worst={k: list(v) for k, v in errs.items()},
           decisions_differing=sum(n for _, _, n, _ in dec.log), worst_kink=dec.worst())
    assert lrel.max() < 1e-5, lrel
    assert dec.worst() < 1e-4, dec.worst()
    assert max(v[1] for v in errs.values()) < 1e-4, errs


@pytest.mark.parametrize("model,identity", CASES)
def test_cycle_train_vs_reference_golden(golden, model, identity, report):
    """Model.train_cycle (two epochs, one batch each) vs the REFERENCE's own train_cycle run
    (tests/golden/cycle_step_32[_id].npz): iteration-0 losses are pre-update (P1, 1e-5);
    iteration-1 losses and post-update outputs are held to the P3 bound max(1e-3, 2x the
    reference's own fp32 envelope under 1e-6 input noise)."""
    g = golden("32_id" if identity else 32, "cycle_step" if model == "attentiongan" else "cyclegan_step")
    env = [0.0, 0.0, 0.0, 0.0]      # loss it0, loss it1, G out after it1, D out after it1
    x0c = torch.from_numpy(g["x0"])
    for trial in range(1, 3):
        torch.manual_seed(trial)
        st = OC.CycleStepOracle(identity=identity, model=model)
        lr = 2e-4
        for it in range(2):
            st.set_lr(lr)
            x = torch.from_numpy(g[f"x{it}"])
            ls = np.array(st.step(x * (1 + 1e-6 * torch.randn_like(x)), torch.from_numpy(g[f"y{it}"])))
            env[it] = max(env[it], float((np.abs(ls - g[f"it{it}_losses"]) / np.abs(g[f"it{it}_losses"])).max()))
            lr = float(g[f"it{it}_lr_after"][0])
        with torch.no_grad():
            env[2] = max(env[2], nrel(_gen_fwd(model, st.P["pre_to_post"], x0c),
                                      torch.from_numpy(g["it1_g_pre_to_post"])))
            env[3] = max(env[3], nrel(O.discriminator_forward(st.P["pre_d"], x0c), torch.from_numpy(g["it1_d_pre"])))
    m = _cycle_model(identity, model)

    class _Loader:
        def __init__(self):
            self.calls = 0

        def __iter__(self):
            it = self.calls
            self.calls += 1
            return iter([(torch.from_numpy(g[f"x{it}"]), torch.from_numpy(g[f"y{it}"]), ["s"] * 2)])

    m.train_loader = _Loader()
    m.train_cycle()
    keys = [str(k) for k in g["loss_keys"]]
    assert list(m.all_losses) == ["all_" + k for k in keys]
    x0 = torch.from_numpy(g["x0"]).to(DEV)
    y0 = torch.from_numpy(g["y0"]).to(DEV)
    with torch.no_grad():
        out = m.pre_to_post_generator(x0)
        d = m.pre_discriminator(x0)
    e_g = nrel(out, torch.from_numpy(g["it1_g_pre_to_post"]))
    e_d = nrel(d, torch.from_numpy(g["it1_d_pre"]))
    lrel = [np.abs(np.array([m.all_losses["all_" + k][it] for k in keys]) - g[f"it{it}_losses"])
            / np.abs(g[f"it{it}_losses"]) for it in range(2)]
    report("cycle_train_vs_reference_golden", model=model, identity=identity, loss_rel_it0=lrel[0].tolist(),
           loss_rel_it1=lrel[1].tolist(), g_out_after=e_g, d_out_after=e_d, reference_envelope=env)
    assert lrel[0].max() < 1e-5, lrel[0]
    assert lrel[1].max() < max(NTOL, 2 * env[1]), (lrel[1], env)
    assert e_g < max(NTOL, 2 * env[2]) and e_d < max(NTOL, 2 * env[3]), (e_g, e_d, env)
