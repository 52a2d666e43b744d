"""Pin the AttentionGAN cycle oracle (oracle/attention_cycle.py) to golden vectors produced by
the REAL reference's Model.train_cycle() (tests/golden/make_golden_cycle.py)."""
import numpy as np
import pytest
import torch

from oracle import attention_cycle as OC
from oracle import paired_attention as O
from test_oracle_golden import _check_checksums, nrel

GOLD_NETS = dict(zip(OC.NETS, ("pre_to_post_generator", "post_to_pre_generator", "pre_discriminator",
                               "post_discriminator")))


def _outputs(P, x0, y0, model="attentiongan"):
    post = torch.cat((y0, x0[:, 3:]), 1)
    with torch.no_grad():
        out = dict(d_pre=O.discriminator_forward(P["pre_d"], x0), d_post=O.discriminator_forward(P["post_d"], post))
        if model == "cyclegan":
            out.update(g_pre_to_post=OC.cyclegan_generator_forward(P["pre_to_post"], x0),
                       g_post_to_pre=OC.cyclegan_generator_forward(P["post_to_pre"], post))
        else:
            a, ma = O.generator_forward(P["pre_to_post"], x0)
            b, mb = O.generator_forward(P["post_to_pre"], post)
            out.update(g_pre_to_post=a, mask_pre_to_post=ma, g_post_to_pre=b, mask_post_to_pre=mb)
        return out


def test_cycle_init_rng_parity(golden):
    g = golden(32, "cycle_step")
    P = OC.init_cycle_params(seed=47, c_in=9)
    for net, gname in GOLD_NETS.items():
        for name, t in P[net].items():
            ref = g[f"init_{gname}/{name}"]
            t = t.double().flatten()
            n8 = min(8, t.numel())
            assert np.array_equal(t[:n8].numpy(), ref[2:2 + n8]), (net, name)   # same RNG stream
            assert abs(t.sum().item() - ref[0]) <= 1e-9 * max(1.0, abs(ref[1])), (net, name)
    assert P["pre_d"]["model.0.weight"].shape == (64, 9, 4, 4)       # AttentionGAN D: input_channels, not +3


def test_cycle_init_forward(golden):
    g = golden(32, "cycle_step")
    P = OC.init_cycle_params()
    x0, y0 = torch.from_numpy(g["x0"]), torch.from_numpy(g["y0"])
    for k, v in _outputs(P, x0, y0).items():
        assert nrel(v, g["init_" + k]) < 1e-6, k


@pytest.mark.parametrize("kind,identity", [("cycle_step", False), ("cycle_step", True)])
def test_cycle_two_training_iterations(golden, kind, identity):
    g = golden("32_id" if identity else 32, kind)
    assert list(g["loss_keys"])[:2] == ["losses_generator_post", "losses_generator_pre"]
    st = OC.CycleStepOracle(identity=identity)
    skip_g, skip_d = O.cancelled_biases()
    x0, y0 = torch.from_numpy(g["x0"]), torch.from_numpy(g["y0"])
    lr = 2e-4
    for it in range(2):
        st.set_lr(lr)
        losses = st.step(torch.from_numpy(g[f"x{it}"]), torch.from_numpy(g[f"y{it}"]))
        assert np.allclose(losses, g[f"it{it}_losses"], rtol=1e-4, atol=1e-6), (it, losses, g[f"it{it}_losses"])
        # after an Adam update the fp32 reference is itself chaotic at ~1e-3
        for k, v in _outputs(st.P, x0, y0).items():
            assert nrel(v, g[f"it{it}_{k}"]) < 1e-4, (it, k)
        for net, gname in GOLD_NETS.items():
            _check_checksums(g, f"it{it}_{gname}", st.P[net], skip_g if net in ("pre_to_post", "post_to_pre") else skip_d)
        lr = float(g[f"it{it}_lr_after"][0])


def test_cyclegan_init_and_forward(golden):
    g = golden(32, "cyclegan_step")
    P = OC.init_cycle_params(model="cyclegan")
    for net, gname in GOLD_NETS.items():
        for name, t in P[net].items():
            ref = g[f"init_{gname}/{name}"]
            t = t.double().flatten()
            assert np.array_equal(t[:min(8, t.numel())].numpy(), ref[2:2 + min(8, t.numel())]), (net, name)
    assert [k for k in P["pre_to_post"]] == [f"{n}.{s}" for n, _, _ in OC.cyclegan_generator_layout() for s in ("weight", "bias")]
    x0, y0 = torch.from_numpy(g["x0"]), torch.from_numpy(g["y0"])
    for k, v in _outputs(P, x0, y0, "cyclegan").items():
        assert nrel(v, g["init_" + k]) < 1e-6, k


def test_cyclegan_two_training_iterations(golden):
    g = golden(32, "cyclegan_step")
    st = OC.CycleStepOracle(model="cyclegan")
    skip_g, (_, skip_d) = OC.cyclegan_cancelled_biases(), O.cancelled_biases()
    x0, y0 = torch.from_numpy(g["x0"]), torch.from_numpy(g["y0"])
    lr = 2e-4
    for it in range(2):
        st.set_lr(lr)
        losses = st.step(torch.from_numpy(g[f"x{it}"]), torch.from_numpy(g[f"y{it}"]))
        assert np.allclose(losses, g[f"it{it}_losses"], rtol=1e-4, atol=1e-6), (it, losses, g[f"it{it}_losses"])
        for k, v in _outputs(st.P, x0, y0, "cyclegan").items():
            assert nrel(v, g[f"it{it}_{k}"]) < 1e-4, (it, k)
        for net, gname in GOLD_NETS.items():
            _check_checksums(g, f"it{it}_{gname}", st.P[net], skip_g if net in ("pre_to_post", "post_to_pre") else skip_d)
        lr = float(g[f"it{it}_lr_after"][0])
