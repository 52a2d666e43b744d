"""Pin the CPU oracle (oracle/paired_attention.py) to golden vectors produced by the REAL
reference's Model.train_paired() (tests/golden/make_golden.py)."""
import numpy as np
import pytest
import torch

from oracle import paired_attention as O


def nrel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _check_checksums(gold, prefix, P, skip=()):
    for name, t in P.items():
        if name in skip:
            continue
        ref = gold[f"{prefix}/{name}"]
        t = t.detach().double().flatten()
        idx = torch.linspace(0, t.numel() - 1, 16).long()
        mine = np.concatenate([[t.sum().item(), t.abs().sum().item()], t[:8].numpy(), t[idx].numpy()])
        scale = max(abs(ref[1]), 1e-12)
        assert abs(mine[1] - ref[1]) / scale < 2e-5, (prefix, name, mine[1], ref[1])
        assert np.allclose(mine[2:], ref[2:], rtol=2e-4, atol=2e-6), (prefix, name)


@pytest.mark.parametrize("R", [32, 64])
def test_init_rng_parity(golden, R):
    g = golden(R)
    G, D = O.init_params(seed=47, c_in=9)
    for prefix, P in (("init_G", G), ("init_D", D)):
        for name, t in P.items():
            ref = g[f"{prefix}/{name}"]
            t = t.double().flatten()
            n8 = min(8, t.numel())
            # initial weights must be bit-identical (same RNG stream)
            assert np.array_equal(t[:n8].numpy(), ref[2:2 + n8]), name
            assert abs(t.sum().item() - ref[0]) <= 1e-9 * max(1.0, abs(ref[1])), name


@pytest.mark.parametrize("R", [32, 64])
def test_init_forward(golden, R):
    g = golden(R)
    G, D = O.init_params()
    x0, y0 = torch.from_numpy(g["x0"]), torch.from_numpy(g["y0"])
    with torch.no_grad():
        out, mask = O.generator_forward(G, x0)
        d = O.discriminator_forward(D, torch.cat((x0, y0), 1))
    assert nrel(out, g["init_g_out"]) < 1e-6
    assert nrel(mask, g["init_mask"]) < 1e-6
    assert nrel(d, g["init_d_out"]) < 1e-6


@pytest.mark.parametrize("R", [32, 64])
def test_two_training_iterations(golden, R):
    g = golden(R)
    st = O.PairedStepOracle()
    skip_g, skip_d = O.cancelled_biases()
    x0, y0 = torch.from_numpy(g["x0"]), torch.from_numpy(g["y0"])
    for it in range(2):
        x, y = torch.from_numpy(g[f"x{it}"]), torch.from_numpy(g[f"y{it}"])
        st.set_lr(float(g[f"it{it}_lr"][0]))
        losses = st.step(x, y)
        assert np.allclose(losses, g[f"it{it}_losses"], rtol=1e-4, atol=1e-6), (it, losses)
        with torch.no_grad():
            out, mask = O.generator_forward(st.G, x0)
            d = O.discriminator_forward(st.D, torch.cat((x0, y0), 1))
        assert nrel(out, g[f"it{it}_g_out"]) < 1e-4, it
        assert nrel(mask, g[f"it{it}_mask"]) < 1e-4, it
        assert nrel(d, g[f"it{it}_d_out"]) < 1e-4, it
        _check_checksums(g, f"it{it}_G", st.G, skip_g)
        _check_checksums(g, f"it{it}_D", st.D, skip_d)
