"""Pin the Pix2Pix CPU oracle (oracle/pix2pix.py) to golden vectors produced by the REAL reference's
Model(model="pix2pix").train_paired() (tests/golden/make_golden_pix2pix.py): initial state_dict
(RNG order of construction + initialise_weights, BatchNorm buffers), the losses of two training
iterations (Dropout masks from the reseeded global generator, BatchNorm batch statistics), the state
after each iteration (Adam, BatchNorm running statistics) and G / D outputs in training mode."""
import copy
import os

import numpy as np
import pytest
import torch

from oracle import pix2pix as OP

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# (file, batch, generator input channels): topography="all" at batch 2, and BASELINE.json configs[0] --
# topography=None (3-ch RGB), batch 1
CASES = {"all_bs2": ("pix2pix_step_256.npz", 2, 9), "rgb_bs1": ("pix2pix_step_256_rgb_bs1.npz", 1, 3)}


def load_gold(case):
    z = np.load(os.path.join(GOLDEN_DIR, CASES[case][0]))
    return {k.replace("__", "."): z[k] for k in z.files}


@pytest.fixture(scope="module", params=sorted(CASES))
def case(request):
    return request.param


@pytest.fixture(scope="module")
def gold(case):
    return load_gold(case)


def synth_inputs(R=256, N=2, C=9):
    """tests/golden/make_golden.py synth(): x ~ U[-1,1)^(N,C,R,R), then y ~ U[-1,1)^(N,3,R,R), twice"""
    gen = torch.Generator().manual_seed(1234)
    out = []
    for _ in range(2):
        x = torch.rand((N, C, R, R), generator=gen) * 2 - 1
        y = torch.rand((N, 3, R, R), generator=gen) * 2 - 1
        out.append((x, y))
    return out


def probe_sample(g):
    g = g.detach().double().flatten()
    idx = torch.linspace(0, g.numel() - 1, 8192).long()
    return np.concatenate([[g.sum().item(), g.abs().sum().item()], g[idx].numpy()])


def probe(st_or_GD, x0, y0):
    """G(x0), D(cat(x0,y0)) in training mode on copies under manual_seed(99) (the golden's probe)"""
    (gp, gb), (dp, db) = st_or_GD
    with torch.no_grad(), torch.random.fork_rng(devices=[]):
        torch.manual_seed(99)
        g = OP.generator_forward(gp, copy.deepcopy(gb), x0)
        d = OP.discriminator_forward(dp, copy.deepcopy(db), torch.cat((x0, y0), 1))
    return probe_sample(g), d.numpy()


def nrel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _check(gold, prefix, P, rtol, elementwise=True):
    for name, t in P.items():
        ref = gold[f"{prefix}/{name}"]
        t = t.detach().double().flatten()
        idx = torch.linspace(0, t.numel() - 1, 16).long()
        mine = np.concatenate([[t.sum().item(), t.abs().sum().item()], t[:8].numpy(), t[idx].numpy()])
        scale = max(abs(ref[1]), 1e-12)
        assert abs(mine[1] - ref[1]) / scale < rtol, (prefix, name, mine[1], ref[1])
        assert abs(mine[0] - ref[0]) / scale < rtol, (prefix, name, mine[0], ref[0])
        if elementwise:
            assert np.allclose(mine[2:], ref[2:], rtol=max(rtol * 10, 1e-5), atol=1e-6), (prefix, name)
        else:
            # after the second step, kink-level gradient differences (deep levels hold 2x2 pixels)
            # move an element's Adam update by a fraction of its lr: bound it at 10% of the total
            # displacement Adam allows (lr 2e-4 + 1e-4)
            assert np.abs(mine[2:] - ref[2:]).max() < 0.1 * 3e-4, (prefix, name)


def test_layout_names_match_golden(gold, case):
    (gp, gb), (dp, db) = OP.init_params(c_in=CASES[case][2])
    mine = {f"init_G/{k}" for k in list(gp) + list(gb)} | {f"init_D/{k}" for k in list(dp) + list(db)}
    theirs = {k for k in gold if k.startswith("init_G/") or k.startswith("init_D/")}
    assert mine == theirs


def test_init_rng_parity(gold, case):
    (gp, gb), (dp, db) = OP.init_params(seed=47, c_in=CASES[case][2])
    for prefix, P in (("init_G", {**gp, **gb}), ("init_D", {**dp, **db})):
        for name, t in P.items():
            ref = gold[f"{prefix}/{name}"]
            t = t.double().flatten()
            n8 = min(8, t.numel())
            assert np.array_equal(t[:n8].numpy(), ref[2:2 + n8]), name      # same RNG stream: bit-identical
            assert abs(t.sum().item() - ref[0]) <= 1e-9 * max(1.0, abs(ref[1])), name


def test_init_forward_training_mode(gold, case):
    _, n, c = CASES[case]
    (x0, y0), _ = synth_inputs(N=n, C=c)
    g, d = probe(OP.init_params(c_in=c), x0, y0)
    assert nrel(g[2:], gold["init_g_out"][2:]) < 1e-6
    assert abs(g[0] - gold["init_g_out"][0]) <= 1e-5 * gold["init_g_out"][1]
    assert nrel(d, gold["init_d_out"]) < 1e-6


def test_two_training_iterations(gold, case):
    _, n, c = CASES[case]
    batches = synth_inputs(N=n, C=c)
    x0, y0 = batches[0]
    st = OP.Pix2PixStepOracle(c_in=c)
    for it, (x, y) in enumerate(batches):
        st.set_lr(float(gold[f"it{it}_lr"][0]))
        torch.manual_seed(it + 1)                        # train_paired: torch.manual_seed(epoch)
        losses = st.step(x, y)
        assert np.allclose(losses, gold[f"it{it}_losses"], rtol=1e-5, atol=1e-7), (it, losses)
        g, d = probe(((st.G, st.GB), (st.D, st.DB)), x0, y0)
        # iteration 0 updates from gradients that agree to summation order; after the second Adam step
        # elements with rounding-level gradients may have moved differently (the P3 bound)
        tol = 1e-4 if it == 0 else 1e-3
        assert nrel(g[2:], gold[f"it{it}_g_out"][2:]) < tol, it
        assert nrel(d, gold[f"it{it}_d_out"]) < tol, it
        _check(gold, f"it{it}_G", {**st.G, **st.GB}, tol / 5, it == 0)
        _check(gold, f"it{it}_D", {**st.D, **st.DB}, tol / 5, it == 0)
