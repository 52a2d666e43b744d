"""Host-side logic that needs no GPU: the drop-in modules' parameter inventory and RNG parity
with the reference, the no-fallback rule, the optimiser state format, and the C-ABI library's
exported symbols (include/floodgan.h)."""
import os
import re

import numpy as np
import pytest
import torch

from oracle import paired_attention as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _init_ours(seed=47):
    from floodgan.model import Model
    from floodgan.model_architectures import PairedAttentionDiscriminator, PairedAttentionGenerator
    torch.manual_seed(seed)
    G = PairedAttentionGenerator(9).apply(Model.initialise_weights)
    D = PairedAttentionDiscriminator(9).apply(Model.initialise_weights)
    return G, D


def test_state_dict_inventory_matches_reference_layout():
    G, D = _init_ours()
    gl = [(n + s, shape if s == ".weight" else ((shape[1],) if k == "convT" else (shape[0],)))
          for n, k, shape in O.generator_layout(9) for s in (".weight", ".bias")]
    assert [(k, tuple(v.shape)) for k, v in G.state_dict().items()] == [(k, tuple(s)) for k, s in gl]
    dl = [(n + s, shape if s == ".weight" else (shape[0],)) for n, k, shape in O.discriminator_layout(9)
          for s in (".weight", ".bias")]
    assert [(k, tuple(v.shape)) for k, v in D.state_dict().items()] == [(k, tuple(s)) for k, s in dl]
    assert sum(p.numel() for p in G.parameters()) == 11841765
    assert sum(p.numel() for p in D.parameters()) == 2773953


@pytest.mark.parametrize("R", [32])
def test_init_is_bit_identical_to_reference(golden, R):
    """torch.manual_seed(47) + construction + Model.initialise_weights reproduces the reference's
    initial weights exactly (models/model.py:80, 102-104, 162-173)."""
    g = golden(R)
    G, D = _init_ours()
    for prefix, mod in (("init_G", G), ("init_D", D)):
        for name, t in mod.state_dict().items():
            ref = g[f"{prefix}/{name}"]
            t = t.double().flatten()
            n8 = min(8, t.numel())
            assert np.array_equal(t[:n8].numpy(), ref[2:2 + n8]), name
            assert abs(t.sum().item() - ref[0]) <= 1e-9 * max(1.0, abs(ref[1])), name


def test_no_cpu_fallback():
    G, D = _init_ours()
    with pytest.raises(RuntimeError, match="HIP device"):
        G(torch.randn(1, 9, 32, 32))
    with pytest.raises(RuntimeError, match="HIP device"):
        D(torch.randn(1, 12, 32, 32))


def test_fused_adam_state_format_matches_torch_adam():
    from floodgan.optim import FusedAdam
    p = torch.nn.Parameter(torch.zeros(3))
    ours = FusedAdam([p], lr=2e-4, betas=(0.5, 0.999))
    ref = torch.optim.Adam([torch.nn.Parameter(torch.zeros(3))], lr=2e-4, betas=(0.5, 0.999))
    assert ours.state_dict()["param_groups"][0].keys() == ref.state_dict()["param_groups"][0].keys()
    with pytest.raises(NotImplementedError):
        FusedAdam([p], weight_decay=0.1)


def test_model_rejects_unknown_models():
    from floodgan.model import Model
    with pytest.raises(NotImplementedError):
        Model(model="UNet", device="cpu")
    m = Model(model="Pix2Pix", device="cpu")
    assert not m.model_is_cycle and not m.model_is_attention


def test_pix2pix_modules_match_reference_init_and_layout():
    """Pix2Pix drop-ins: torch.manual_seed(47) + construction + initialise_weights reproduces the
    reference's state_dict (parameters and BatchNorm buffers, same keys in the same order) bit for bit
    (tests/golden/pix2pix_step_256.npz from the reference's own Model)."""
    from floodgan import pix2pix as P2P
    from floodgan.model import Model
    gold = np.load(os.path.join(ROOT, "tests", "golden", "pix2pix_step_256.npz"))
    m = Model(model="Pix2Pix", device="cpu")
    for prefix, mod in (("init_G", m.generator), ("init_D", m.discriminator)):
        keys = [k for k in (f.replace("__", ".") for f in gold.files) if k.startswith(prefix + "/")]
        assert [prefix + "/" + k for k in mod.state_dict()] == keys
        for name, t in mod.state_dict().items():
            ref = gold[f"{prefix}/{name}".replace(".", "__")]
            t = t.double().flatten()
            n8 = min(8, t.numel())
            assert np.array_equal(t[:n8].numpy(), ref[2:2 + n8]), name
            assert abs(t.sum().item() - ref[0]) <= 1e-9 * max(1.0, abs(ref[1])), name
    # the executor's parameter inventory / bucket layout cover every parameter exactly once
    assert list(m.generator.param_dict()) == [k for k, _ in m.generator.named_parameters()]
    assert sorted(k for b in P2P.gen_bucket_names() for k in b) == sorted(m.generator.param_dict())
    assert sorted(k for b in P2P.disc_bucket_names() for k in b) == sorted(m.discriminator.param_dict())
    assert sum(p.numel() for p in m.generator.parameters()) == 54420099     # U-Net-256 with 9 input channels
    with pytest.raises(RuntimeError, match="HIP device"):
        m.generator(torch.randn(1, 9, 256, 256))


def test_lambda_rule_matches_reference():
    from floodgan.model import Model
    m = Model(model="PairedAttention", num_epochs=2, device="cpu")
    for e in range(4):
        assert m.lambda_rule(e) == O.lambda_rule(e, 2)
    assert m.optimizer_generator.param_groups[0]["lr"] == pytest.approx(2e-4)
    m1 = Model(model="PairedAttention", num_epochs=1, device="cpu")
    assert m1.optimizer_generator.param_groups[0]["lr"] == pytest.approx(2e-4 * 2 / 3)


def test_c_abi_library_exports_every_declared_symbol():
    """The library loads (no GPU needed) and exports every function include/floodgan.h declares;
    the ctypes table in floodgan/_lib.py binds exactly that set."""
    from floodgan import _lib as L
    lib = L.load()
    header = open(os.path.join(ROOT, "include", "floodgan.h")).read()
    declared = set(re.findall(r"^\s*(?:const\s+)?[a-z_ ]+\*?\s*(fg_[a-z0-9_]+)\s*\(", header, re.M))
    assert declared, "no declarations parsed"
    for name in declared:
        assert hasattr(lib, name), name
    assert declared == set(L.SIGNATURES), declared ^ set(L.SIGNATURES)
    assert lib.fg_version() >= 1
    assert lib.fg_in_workspace_doubles(8, 256) > 0


def test_two_n_batched_d_step_equals_reference_two_calls():
    """The fused step evaluates D(fake) and D(real) as ONE 2N batch (InstanceNorm is per
    sample): loss and gradients equal the reference's two calls (models/model.py:624-632)."""
    torch.manual_seed(3)
    _, D = O.init_params()
    x = torch.rand(2, 9, 32, 32) * 2 - 1
    f = torch.rand(2, 3, 32, 32) * 2 - 1
    y = torch.rand(2, 3, 32, 32) * 2 - 1
    Da = {k: v.double().requires_grad_(True) for k, v in D.items()}
    Db = {k: v.double().requires_grad_(True) for k, v in D.items()}
    F = torch.nn.functional
    pf = O.discriminator_forward(Da, torch.cat((x, f), 1).double())
    pr = O.discriminator_forward(Da, torch.cat((x, y), 1).double())
    la = (F.mse_loss(pf, torch.zeros_like(pf)) + F.mse_loss(pr, torch.ones_like(pr))) * 0.5
    la.backward()
    both = torch.cat((torch.cat((x, f), 1), torch.cat((x, y), 1)), 0).double()
    p = O.discriminator_forward(Db, both)
    lb = (F.mse_loss(p[:2], torch.zeros_like(p[:2])) + F.mse_loss(p[2:], torch.ones_like(p[2:]))) * 0.5
    lb.backward()
    assert abs(float(la) - float(lb)) < 1e-12
    for k in D:
        assert torch.allclose(Da[k].grad, Db[k].grad, rtol=1e-10, atol=1e-14), k
