"""Host-side checks of the AttentionGAN cycle path (no GPU): module inventory and RNG parity
of Model(model="AttentionGAN") against the reference's own initial weights (golden from its
train_cycle run), optimiser parameter order, loss keys, checkpoint keys, and the image pool."""
import random

import numpy as np
import torch

from oracle import attention_cycle as OC

NETS = dict(zip(("pre_to_post_generator", "post_to_pre_generator", "pre_discriminator", "post_discriminator"),
                OC.NETS))


def _model(identity=False):
    from floodgan.model import Model
    return Model(model="AttentionGAN", num_epochs=2, topography="all", device="cpu", add_identity_loss=identity)


def test_attentiongan_init_is_bit_identical_to_reference(golden):
    g = golden(32, "cycle_step")
    m = _model()
    for net in NETS:
        for name, t in getattr(m, net).state_dict().items():
            ref = g[f"init_{net}/{name}"]
            t = t.double().flatten()
            n8 = min(8, t.numel())
            assert np.array_equal(t[:n8].numpy(), ref[2:2 + n8]), (net, name)
            assert abs(t.sum().item() - ref[0]) <= 1e-9 * max(1.0, abs(ref[1])), (net, name)
    assert m.pre_discriminator.model[0].weight.shape == (64, 9, 4, 4)


def test_attentiongan_optimiser_order_and_losses():
    m = _model(identity=True)
    g_params = list(m.pre_to_post_generator.parameters()) + list(m.post_to_pre_generator.parameters())
    d_params = list(m.post_discriminator.parameters()) + list(m.pre_discriminator.parameters())
    assert m.optimizer_generator.param_groups[0]["params"] == g_params       # models/model.py:110-112
    assert m.optimizer_discriminator.param_groups[0]["params"] == d_params   # models/model.py:113-115
    keys = list(m.initialise_loss_storage(overall=False))
    assert keys[:2] == ["losses_generator_post", "losses_generator_pre"] and len(keys) == 10
    ck = m.checkpoint(1)
    for k in NETS:
        assert k in ck
    assert "generator" not in ck


def test_attentiongan_loss_keys_match_reference(golden):
    g = golden("32_id", "cycle_step")
    m = _model(identity=True)
    assert list(m.initialise_loss_storage(overall=False)) == [str(k) for k in g["loss_keys"]]


def test_image_pool_semantics():
    from floodgan.cycle import ImagePool
    pool = ImagePool(size=3, rng=random.Random(0))
    imgs = [(torch.full((1, 3, 2, 2), float(i)), torch.full((1, 6, 2, 2), float(-i))) for i in range(40)]
    for i in range(3):                                   # not full: store and return the new image
        a, b = pool(*imgs[i])
        assert a is imgs[i][0] and float(b[0, 0, 0, 0]) == -i
    swapped = kept = 0
    for i in range(3, 40):
        a, b = pool(*imgs[i])
        if a is imgs[i][0]:
            kept += 1
        else:
            swapped += 1
            assert float(a[0, 0, 0, 0]) == -float(b[0, 0, 0, 0])      # pairs stay together
    assert swapped > 5 and kept > 5
    assert len(pool.images) == 3


def test_cyclegan_modules_match_reference_layout_and_init(golden):
    """CycleGAN: Sequential state_dict keys / shapes in the reference's order, bit-identical
    seed-47 initial weights (golden from the reference's own construction)."""
    from floodgan.model import Model
    from floodgan.model_architectures import CYCLEGAN_GEN_KEYS
    g = golden(32, "cyclegan_step")
    m = Model(model="CycleGAN", num_epochs=2, topography="all", device="cpu")
    lay = OC.cyclegan_generator_layout(9)
    want = [(n + s, shape if s == ".weight" else ((shape[1],) if k == "convT" else (shape[0],)))
            for n, k, shape in lay for s in (".weight", ".bias")]
    sd = m.pre_to_post_generator.state_dict()
    assert [(k, tuple(v.shape)) for k, v in sd.items()] == [(k, tuple(s)) for k, s in want]
    assert len(m.pre_to_post_generator.param_dict()) == len(CYCLEGAN_GEN_KEYS) == len(sd)
    for net in NETS:
        for name, t in getattr(m, net).state_dict().items():
            ref = g[f"init_{net}/{name}"]
            t = t.double().flatten()
            n8 = min(8, t.numel())
            assert np.array_equal(t[:n8].numpy(), ref[2:2 + n8]), (net, name)
            assert abs(t.sum().item() - ref[0]) <= 1e-9 * max(1.0, abs(ref[1])), (net, name)
