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


def test_image_pool_matches_oracle_buffer_when_full():
    """The device pool and the oracle's ImageBuffer (models/model.py:275-294) draw the same swap /
    keep decisions and indices from the same rng once full: identical returned images."""
    from floodgan.cycle import ImagePool
    pool, ref = ImagePool(size=2, rng=random.Random(7)), OC.ImageBuffer(size=2, rng=random.Random(7))
    swaps = 0
    for i in range(30):
        img = torch.full((1, 3, 2, 2), float(i))
        a, c = pool(img, torch.full((1, 6, 2, 2), float(-i)))
        b = ref(img)
        assert torch.equal(a, b), i
        assert float(c[0, 0, 0, 0]) == -float(a[0, 0, 0, 0])
        swaps += int(float(a[0, 0, 0, 0]) != float(i))
    assert swaps > 5


def test_image_pool_without_conditions():
    """topography=None: the cycle path stores bare synthetic images (no conditions cat)."""
    from floodgan.cycle import ImagePool
    pool = ImagePool(size=1, rng=random.Random(3))
    a, c = pool(torch.zeros(1, 3, 2, 2), None)
    assert c is None
    for i in range(1, 10):
        a, c = pool(torch.full((1, 3, 2, 2), float(i)), None)
        assert c is None


def test_cycle_step_gradient_buckets_cover_every_parameter():
    """CycleStep's flat G / D gradient buffers (one per optimiser group) list each parameter once,
    bucket by bucket in backward-completion order, for both cycle models."""
    from floodgan.cycle import CycleStep
    from floodgan.model import Model
    for name in ("AttentionGAN", "CycleGAN"):
        m = Model(model=name, num_epochs=2, topography="all", device="cpu")
        st = CycleStep(m.pre_to_post_generator, m.post_to_pre_generator, m.pre_discriminator, m.post_discriminator,
                       m.optimizer_generator, m.optimizer_discriminator)
        ng = sum(p.numel() for p in m.optimizer_generator.param_groups[0]["params"])
        nd = sum(p.numel() for p in m.optimizer_discriminator.param_groups[0]["params"])
        assert st.gflat.flat.numel() == ng and st.dflat.flat.numel() == nd
        for p in m.optimizer_generator.param_groups[0]["params"]:
            assert p.grad is not None and p.grad.data_ptr() >= st.gflat.flat.data_ptr()
        # the encoder bucket of each generator is the last one its backward completes
        assert st.gflat.bucket_index("g1.conv1") < st.gflat.bucket_index("g2.deconv1_content")
        assert st.dflat.bucket_index("dpre.model.0") < st.dflat.bucket_index("dpost.model.11")


def test_checkpoint_reload_takes_architecture_from_checkpoint(tmp_path):
    """models/model.py:52-57: a pretrained checkpoint names its own architecture; loading it with
    the default `model` argument rebuilds that architecture with the saved weights."""
    from floodgan.model import Model
    for name, nets in (("AttentionGAN", ("pre_to_post_generator", "pre_discriminator")),
                       ("CycleGAN", ("post_to_pre_generator", "post_discriminator")),
                       ("PairedAttention", ("generator", "discriminator"))):
        m = Model(model=name, num_epochs=3, topography="all", device="cpu", seed=5)
        path = tmp_path / f"{name}.pth.tar"
        torch.save(m.checkpoint(2), path)
        r = Model(load_pretrained_model=True, pretrained_model_path=str(path), device="cpu")
        assert r.model == name.lower() and r.num_epochs == 3 and r.starting_epoch == 3
        for net in nets:
            a, b = getattr(m, net).state_dict(), getattr(r, net).state_dict()
            assert all(torch.equal(a[k], b[k]) for k in a)
