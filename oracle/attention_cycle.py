"""CPU ORACLE for the AttentionGAN cycle training step -- TEST INFRASTRUCTURE ONLY.

Like oracle/paired_attention.py this is the checker, never the product: only `tests/` (and
`__graft_entry__.smoke()` / `bench.py`'s cpu_baseline leg) may import it.

Functional restatement on PyTorch-CPU of:

  generator     models/model_architectures.py:163-258 (AttentionGANGenerator: layer for layer the
                PairedAttention generator, so generator_forward is shared); CycleGAN's ResNet
                generator :91-134 (cyclegan_generator_forward)
  discriminator models/model_architectures.py:278-299 (PatchGAN over input_channels, not +3; CycleGAN's
                :136-157 is the same network)
  init          models/model.py:80, :97-100 (pre_to_post G, post_to_pre G, pre D, post D, each
                constructed then .apply(initialise_weights)), :162-173
  optimisers    models/model.py:110-115 (Adam over chain(G_pre_to_post, G_post_to_pre) and over
                chain(D_post, D_pre), lr 2e-4, betas (0.5, 0.999))
  train step    models/model.py:677-752 (Model.train_cycle inner iteration)
  image buffer  models/model.py:275-294 (get_buffer_image; < 50 stored images => returns the new one)

Parity pin: tests/test_oracle_cycle_golden.py checks it against tests/golden/cycle_step_32[_id].npz
and cyclegan_step_32.npz,
produced by tests/golden/make_golden_cycle.py from the reference's unmodified train_cycle().
"""
import random
from collections import OrderedDict

import torch
import torch.nn.functional as F

from .paired_attention import (_act, _construct, _forced, _initialise, discriminator_forward, discriminator_layout,
                               generator_forward, generator_layout)

NETS = ("pre_to_post", "post_to_pre", "pre_d", "post_d")


def cyclegan_generator_layout(c_in=9):
    """models/model_architectures.py:95-117 in construction (= registration) order; the
    nn.Sequential indices: 1, 4, 7 convs, 10..18 CycleGANBlocks (conv_block.1 / .5), 19, 22
    transposed convs, 26 the 7x7 head."""
    L = [("model.1", "conv", (64, c_in, 7, 7)), ("model.4", "conv", (128, 64, 3, 3)),
         ("model.7", "conv", (256, 128, 3, 3))]
    for i in range(9):
        L += [(f"model.{10 + i}.conv_block.1", "conv", (256, 256, 3, 3)),
              (f"model.{10 + i}.conv_block.5", "conv", (256, 256, 3, 3))]
    L += [("model.19", "convT", (256, 128, 3, 3)), ("model.22", "convT", (128, 64, 3, 3)),
          ("model.26", "conv", (3, 64, 7, 7))]
    return L


def _in(x):
    return F.instance_norm(x, eps=1e-5)


def cyclegan_generator_forward(P, x, forced=None):
    """models/model_architectures.py:95-120 (CycleGANBlock.forward :132-134).  forced: teacher-forced
    ReLU decisions keyed by the executor's layer names (conv1..3, block<i>, deconv1/2_content)."""
    def conv(name, h, stride=1, padding=0):
        return F.conv2d(h, P[name + ".weight"], P[name + ".bias"], stride=stride, padding=padding)

    def convT(name, h):
        return F.conv_transpose2d(h, P[name + ".weight"], P[name + ".bias"], stride=2, padding=1, output_padding=1)

    h = _act(_in(conv("model.1", F.pad(x, (3, 3, 3, 3), mode="reflect"))), 0, "conv1", forced)
    h = _act(_in(conv("model.4", h, 2, 1)), 0, "conv2", forced)
    h = _act(_in(conv("model.7", h, 2, 1)), 0, "conv3", forced)
    for i in range(9):
        pre = f"model.{10 + i}.conv_block."
        r = _act(_in(conv(pre + "1", F.pad(h, (1, 1, 1, 1), mode="reflect"))), 0, f"block{i}", forced)
        h = h + _in(conv(pre + "5", F.pad(r, (1, 1, 1, 1), mode="reflect")))
    h = _act(_in(convT("model.19", h)), 0, "deconv1_content", forced)
    h = _act(_in(convT("model.22", h)), 0, "deconv2_content", forced)
    return torch.tanh(conv("model.26", F.pad(h, (3, 3, 3, 3), mode="reflect")))


def cyclegan_cancelled_biases():
    """conv biases feeding an InstanceNorm in the CycleGAN generator (all but model.26)"""
    return {n + ".bias" for n, _, _ in cyclegan_generator_layout()[:-1]}


def init_cycle_params(seed=47, c_in=9, model="attentiongan"):
    """models/model.py:80, :97-100: manual_seed(seed) then G_pre_to_post, G_post_to_pre, D_pre,
    D_post, each built (nn.Conv2d RNG) and re-initialised (N(0, 0.02)) before the next."""
    torch.manual_seed(seed)
    gl = generator_layout(c_in) if model == "attentiongan" else cyclegan_generator_layout(c_in)
    dl = discriminator_layout(c_in, extra=0)
    return OrderedDict((n, _initialise(_construct(L), L)) for n, L in zip(NETS, (gl, gl, dl, dl)))


class ImageBuffer:
    """models/model.py:275-294 (pool of 50 past synthetic images), held on the oracle's device."""

    def __init__(self, size=50, rng=None):
        self.size, self.images, self.rng = size, [], rng or random.Random()

    def __call__(self, image):
        image = image.detach()
        if len(self.images) < self.size:
            self.images.append(image.clone())
            return image
        if self.rng.uniform(0, 1) > 0.5:
            i = self.rng.randint(0, self.size - 1)
            old, self.images[i] = self.images[i], image.clone()
            return old
        return image


class CycleStepOracle:
    """Holds the four networks + the two Adam optimisers and performs reference train_cycle
    iterations (models/model.py:677-752) with autograd on the CPU."""

    def __init__(self, params=None, seed=47, c_in=9, lr=2e-4, identity=False, dtype=torch.float32,
                 model="attentiongan"):
        params = params or init_cycle_params(seed, c_in, model)
        self.model = model
        self.P = OrderedDict((n, OrderedDict((k, v.detach().clone().to(dtype).requires_grad_(True))
                                             for k, v in params[n].items())) for n in NETS)
        G1, G2, D1, D2 = (list(self.P[n].values()) for n in NETS)
        self.opt_g = torch.optim.Adam(G1 + G2, lr=lr, betas=(0.5, 0.999))
        self.opt_d = torch.optim.Adam(D2 + D1, lr=lr, betas=(0.5, 0.999))
        self.identity, self.dtype = identity, dtype
        self.pre_buffer, self.post_buffer = ImageBuffer(), ImageBuffer()

    def set_lr(self, lr):
        for opt in (self.opt_g, self.opt_d):
            for g in opt.param_groups:
                g["lr"] = lr

    def _g(self, name, x):
        f = _forced(self._dec, name)
        if self.model == "cyclegan":
            return cyclegan_generator_forward(self.P[name], x, f)
        return generator_forward(self.P[name], x, f)[0]

    def _d(self, name, x):
        return discriminator_forward(self.P[name], x, _forced(self._dec, name))

    _dec = None

    def step(self, input_stack, output_image, record=None, decisions=None):
        """One iteration; returns the losses in the reference's `losses` dict order
        (models/model.py:189-199, appended at :741-752).  decisions (tests only): ActDecisions keyed
        by network name (NETS), each queue in that network's call order."""
        self._dec = decisions
        real_pre = input_stack.to(self.dtype)
        conditions = real_pre[:, 3:].detach().clone()
        real_post = torch.cat((output_image.to(self.dtype), conditions), 1)
        syn_post = self._g("pre_to_post", real_pre)
        syn_pre = self._g("post_to_pre", real_post)
        syn_post = torch.cat((syn_post, conditions), 1)
        syn_pre = torch.cat((syn_pre, conditions), 1)
        rec_post = self._g("pre_to_post", syn_pre)
        rec_pre = self._g("post_to_pre", syn_post)
        # generators (D frozen)
        for n in ("pre_d", "post_d"):
            for p in self.P[n].values():
                p.requires_grad_(False)
        self.opt_g.zero_grad()
        id_post = id_pre = 0
        if self.identity:
            id_post = F.l1_loss(self._g("pre_to_post", real_post), real_post[:, :3]) * 5
            id_pre = F.l1_loss(self._g("post_to_pre", real_pre), real_pre[:, :3]) * 5
        pd = self._d("post_d", syn_post)
        g_post = F.mse_loss(pd, torch.ones_like(pd))
        pp = self._d("pre_d", syn_pre)
        g_pre = F.mse_loss(pp, torch.ones_like(pp))
        cyc_pre = F.l1_loss(rec_pre, real_pre[:, :3]) * 10
        cyc_post = F.l1_loss(rec_post, real_post[:, :3]) * 10
        (g_post + g_pre + cyc_pre + cyc_post + id_post + id_pre).backward()
        if record is not None:
            record["g_grads"] = {n: OrderedDict((k, v.grad.detach().clone()) for k, v in self.P[n].items())
                                 for n in ("pre_to_post", "post_to_pre")}
        self.opt_g.step()
        # discriminators
        for n in ("pre_d", "post_d"):
            for p in self.P[n].values():
                p.requires_grad_(True)
        self.opt_d.zero_grad()
        syn_pre = self.pre_buffer(syn_pre)
        syn_post = self.post_buffer(syn_post)
        pr = self._d("pre_d", real_pre)
        d_pre_real = F.mse_loss(pr, torch.ones_like(pr))
        ps = self._d("pre_d", syn_pre.detach())
        d_pre_syn = F.mse_loss(ps, torch.zeros_like(ps))
        ((d_pre_real + d_pre_syn) * 0.5).backward()
        pr = self._d("post_d", real_post)
        d_post_real = F.mse_loss(pr, torch.ones_like(pr))
        ps = self._d("post_d", syn_post.detach())
        d_post_syn = F.mse_loss(ps, torch.zeros_like(ps))
        ((d_post_real + d_post_syn) * 0.5).backward()
        if record is not None:
            record["d_grads"] = {n: OrderedDict((k, v.grad.detach().clone()) for k, v in self.P[n].items())
                                 for n in ("pre_d", "post_d")}
        self.opt_d.step()
        self._dec = None
        out = [g_post, g_pre, cyc_pre, cyc_post, d_pre_real, d_post_real, d_pre_syn, d_post_syn]
        if self.identity:
            out += [id_post, id_pre]
        return [float(v.detach()) for v in out]
