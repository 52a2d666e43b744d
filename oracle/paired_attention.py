"""CPU ORACLE for the PairedAttention paired-GAN training step -- TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg may import it.  The product path (flood-prediction-gan_amd/
floodgan) never imports it and fails loudly when its HIP library is missing.

It is a functional restatement, on PyTorch-CPU fp32 (or fp64) ops, of the reference's
algorithm for the hot path:

  generator     models/model_architectures.py:305-400  (PairedAttentionGenerator.forward :339-400)
  resnet block  models/model_architectures.py:402-418  (PairedAttentionBlock.forward :412-418)
  discriminator models/model_architectures.py:420-441
  init          models/model.py:80 (seed), :102-104 (construct + .apply), :162-173 (N(0,0.02), bias 0)
  optimiser     models/model.py:121-124 (Adam lr 2e-4, betas (0.5, 0.999)), :175-181 (LambdaLR rule)
  train step    models/model.py:611-651 (Model.train_paired inner iteration)

Parity pin: tests/test_oracle_golden.py checks this restatement against golden vectors that
tests/golden/make_golden.py produced by running the reference's own, unmodified
`Model.train_paired()` in the build container (see that script's header).

Parameters are held in a plain ordered dict `name -> tensor` whose keys, shapes and order
are exactly the reference modules' `state_dict()` keys.
"""
import copy
import math
from collections import OrderedDict

import torch
import torch.nn.functional as F

EPS_IN = 1e-5  # nn.InstanceNorm2d default eps (affine=False, track_running_stats=False)

# ---------------------------------------------------------------------------------------
# parameter inventory (name, kind, shape) in registration order
# ---------------------------------------------------------------------------------------


def generator_layout(c_in=9):
    """(name, 'conv'|'convT', weight shape) in the reference's registration order
    (models/model_architectures.py:312-334)."""
    L = [("conv1", "conv", (64, c_in, 7, 7)),
         ("conv2", "conv", (128, 64, 3, 3)),
         ("conv3", "conv", (256, 128, 3, 3))]
    for i in range(9):
        L += [(f"resnet_blocks.{i}.conv1", "conv", (256, 256, 3, 3)),
              (f"resnet_blocks.{i}.conv2", "conv", (256, 256, 3, 3))]
    L += [("deconv1_content", "convT", (256, 128, 3, 3)),
          ("deconv2_content", "convT", (128, 64, 3, 3)),
          ("deconv3_content", "conv", (27, 64, 7, 7)),
          ("deconv1_attention", "convT", (256, 128, 3, 3)),
          ("deconv2_attention", "convT", (128, 64, 3, 3)),
          ("deconv3_attention", "conv", (10, 64, 1, 1))]
    return L


def discriminator_layout(c_in=9, extra=3):
    """models/model_architectures.py:424-438: Sequential indices 0, 2, 5, 8, 11 hold convs.
    extra = 3 for the paired D (input_channels + 3, :424), 0 for AttentionGAN's (:281)."""
    return [("model.0", "conv", (64, c_in + extra, 4, 4)),
            ("model.2", "conv", (128, 64, 4, 4)),
            ("model.5", "conv", (256, 128, 4, 4)),
            ("model.8", "conv", (512, 256, 4, 4)),
            ("model.11", "conv", (1, 512, 4, 4))]


def _construct(layout):
    """Consume the global RNG exactly like nn.Conv2d / nn.ConvTranspose2d.reset_parameters:
    kaiming_uniform_(a=sqrt(5)) on the weight, then U(-1/sqrt(fan_in), 1/sqrt(fan_in)) bias."""
    P = OrderedDict()
    for name, kind, shape in layout:
        w = torch.empty(shape)
        torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        fan_in, _ = torch.nn.init._calculate_fan_in_and_fan_out(w)
        bound = 1 / math.sqrt(fan_in) if fan_in > 0 else 0
        out_ch = shape[1] if kind == "convT" else shape[0]
        b = torch.empty(out_ch).uniform_(-bound, bound)
        P[name + ".weight"], P[name + ".bias"] = w, b
    return P


def _initialise(P, layout):
    """models/model.py:162-173: every Conv* gets weight ~ N(0, 0.02), bias = 0, in module
    post-order (= registration order of the convs)."""
    for name, _, _ in layout:
        torch.nn.init.normal_(P[name + ".weight"], 0.0, 0.02)
        torch.nn.init.constant_(P[name + ".bias"], 0.0)
    return P


def init_params(seed=47, c_in=9):
    """models/model.py:80-104: manual_seed(seed); G built + initialised, then D."""
    torch.manual_seed(seed)
    gl, dl = generator_layout(c_in), discriminator_layout(c_in)
    G = _initialise(_construct(gl), gl)
    D = _initialise(_construct(dl), dl)
    return G, D


# ---------------------------------------------------------------------------------------
# forward passes
# ---------------------------------------------------------------------------------------


def _in(x):
    return F.instance_norm(x, eps=EPS_IN)


class ActDecisions:
    """Teacher-forced activation decisions (tests only).  A ReLU / LeakyReLU whose input sits within
    rounding of 0 can be decided differently by any two fp32 evaluations, and one such flip moves
    the gradients of a whole network by ~1/sqrt(pixels x channels) of their norm.
    To compare gradients at full size, the oracle can take the implementation's decisions:
    `masks` = {network: [ {layer: bool tensor NCHW}, ... one per call of that network in call
    order ]}.  Each forced layer logs (network, layer, disagreements, max |pre-activation| / rms
    of the layer over the disagreements): the caller asserts that every disagreement is at the kink."""

    def __init__(self, masks):
        self.queues = {k: list(v) for k, v in masks.items()}
        self.log = []

    def take(self, net):
        q = self.queues.get(net)
        return (q.pop(0), net) if q else None

    def worst(self):
        """largest normalized |pre-activation| at which a decision differed (0 if none)"""
        return max([w for _, _, n, w in self.log if n] or [0.0])


def _act(h, slope, name, forced):
    """ReLU (slope 0) / LeakyReLU(slope), or the teacher-forced decision of `forced` = (masks, net, log)"""
    if forced is None or name not in forced[0]:
        return F.relu(h) if slope == 0 else F.leaky_relu(h, slope)
    masks, net, log = forced
    # contiguous NCHW: a channels-last-strided mask makes torch.where's output channels-last, and
    # that memory format propagating through the fp64 CPU graph changed its backward (forward
    # bit-identical, weight gradients off by O(1): tests/test_oracle_decisions_cpu.py guards this)
    m = masks[name].to(h.device).contiguous()
    hd = h.detach()
    dis = (hd > 0) != m
    n = int(dis.sum())
    rms = float(hd.pow(2).mean().sqrt()) or 1.0
    log.append((net, name, n, float(hd[dis].abs().max()) / rms if n else 0.0))
    return torch.where(m, h, h * slope)


def _l1(fake, y, decisions):
    """F.l1_loss(fake, y) (models/model.py:643); with decisions holding an "L1" entry (tests only) each element's
    gradient sign is the implementation's, sign(fake - y) in {-1, 0, +1} (0 where its fp32 fake equals y exactly, as
    torch's own l1 backward gives): an element within rounding of fake == y can be decided differently by two
    evaluations, and one flip moves the G output gradient by ~2 / sqrt(elements) of its norm.  Disagreements are
    logged like the activation kinks (|fake - y| / rms)."""
    t = decisions.take("L1") if decisions is not None else None
    if t is None:
        return F.l1_loss(fake, y)
    (masks, net), d = t, fake - y
    s = masks["l1"].to(d.device, d.dtype).contiguous()
    dd = d.detach()
    dis = torch.sign(dd) != s
    n = int(dis.sum())
    rms = float(dd.pow(2).mean().sqrt()) or 1.0
    decisions.log.append((net, "l1", n, float(dd[dis].abs().max()) / rms if n else 0.0))
    return (s * d).mean()


def _forced(decisions, net):
    """(masks, net, log) for the next call of `net`, or None"""
    if decisions is None:
        return None
    t = decisions.take(net)
    return None if t is None else (t[0], t[1], decisions.log)


def _conv(P, name, x, stride=1, padding=0):
    return F.conv2d(x, P[name + ".weight"], P[name + ".bias"], stride=stride, padding=padding)


def _convT(P, name, x):
    # nn.ConvTranspose2d(k=3, stride=2, padding=1, output_padding=1)  (:324-333)
    return F.conv_transpose2d(x, P[name + ".weight"], P[name + ".bias"], stride=2, padding=1,
                              output_padding=1)


def resnet_block(P, i, x, forced=None):
    """models/model_architectures.py:412-418."""
    pre = f"resnet_blocks.{i}."
    h = _act(_in(_conv(P, pre + "conv1", F.pad(x, (1, 1, 1, 1), mode="reflect"))), 0, f"block{i}", forced)
    h = _in(_conv(P, pre + "conv2", F.pad(h, (1, 1, 1, 1), mode="reflect")))
    return x + h


def generator_forward(P, x, forced=None):
    """models/model_architectures.py:339-400. Returns (output [N,3,H,W], mask [N,H,W]).
    forced: teacher-forced ReLU decisions (ActDecisions / _forced), tests only."""
    h = _act(_in(_conv(P, "conv1", F.pad(x, (3, 3, 3, 3), mode="reflect"))), 0, "conv1", forced)
    h = _act(_in(_conv(P, "conv2", h, stride=2, padding=1)), 0, "conv2", forced)
    h = _act(_in(_conv(P, "conv3", h, stride=2, padding=1)), 0, "conv3", forced)
    for i in range(9):
        h = resnet_block(P, i, h, forced)
    c = _act(_in(_convT(P, "deconv1_content", h)), 0, "deconv1_content", forced)
    c = _act(_in(_convT(P, "deconv2_content", c)), 0, "deconv2_content", forced)
    content = torch.tanh(_conv(P, "deconv3_content", F.pad(c, (3, 3, 3, 3), mode="reflect")))
    a = _act(_in(_convT(P, "deconv1_attention", h)), 0, "deconv1_attention", forced)
    a = _act(_in(_convT(P, "deconv2_attention", a)), 0, "deconv2_attention", forced)
    att = torch.softmax(_conv(P, "deconv3_attention", a), dim=1)
    # composite: sum_{i<9} content[3i:3i+3] * att[i]  +  input[:, :3] * att[9]   (:371-399)
    # (summed left to right in the reference's order: output1 + ... + output9 + output10)
    out = content[:, 0:3] * att[:, 0:1]
    for i in range(1, 9):
        out = out + content[:, 3 * i:3 * i + 3] * att[:, i:i + 1]
    out = out + x[:, :3] * att[:, 9:10]
    return out, att[:, 9]


def discriminator_forward(P, x, forced=None):
    """models/model_architectures.py:424-441 (LeakyReLU 0.2 after every conv but the last)."""
    h = _act(_conv(P, "model.0", x, 2, 1), 0.2, "model.0", forced)
    h = _act(_in(_conv(P, "model.2", h, 2, 1)), 0.2, "model.2", forced)
    h = _act(_in(_conv(P, "model.5", h, 2, 1)), 0.2, "model.5", forced)
    h = _act(_in(_conv(P, "model.8", h, 1, 1)), 0.2, "model.8", forced)
    return _conv(P, "model.11", h, 1, 1)


# ---------------------------------------------------------------------------------------
# optimiser + training step
# ---------------------------------------------------------------------------------------


def lambda_rule(epoch, num_epochs):
    """models/model.py:175-181."""
    return 1.0 - max(0, epoch + 1 - (num_epochs / 2)) / float((num_epochs / 2) + 1)


class PairedStepOracle:
    """Holds G/D params + torch.optim.Adam states and performs reference training steps
    (models/model.py:611-651) with autograd on the CPU."""

    def __init__(self, G=None, D=None, seed=47, c_in=9, lr=2e-4, dtype=torch.float32):
        if G is None:
            G, D = init_params(seed, c_in)
        self.G = OrderedDict((k, v.detach().clone().to(dtype).requires_grad_(True)) for k, v in G.items())
        self.D = OrderedDict((k, v.detach().clone().to(dtype).requires_grad_(True)) for k, v in D.items())
        self.opt_g = torch.optim.Adam(list(self.G.values()), lr=lr, betas=(0.5, 0.999))
        self.opt_d = torch.optim.Adam(list(self.D.values()), lr=lr, betas=(0.5, 0.999))
        self.dtype = dtype

    def set_lr(self, lr):
        for opt in (self.opt_g, self.opt_d):
            for g in opt.param_groups:
                g["lr"] = lr

    def load_state(self, G, D, opt_g_state=None, opt_d_state=None):
        """Teacher forcing: continue from another implementation's state -- parameters (name ->
        tensor) and torch.optim.Adam-format optimiser state dicts (FusedAdam writes that format)."""
        with torch.no_grad():
            for P, src in ((self.G, G), (self.D, D)):
                for k, v in P.items():
                    v.copy_(src[k].detach().to(v.device, v.dtype))
        # deep copies: a state_dict holds the optimiser's LIVE tensors (its CPU 'step' counter is
        # shared and would keep counting with the implementation's own steps)
        if opt_g_state is not None:
            self.opt_g.load_state_dict(copy.deepcopy(opt_g_state))
        if opt_d_state is not None:
            self.opt_d.load_state_dict(copy.deepcopy(opt_d_state))

    def step(self, x, y, record=None, d_after=None, decisions=None):
        """One iteration of models/model.py:615-646. Returns the four losses (D real,
        D synthetic, G synthetic, raw L1 before x100) as floats.
        d_after (teacher forcing, tests only): discriminator parameters to continue the G step
        with instead of this oracle's own Adam(D) result, so that the G half is compared on the
        same D as the implementation under test.
        decisions (tests only): ActDecisions with networks "G" (one call) and "D" (three calls:
        synthetic and real of the D step, synthetic of the G step)."""
        x, y = x.to(self.dtype), y.to(self.dtype)
        fake, mask = generator_forward(self.G, x, _forced(decisions, "G"))
        cat_real = torch.cat((x, y), 1)
        cat_fake = torch.cat((x, fake), 1)
        for p in self.D.values():
            p.requires_grad_(True)
        self.opt_d.zero_grad()
        pred_fake = discriminator_forward(self.D, cat_fake.detach(), _forced(decisions, "D"))
        l_d_fake = F.mse_loss(pred_fake, torch.zeros_like(pred_fake))
        pred_real = discriminator_forward(self.D, cat_real, _forced(decisions, "D"))
        l_d_real = F.mse_loss(pred_real, torch.ones_like(pred_real))
        l_d = (l_d_fake + l_d_real) * 0.5
        l_d.backward()
        if record is not None:
            record["d_grads"] = OrderedDict((k, v.grad.detach().clone()) for k, v in self.D.items())
            # dl_d/d(model.11.bias) = mean(pred_fake) + mean(pred_real - 1): a sum whose terms can cancel, so its
            # attainable relative accuracy is u * (mean|pred_fake| + mean|pred_real - 1|) / |sum| (checked against
            # that mass, tests/test_gpu_northstar.py u_compare)
            record["d_sum_mass"] = {"model.11.bias": float(pred_fake.detach().abs().mean() +
                                                          (pred_real.detach() - 1).abs().mean())}
        self.opt_d.step()
        if record is not None:
            record["d_after_own"] = OrderedDict((k, v.detach().clone()) for k, v in self.D.items())
        if d_after is not None:
            with torch.no_grad():
                for k, v in self.D.items():
                    v.copy_(d_after[k].detach().to(v.device, v.dtype))
        for p in self.D.values():
            p.requires_grad_(False)
        self.opt_g.zero_grad()
        pred = discriminator_forward(self.D, cat_fake, _forced(decisions, "D"))
        l_g = F.mse_loss(pred, torch.ones_like(pred))
        l1 = _l1(fake, y, decisions)
        (l_g + l1 * 100).backward()
        if record is not None:
            record["g_grads"] = OrderedDict((k, v.grad.detach().clone()) for k, v in self.G.items())
            record["fake"] = fake.detach().clone()
            record["mask"] = mask.detach().clone()
        self.opt_g.step()
        for p in self.D.values():
            p.requires_grad_(True)
        return [float(v.detach()) for v in (l_d_real, l_d_fake, l_g, l1)]


# Conv biases whose output feeds an InstanceNorm are mathematically cancelled; their
# gradients are floating-point noise and Adam turns that into +-lr steps.
# Parity comparisons of post-step parameters exclude them.
def cancelled_biases():
    g = ["conv1", "conv2", "conv3"] + [f"resnet_blocks.{i}.conv{j}" for i in range(9) for j in (1, 2)]
    g += ["deconv1_content", "deconv2_content", "deconv1_attention", "deconv2_attention"]
    d = ["model.2", "model.5", "model.8"]
    return {n + ".bias" for n in g}, {n + ".bias" for n in d}
