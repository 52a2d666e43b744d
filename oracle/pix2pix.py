"""CPU ORACLE for the Pix2Pix paired-GAN training step -- TEST INFRASTRUCTURE ONLY (only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import it).

Functional restatement on PyTorch-CPU of:

  generator     models/model_architectures.py:9-62  (Pix2PixGenerator: U-Net-256, 8 Pix2PixBlocks)
  discriminator models/model_architectures.py:64-85 (PatchGAN over input_channels + 3, BatchNorm)
  init          models/model.py:80 (seed), :102-104 (construct + .apply(initialise_weights)), :162-173
                (Conv*: N(0, 0.02), bias 0; BatchNorm2d: weight N(1, 0.02), bias 0)
  train step    models/model.py:611-651 (the same train_paired iteration as PairedAttention)

What the restatement has to reproduce exactly:
  * the RNG order of construction (innermost block first: downconv, then upconv, per block) and of
    initialise_weights (module post-order: outermost downconv, each level's downconv + downnorm on the
    way in, the innermost up path, then each level's upconv + upnorm on the way out);
  * Pix2PixBlock.forward = torch.cat([x, model(x)], 1) where model(x) begins with an IN-PLACE
    LeakyReLU on x: the skip carries LeakyReLU(x), and the parent's in-place ReLU makes the up path
    see cat[ReLU(x), ReLU(up)] (:31-62);
  * nn.BatchNorm2d in training mode (batch statistics, running statistics updated with momentum 0.1
    and the unbiased variance) -- the discriminator's D(fake) and D(real) of the D step are separate
    calls (models/model.py:624-628), so separate statistics and two running-stat updates;
  * nn.Dropout(0.5) in the three 512-channel blocks next to the innermost one: on the CPU,
    F.dropout draws torch.empty_like(x).bernoulli_(0.5) from the global generator, innermost level
    first (the order their up paths finish), and multiplies by mask / 0.5.

Parameters / buffers are plain ordered dicts keyed exactly like the reference modules' state_dict.
Parity pin: tests/test_oracle_pix2pix_golden.py vs tests/golden/pix2pix_step_256.npz, produced by
tests/golden/make_golden_pix2pix.py from the reference's unmodified train_paired().
"""
import copy
import math
from collections import OrderedDict

import torch
import torch.nn.functional as F

from .paired_attention import _act, _forced, _l1

BN_EPS, BN_MOMENTUM = 1e-5, 0.1
N_LEVELS = 8


def level_channels(c_in=9):
    """(input_nc, inner_nc, outer_nc) of levels 1 (outermost) .. 8 (innermost), models/model_architectures.py:13-19"""
    return [(c_in, 64, 3), (64, 128, 64), (128, 256, 128), (256, 512, 256), (512, 512, 512), (512, 512, 512),
            (512, 512, 512), (512, 512, 512)]


def level_prefix(k):
    """state_dict prefix of level k's Sequential: Pix2PixGenerator.model (level 1) .model, then the
    submodule sits at index 1 of the outermost Sequential and at index 3 of the middle ones"""
    return "model.model." + "1.model." * (k > 1) + "3.model." * max(0, k - 2)


def dropout_levels():
    return (5, 6, 7)


def generator_layout(c_in=9):
    """[(state_dict name, kind, shape)] per module: 'conv' / 'convT' (+ '_bias'), 'bn'"""
    ch = level_channels(c_in)
    out = {}
    for k in range(1, N_LEVELS + 1):
        i, inner, outer = ch[k - 1]
        p = level_prefix(k)
        if k == 1:
            out[k] = dict(down=(p + "0", (inner, i, 4, 4)), up=(p + "3", (inner * 2, outer, 4, 4)), up_bias=True)
        elif k == N_LEVELS:
            out[k] = dict(down=(p + "1", (inner, i, 4, 4)), up=(p + "3", (inner, outer, 4, 4)), upnorm=(p + "4", outer))
        else:
            out[k] = dict(down=(p + "1", (inner, i, 4, 4)), downnorm=(p + "2", inner),
                          up=(p + "5", (inner * 2, outer, 4, 4)), upnorm=(p + "6", outer))
    return out


def discriminator_layout(c_in=9):
    return [("model.0", "conv", (64, c_in + 3, 4, 4), True), ("model.2", "conv", (128, 64, 4, 4), False),
            ("model.3", "bn", 128), ("model.5", "conv", (256, 128, 4, 4), False), ("model.6", "bn", 256),
            ("model.8", "conv", (512, 256, 4, 4), False), ("model.9", "bn", 512),
            ("model.11", "conv", (1, 512, 4, 4), True)]


def _kaiming(shape):
    w = torch.empty(shape)
    torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
    return w


def _bias_for(w, n):
    fan_in, _ = torch.nn.init._calculate_fan_in_and_fan_out(w)
    bound = 1 / math.sqrt(fan_in) if fan_in > 0 else 0
    return torch.empty(n).uniform_(-bound, bound)


def _bn(P, B, name, n):
    P[name + ".weight"], P[name + ".bias"] = torch.ones(n), torch.zeros(n)
    B[name + ".running_mean"], B[name + ".running_var"] = torch.zeros(n), torch.ones(n)
    B[name + ".num_batches_tracked"] = torch.tensor(0, dtype=torch.long)


def init_generator(c_in=9):
    """Construction (RNG: innermost block first; in each block downconv, then upconv) and
    initialise_weights in module post-order.  Returns (params, buffers) in state_dict order."""
    lay = generator_layout(c_in)
    made = {}
    for k in range(N_LEVELS, 0, -1):                    # constructor: innermost first (:13-19)
        L = lay[k]
        made[L["down"][0] + ".weight"] = _kaiming(L["down"][1])
        w = _kaiming(L["up"][1])
        made[L["up"][0] + ".weight"] = w
        if L.get("up_bias"):
            made[L["up"][0] + ".bias"] = _bias_for(w, L["up"][1][1])
    P, B = OrderedDict(), OrderedDict()
    # state_dict / post-order traversal: level 1 down, level 2 (down, downnorm), ..., level 8 (down,
    # up, upnorm), ..., level 2 (up, upnorm), level 1 up
    order = [("down", 1)] + [(t, k) for k in range(2, N_LEVELS) for t in ("down", "downnorm")] + \
            [("down", N_LEVELS), ("up", N_LEVELS), ("upnorm", N_LEVELS)] + \
            [(t, k) for k in range(N_LEVELS - 1, 1, -1) for t in ("up", "upnorm")] + [("up", 1)]
    for t, k in order:
        L = lay[k]
        if t in ("down", "up"):
            name = L[t][0]
            P[name + ".weight"] = torch.nn.init.normal_(made[name + ".weight"], 0.0, 0.02)
            if name + ".bias" in made:
                P[name + ".bias"] = torch.nn.init.constant_(made[name + ".bias"], 0.0)
        else:
            name, n = L[t]
            _bn(P, B, name, n)
            torch.nn.init.normal_(P[name + ".weight"], 1.0, 0.02)
    return P, B


def init_discriminator(c_in=9):
    lay = discriminator_layout(c_in)
    P, B = OrderedDict(), OrderedDict()
    for entry in lay:                                   # construction RNG in Sequential order
        if entry[1] == "conv":
            name, _, shape, bias = entry
            P[name + ".weight"] = _kaiming(shape)
            if bias:
                P[name + ".bias"] = _bias_for(P[name + ".weight"], shape[0])
        else:
            _bn(P, B, entry[0], entry[2])
    for entry in lay:                                   # initialise_weights, same (post-)order
        name = entry[0]
        if entry[1] == "conv":
            torch.nn.init.normal_(P[name + ".weight"], 0.0, 0.02)
            if name + ".bias" in P:
                torch.nn.init.constant_(P[name + ".bias"], 0.0)
        else:
            torch.nn.init.normal_(P[name + ".weight"], 1.0, 0.02)
    return P, B


def init_params(seed=47, c_in=9):
    """models/model.py:80-104: manual_seed(seed); generator built + initialised, then the discriminator."""
    torch.manual_seed(seed)
    G = init_generator(c_in)
    D = init_discriminator(c_in)
    return G, D


# ------------------------------------------------------------------------------------------ forward

def _batchnorm(P, B, name, x):
    """nn.BatchNorm2d(train): batch statistics, running statistics updated in place"""
    return F.batch_norm(x, B[name + ".running_mean"], B[name + ".running_var"], P[name + ".weight"],
                        P[name + ".bias"], training=True, momentum=BN_MOMENTUM, eps=BN_EPS)


def _bn_call(P, B, name, x, training=True):
    if not training:     # module.eval(): running statistics, nothing updated
        return F.batch_norm(x, B[name + ".running_mean"], B[name + ".running_var"], P[name + ".weight"],
                            P[name + ".bias"], training=False, eps=BN_EPS)
    B[name + ".num_batches_tracked"] += 1
    return _batchnorm(P, B, name, x)


def _dropout_mask(shape):
    """F.dropout(x, 0.5, training=True) on the CPU: empty_like(x).bernoulli_(1 - p), then / (1 - p)"""
    return torch.empty(shape, dtype=torch.float32).bernoulli_(0.5)


def generator_forward(P, B, x, forced=None, masks=None, training=True):
    """models/model_architectures.py:21-62.  masks: {level: dropout mask} to use instead of drawing
    (drawn masks are recorded into it when a dict is given empty); training=False: eval mode (running
    statistics, no dropout)."""
    lay = generator_layout(x.shape[1])

    def level(k, h):
        L = lay[k]
        a = h if k == 1 else _act(h, 0.2, f"down{k - 1}", forced)      # in-place LeakyReLU of the input
        d = F.conv2d(a, P[L["down"][0] + ".weight"], None, stride=2, padding=1)
        if "downnorm" in L:
            d = _bn_call(P, B, L["downnorm"][0], d, training)
        if k == N_LEVELS:
            r = _act(d, 0.0, "inner", forced)
        else:
            u_sub = level(k + 1, d)                                     # the submodule's up output
            r = torch.cat((_act(d, 0.0, f"down{k}", forced), _act(u_sub, 0.0, f"up{k + 1}", forced)), 1)
        w = P[L["up"][0] + ".weight"]
        u = F.conv_transpose2d(r, w, P.get(L["up"][0] + ".bias"), stride=2, padding=1)
        if k == 1:
            return torch.tanh(u)
        u = _bn_call(P, B, L["upnorm"][0], u, training)
        if training and k in dropout_levels():
            if masks is not None and k in masks:
                m = masks[k]
            else:
                m = _dropout_mask(u.shape)
                if masks is not None:
                    masks[k] = m
            u = u * (m.to(u.dtype) / 0.5)
        return u
    return level(1, x)


def discriminator_forward(P, B, x, forced=None):
    """models/model_architectures.py:84-85 (training mode)"""
    h = _act(F.conv2d(x, P["model.0.weight"], P["model.0.bias"], stride=2, padding=1), 0.2, "model.0", forced)
    h = _act(_bn_call(P, B, "model.3", F.conv2d(h, P["model.2.weight"], None, stride=2, padding=1)), 0.2, "model.2",
             forced)
    h = _act(_bn_call(P, B, "model.6", F.conv2d(h, P["model.5.weight"], None, stride=2, padding=1)), 0.2, "model.5",
             forced)
    h = _act(_bn_call(P, B, "model.9", F.conv2d(h, P["model.8.weight"], None, stride=1, padding=1)), 0.2, "model.8",
             forced)
    return F.conv2d(h, P["model.11.weight"], P["model.11.bias"], stride=1, padding=1)


class Pix2PixStepOracle:
    """Holds G/D params + buffers + torch.optim.Adam and performs reference training steps
    (models/model.py:611-651) with autograd on the CPU."""

    def __init__(self, G=None, D=None, seed=47, c_in=9, lr=2e-4, dtype=torch.float32):
        if G is None:
            G, D = init_params(seed, c_in)
        (gp, gb), (dp, db) = G, D
        self.G = OrderedDict((k, v.detach().clone().to(dtype).requires_grad_(True)) for k, v in gp.items())
        self.D = OrderedDict((k, v.detach().clone().to(dtype).requires_grad_(True)) for k, v in dp.items())
        self.GB = OrderedDict((k, v.clone().to(dtype) if v.is_floating_point() else v.clone()) for k, v in gb.items())
        self.DB = OrderedDict((k, v.clone().to(dtype) if v.is_floating_point() else v.clone()) for k, v in db.items())
        self.opt_g = torch.optim.Adam(list(self.G.values()), lr=lr, betas=(0.5, 0.999))
        self.opt_d = torch.optim.Adam(list(self.D.values()), lr=lr, betas=(0.5, 0.999))
        self.dtype = dtype

    def load_state(self, G, GB, D, DB, opt_g_state=None, opt_d_state=None):
        """continue from another implementation's state (parameters, BatchNorm buffers, Adam states as
        state_dict()s, deep-copied: a live optimizer's step tensors must not alias ours)"""
        for mine, theirs in ((self.G, G), (self.D, D)):
            with torch.no_grad():
                for k, v in theirs.items():
                    mine[k].copy_(v.detach().cpu().to(self.dtype))
        for mine, theirs in ((self.GB, GB), (self.DB, DB)):
            for k, v in theirs.items():
                mine[k] = v.detach().cpu().clone().to(self.dtype if v.is_floating_point() else v.dtype)
        for opt, st in ((self.opt_g, opt_g_state), (self.opt_d, opt_d_state)):
            if st is not None:     # Adam.load_state_dict casts the moments to the parameters' dtype / device
                opt.load_state_dict(copy.deepcopy(st))

    def set_lr(self, lr):
        for opt in (self.opt_g, self.opt_d):
            for g in opt.param_groups:
                g["lr"] = lr

    def step(self, x, y, record=None, masks=None, decisions=None, d_after=None):
        """One iteration of models/model.py:615-646; returns (D real, D synthetic, G synthetic, raw L1).
        masks: dropout masks by level (drawn from the global generator when absent, recorded when given
        empty); decisions (tests only): ActDecisions for "G" (one call) and "D" (fake, real, G step);
        d_after (tests only): discriminator parameters to continue the G half with instead of this
        oracle's own Adam(D) result (recorded as record["d_after_own"])."""
        x, y = x.to(self.dtype), y.to(self.dtype)
        fake = generator_forward(self.G, self.GB, x, _forced(decisions, "G"), masks)
        cat_real, cat_fake = torch.cat((x, y), 1), torch.cat((x, fake), 1)
        for p in self.D.values():
            p.requires_grad_(True)
        self.opt_d.zero_grad()
        pf = discriminator_forward(self.D, self.DB, cat_fake.detach(), _forced(decisions, "D"))
        l_d_fake = F.mse_loss(pf, torch.zeros_like(pf))
        pr = discriminator_forward(self.D, self.DB, cat_real, _forced(decisions, "D"))
        l_d_real = F.mse_loss(pr, torch.ones_like(pr))
        ((l_d_fake + l_d_real) * 0.5).backward()
        if record is not None:
            record["d_grads"] = OrderedDict((k, v.grad.detach().clone()) for k, v in self.D.items())
        self.opt_d.step()
        if record is not None:
            record["d_after_own"] = OrderedDict((k, v.detach().clone()) for k, v in self.D.items())
        if d_after is not None:
            with torch.no_grad():
                for k, v in d_after.items():
                    self.D[k].copy_(v.to(self.dtype))
        for p in self.D.values():
            p.requires_grad_(False)
        self.opt_g.zero_grad()
        pg = discriminator_forward(self.D, self.DB, cat_fake, _forced(decisions, "D"))
        l_g = F.mse_loss(pg, torch.ones_like(pg))
        l1 = _l1(fake, y, decisions)        # the implementation's L1 sign decisions when given (tests)
        (l_g + l1 * 100).backward()
        if record is not None:
            record["g_grads"] = OrderedDict((k, v.grad.detach().clone()) for k, v in self.G.items())
            record["fake"] = fake.detach().clone()
        self.opt_g.step()
        for p in self.D.values():
            p.requires_grad_(True)
        return [float(v.detach()) for v in (l_d_real, l_d_fake, l_g, l1)]
