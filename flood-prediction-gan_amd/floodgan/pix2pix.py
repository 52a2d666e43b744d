"""Native forward / backward executors of the Pix2Pix U-Net-256 generator and its BatchNorm PatchGAN
discriminator, and the fused Pix2Pix training iteration.

Reference: models/model_architectures.py:9-62 (Pix2PixGenerator / Pix2PixBlock), :64-85
(Pix2PixDiscriminator), models/model.py:611-651 (train_paired, shared with PairedAttention).

Layout.  Level k = 1 (outermost) .. 8 (innermost) of the U-Net; at input H x W level k's down conv
(4x4, stride 2, no bias) produces D_k at H/2^k.  Every activation lives in an NHWC Buf whose zero
border is the next conv's padding:
  a_{k+1} = LeakyReLU(D_k)      -- level k+1's down-conv input (the in-place LeakyReLU of
                                   Pix2PixBlock.forward's x, :58-62, so the skip carries it too)
  cat_k   = [ReLU(D_k) | ReLU(U_{k+1})]  -- level k's up-conv input: torch.cat([x, model(x)], 1)
                                   followed by the parent's in-place ReLU, as two channel slices of
                                   one buffer, each written by the BatchNorm pass that produces it
  r_8     = ReLU(D_8)           -- the innermost up-conv input
The up convs (ConvTranspose2d 4x4 s2 p1) run as four sub-pixel phase GEMMs; the outermost one adds
its bias and feeds the tanh head.  BatchNorm (training mode: batch statistics, running statistics
updated in place on the module buffers; eval mode: running statistics) is one statistics pass and
one apply pass that also writes the activated copies.  Dropout(0.5) of levels 5-7 is fused into the
BatchNorm apply / backward passes, its keep decisions either
  "device":  a counter-based hash of (seed, element) evaluated in the apply pass and
             recomputed in the backward -- no mask is drawn, stored or copied; one 62-bit seed per
             generator call comes from torch's CPU generator, so torch.manual_seed fixes the masks; or
  "host" (default since round 5): the 0/1 masks torch's CPU generator gives the reference's CPU path (F.dropout:
             empty_like(x).bernoulli_(0.5), innermost level first: 7, 6, 5), bit for bit -- a seeded run then
             reproduces the reference's CPU run (the parity mode).  Round 5: the masks are no longer drawn on
             the host; the device regenerates torch's MT19937 stream from the generator's state with chunked
             jump-ahead (floodgan.torch_rng, csrc/mt19937.hip) and hands the advanced state back to torch.

The discriminator's D(fake) and D(real) of the D step are separate BatchNorm calls in the
reference (:624-628): one 2N-image pass with groups=2 (statistics per half, the running statistics
updated twice, in order).
"""
import torch

from . import executor as X
from . import ops
from . import plans as PL
from . import torch_rng
from ._lib import FG_ACT_LRELU, FG_ACT_NONE, FG_ACT_RELU, FG_PAD_ZERO, require_device
from .plans import Buf, Slice

N_LEVELS = 8
DROPOUT_LEVELS = (7, 6, 5)          # draw order (innermost first)
DROP_P = 0.5


def level_channels(c_in):
    """(input_nc, inner_nc, outer_nc) of levels 1..8 (models/model_architectures.py:13-19)"""
    return [(c_in, 64, 3), (64, 128, 64), (128, 256, 128), (256, 512, 256)] + [(512, 512, 512)] * 4


def level_prefix(k):
    """state_dict prefix of level k's nn.Sequential: the outermost block is Pix2PixGenerator.model;
    a submodule sits at index 1 of the outermost Sequential and at index 3 of the middle ones"""
    return "model.model." + "1.model." * (k > 1) + "3.model." * max(0, k - 2)


def level_names(k):
    """{'down', 'downnorm', 'up', 'upnorm'} module names of level k (absent where the reference has none)"""
    p = level_prefix(k)
    if k == 1:
        return dict(down=p + "0", up=p + "3")
    if k == N_LEVELS:
        return dict(down=p + "1", up=p + "3", upnorm=p + "4")
    return dict(down=p + "1", downnorm=p + "2", up=p + "5", upnorm=p + "6")


def gen_state_keys():
    """parameter names in registration order (= state_dict / .parameters() order)"""
    keys = [level_names(1)["down"] + ".weight"]
    for k in range(2, N_LEVELS):
        n = level_names(k)
        keys += [n["down"] + ".weight", n["downnorm"] + ".weight", n["downnorm"] + ".bias"]
    n = level_names(N_LEVELS)
    keys += [n["down"] + ".weight", n["up"] + ".weight", n["upnorm"] + ".weight", n["upnorm"] + ".bias"]
    for k in range(N_LEVELS - 1, 1, -1):
        n = level_names(k)
        keys += [n["up"] + ".weight", n["upnorm"] + ".weight", n["upnorm"] + ".bias"]
    n = level_names(1)
    keys += [n["up"] + ".weight", n["up"] + ".bias"]
    return keys


def gen_bucket_names():
    """the generator's gradient buckets in the order gen_backward completes them (parallel.FlatGrads)"""
    n1 = level_names(1)
    out = [[n1["up"] + ".weight", n1["up"] + ".bias"]]
    for k in range(2, N_LEVELS + 1):
        n = level_names(k)
        out.append([n["upnorm"] + ".weight", n["upnorm"] + ".bias", n["up"] + ".weight"])
    out.append([level_names(N_LEVELS)["down"] + ".weight"])
    for k in range(N_LEVELS - 1, 1, -1):
        n = level_names(k)
        out.append([n["downnorm"] + ".weight", n["downnorm"] + ".bias", n["down"] + ".weight"])
    out.append([n1["down"] + ".weight"])
    return out


DISC_CONVS = ["model.0", "model.2", "model.5", "model.8", "model.11"]
DISC_NORMS = {"model.2": "model.3", "model.5": "model.6", "model.8": "model.9"}
DISC_KEYS = ["model.0.weight", "model.0.bias", "model.2.weight", "model.3.weight", "model.3.bias", "model.5.weight",
             "model.6.weight", "model.6.bias", "model.8.weight", "model.9.weight", "model.9.bias", "model.11.weight",
             "model.11.bias"]


def disc_bucket_names():
    return [["model.11.weight", "model.11.bias"], ["model.9.weight", "model.9.bias", "model.8.weight"],
            ["model.6.weight", "model.6.bias", "model.5.weight"], ["model.3.weight", "model.3.bias", "model.2.weight"],
            ["model.0.weight", "model.0.bias"]]


def _mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def dropout_shapes(n, h, w):
    """{level: NCHW shape of the tensor its Dropout applies to} at input h x w"""
    return {k: (n, 512, h >> (k - 1), w >> (k - 1)) for k in DROPOUT_LEVELS}


def draw_dropout(n, h, w, mode="host", device="cuda"):
    """One generator call's Dropout decisions: {level: device 0/1 mask} ("host": torch's CPU stream, regenerated
    on the device; the generator advanced before returning) or {level: seed} ("device")"""
    if mode == "host":
        masks, commit = draw_dropout_deferred(n, h, w, device)
        commit()
        return masks
    if mode != "device":
        raise ValueError(f"dropout mode must be 'device' or 'host' (got {mode!r})")
    base = int(torch.randint(1, 2 ** 62, (1,)).item())
    return {k: (_mix64(base + k) & 0x7FFFFFFFFFFFFFFF) or 1 for k in DROPOUT_LEVELS}


def dropout_masks(drop, n, h, w, device="cuda"):
    """{level: 0/1 mask} of a draw_dropout result (seeds materialised on the device; tests / inspection)"""
    out = {}
    for k, shape in dropout_shapes(n, h, w).items():
        d = drop[k]
        out[k] = ops.dropout_mask(d, shape, device) if isinstance(d, int) else d
    return out


def draw_dropout_deferred(n, h, w, device="cuda"):
    """"host" mode's masks as ({level: device 0/1 mask}, commit): commit() advances torch's CPU generator past
    the draw (the fused step calls it at its end: nothing else in the iteration draws from that generator)"""
    shapes = dropout_shapes(n, h, w)
    outs, commit = torch_rng.draw(list(shapes.values()), 1 - DROP_P, device)
    return dict(zip(shapes, outs)), commit


def draw_dropout_masks(n, h, w):
    """The Dropout masks of one generator call at input h x w, from torch's (CPU) global generator in
    the reference's CPU order: F.dropout draws empty_like(x).bernoulli_(1 - p) per call, levels 7, 6, 5.
    Returns {level: float32 0/1 mask [n, 512, h_k, w_k]} on the host."""
    masks = {}
    for k, shape in dropout_shapes(n, h, w).items():      # level k's up output = its input size
        masks[k] = torch.empty(shape, dtype=torch.float32).bernoulli_(1 - DROP_P)
    return masks


# ======================================================================================
# generator
# ======================================================================================

def _conv_nb(P, name, X_, pad, k, stride, Y, act=FG_ACT_NONE, tag=None):
    """conv whose module may have no bias (bias=False in the reference)"""
    w = P[name + ".weight"]
    m = PL.wmap_conv_fwd(w.shape, X_.c)
    ops.conv([PL.conv_problem(X_, pad, k, stride, ops.pack_weight(w, m), m, Y, bias=P.get(name + ".bias"), act=act)],
             tag=tag)


def _convT4(P, name, X_, Y):
    """ConvTranspose2d(k=4, s=2, p=1) over X_ (zero border >= 1): four phase GEMMs"""
    w = P[name + ".weight"]
    maps = PL.phase_maps(w.shape, 4, 1, X_.c)
    wps = [ops.pack_weight(w, m) for m, _, _ in maps]
    ops.conv(PL.phase_problems(X_, w.shape, 4, 1, Y, wps, maps, bias=P.get(name + ".bias")))


def _stats(B, name, src, groups, training):
    """batch statistics (+ running-stat update) or, in eval mode, the running statistics"""
    rm, rv = B[name + ".running_mean"], B[name + ".running_var"]
    if training:
        return ops.bn_stats(src, groups, (rm, rv, B.get(name + ".num_batches_tracked")))
    mean, invstd = ops.bn_eval_stats(rm, rv)
    if groups > 1:
        mean, invstd = mean.repeat(groups), invstd.repeat(groups)
    return mean, invstd


def check_input_size(H, W):
    if H < 256 or W < 256 or H % 256 or W % 256:
        raise RuntimeError(f"Pix2PixGenerator (U-Net-256) needs H, W multiples of 256 (got {H}x{W}): its eight "
                           "stride-2 levels and skip concatenations only line up there")


def gen_forward(P, B, x, masks=None, training=True, save=True):
    """x: [N, C, H, W] fp32 on the device (any strides); P: parameters, B: BatchNorm buffers (updated
    in place in training mode), masks: a draw_dropout result (training mode; drawn here, device mode,
    when None).  Returns (out [N, 3, H, W], saved)."""
    require_device(x, "generator input")
    N, Cin, H, W = x.shape
    check_input_size(H, W)
    dev = x.device
    if training and masks is None:
        masks = draw_dropout(N, H, W, device=x.device)
    dmask = {k: (m if isinstance(m, int) else m.to(dev)) for k, m in masks.items()} if training else {}
    ch = level_channels(Cin)
    S = dict(x=x, N=N, H=H, W=W, training=training, lv={})
    X0 = Buf.empty(N, H, W, PL.rup(Cin, 4), 1, dev)
    ops.pack_input(x, Cin, None, 0, X0, 0, N, FG_PAD_ZERO)
    a = X0                                             # level k's down-conv input
    for k in range(1, N_LEVELS + 1):
        nm = level_names(k)
        inner = ch[k - 1][1]
        h, w = H >> k, W >> k
        c = Buf.empty(N, h, w, inner, 0, dev)
        _conv_nb(P, nm["down"], a, 1, 4, 2, c)
        L = dict(a=a, c=c)
        if k == N_LEVELS:
            r = Buf.zeros(N, h, w, inner, 1, dev)
            ops.bn_apply(c, 1, None, None, None, None, None, FG_ACT_RELU, r)
            L["r"] = r
        else:
            mean = invstd = None
            if "downnorm" in nm:
                mean, invstd = _stats(B, nm["downnorm"], c, 1, training)
            nxt = Buf.zeros(N, h, w, inner, 1, dev)
            cat = Buf.zeros(N, h, w, 2 * inner, 1, dev)
            slot = ops._amax_out(cat)                 # one operand-scale slot, raised by both halves' producers
            gam = P.get(nm.get("downnorm", "") + ".weight")
            bet = P.get(nm.get("downnorm", "") + ".bias")
            ops.bn_apply(c, 1, mean, invstd, gam, bet, None, FG_ACT_LRELU, nxt, FG_ACT_RELU, Slice(cat, 0, inner),
                         slots=(None, slot))
            L.update(mean=mean, invstd=invstd, cat=cat, cat_slot=slot)
            a = nxt
        S["lv"][k] = L
    # up path, innermost first
    for k in range(N_LEVELS, 1, -1):
        nm = level_names(k)
        L = S["lv"][k]
        outer = ch[k - 1][2]
        h, w = H >> (k - 1), W >> (k - 1)
        u = Buf.empty(N, h, w, outer, 0, dev)
        _convT4(P, nm["up"], L["r"] if k == N_LEVELS else L["cat"], u)
        mean, invstd = _stats(B, nm["upnorm"], u, 1, training)
        parent = S["lv"][k - 1]
        inner_p = ch[k - 2][1]
        ops.bn_apply(u, 1, mean, invstd, P[nm["upnorm"] + ".weight"], P[nm["upnorm"] + ".bias"], dmask.get(k),
                     FG_ACT_RELU, Slice(parent["cat"], inner_p, inner_p), slots=(parent["cat_slot"], None))
        L.update(u=u, umean=mean, uinvstd=invstd, mask=dmask.get(k))
    nm = level_names(1)
    logits = Buf.empty(N, H, W, 4, 0, dev)
    _convT4(P, nm["up"], S["lv"][1]["cat"], logits)
    out = torch.empty(N, 3, H, W, dtype=torch.float32, device=dev)
    ops.tanh_head_fwd(logits, 3, out)
    S["logits"] = logits
    return out, (S if save else None)


def gen_backward(P, S, g_out, grads_into=None, ready=None, accumulate=False):
    """Explicit backward of gen_forward (training-mode BatchNorm: through the batch statistics).
    g_out: [N, 3, H, W] (any strides).  Returns {parameter name: gradient}."""
    ready = ready or (lambda name: None)
    N, H, W = S["N"], S["H"], S["W"]
    dev = g_out.device
    G = X._Grads(P, grads_into, accumulate, device=dev)
    ch = level_channels(S["x"].shape[1])
    lv = S["lv"]
    # ---- tanh head + outermost up conv (bias)
    nm = level_names(1)
    g_logits = Buf.empty(N, H, W, 4, 1, dev)
    ops.tanh_head_bwd(S["logits"], 3, g_out, g_logits)
    w = P[nm["up"] + ".weight"]
    G.wgrad(PL.wgrad_convT(lv[1]["cat"], g_logits, 4, 1, w.shape[0]), PL.wmap_wgrad(w.shape, True, g_logits.c, 4),
            nm["up"] + ".weight", (lv[1]["cat"], g_logits))
    ops.channel_sum(g_logits, 3, G.get(nm["up"] + ".bias"), G.acc)
    G.ready(ready, nm["up"])
    g_cat = {}
    g_cat[1] = Buf.empty(N, H >> 1, W >> 1, w.shape[0], 0, dev)
    m = PL.wmap_convT_dgrad(w.shape, g_logits.c)
    ops.conv([PL.conv_problem(g_logits, 1, 4, 2, ops.pack_weight(w, m), m, g_cat[1])])
    # ---- up chain: level k's upnorm + up conv, k = 2 .. 8
    g_c = None
    for k in range(2, N_LEVELS + 1):
        nm = level_names(k)
        L = lv[k]
        outer, inner_p = ch[k - 1][2], ch[k - 2][1]
        u = L["u"]
        g_u = Buf.empty(N, u.h, u.w, outer, 1, dev)
        ops.bn_bwd(Slice(g_cat[k - 1], inner_p, inner_p), FG_ACT_RELU, None, 0, u, 1, L["umean"], L["uinvstd"],
                   P[nm["upnorm"] + ".weight"], P[nm["upnorm"] + ".bias"], L["mask"], g_u,
                   G.get(nm["upnorm"] + ".weight"), G.get(nm["upnorm"] + ".bias"), G.acc)
        ops.zero_border(g_u)
        xin = L["r"] if k == N_LEVELS else L["cat"]
        w = P[nm["up"] + ".weight"]
        G.wgrad(PL.wgrad_convT(xin, g_u, 4, 1, w.shape[0]), PL.wmap_wgrad(w.shape, True, g_u.c, 4),
                nm["up"] + ".weight", (xin, g_u))
        G.ready(ready, nm["up"])
        g_x = Buf.empty(N, xin.h, xin.w, xin.c, 0, dev)
        m = PL.wmap_convT_dgrad(w.shape, g_u.c)
        ops.conv([PL.conv_problem(g_u, 1, 4, 2, ops.pack_weight(w, m), m, g_x)])
        if k == N_LEVELS:
            g_c = Buf.empty(N, xin.h, xin.w, xin.c, 1, dev)      # through ReLU(D_8)
            ops.bn_bwd(g_x, FG_ACT_RELU, None, 0, L["c"], 1, None, None, None, None, None, g_c)
            ops.zero_border(g_c)
        else:
            g_cat[k] = g_x
    # ---- down chain: level k's down conv (+ downnorm), k = 8 .. 2, then level 1
    for k in range(N_LEVELS, 1, -1):
        nm = level_names(k)
        L = lv[k]
        if k < N_LEVELS:
            inner = ch[k - 1][1]
            c = L["c"]
            g_c = Buf.empty(N, c.h, c.w, inner, 1, dev)
            ops.bn_bwd(g_a, FG_ACT_LRELU, Slice(g_cat[k], 0, inner), FG_ACT_RELU, c, 1, L["mean"], L["invstd"],
                       P[nm["downnorm"] + ".weight"], P[nm["downnorm"] + ".bias"], None, g_c,
                       G.get(nm["downnorm"] + ".weight"), G.get(nm["downnorm"] + ".bias"), G.acc)
            ops.zero_border(g_c)
        X._wgrad_conv(P, G, nm["down"], g_c, L["a"], 1, 4, 2)
        G.ready(ready, nm["down"])
        a = L["a"]
        g_a = Buf.empty(N, a.h, a.w, a.c, 0, dev)
        X._dgrad_s2(P, nm["down"], g_c, 4, Y=g_a)
    L = lv[1]
    nm = level_names(1)
    g_d1 = Buf.empty(N, L["c"].h, L["c"].w, 64, 0, dev)
    ops.bn_bwd(g_a, FG_ACT_LRELU, Slice(g_cat[1], 0, 64), FG_ACT_RELU, L["c"], 1, None, None, None, None, None, g_d1)
    X._wgrad_conv(P, G, nm["down"], g_d1, L["a"], 1, 4, 2)
    G.ready(ready, nm["down"])
    G.join()
    return G.out


def gen_act_decisions(S):
    """the generator's activation decisions in a saved forward, keyed by oracle/pix2pix.py's names
    (test instrumentation for teacher-forced gradient comparisons)"""
    lv = S["lv"]
    ch = level_channels(S["x"].shape[1])
    out = {"inner": X._decided(lv[N_LEVELS]["r"])}
    for k in range(1, N_LEVELS):
        out[f"down{k}"] = X._decided(lv[k + 1]["a"])
    for k in range(2, N_LEVELS + 1):
        inner_p = ch[k - 2][1]
        out[f"up{k}"] = X._decided(Slice(lv[k - 1]["cat"], inner_p, inner_p))
    return out


# ======================================================================================
# discriminator
# ======================================================================================

def disc_forward(P, B, inp, groups=1, training=True, save=True):
    """inp: Buf from executor.disc_pack (zero border 1), groups: separate BatchNorm calls stacked
    along the batch.  Returns (pred [N, 1, ho, wo], saved)."""
    N, H, W = inp.n, inp.h, inp.w
    dev = inp.t.device
    if H < 24 or W < 24:
        raise RuntimeError(f"Pix2PixDiscriminator needs H, W >= 24 (got {H}x{W})")
    h1, w1 = PL.out_size(H, 4, 2, 1), PL.out_size(W, 4, 2, 1)
    e0 = Buf.empty(N, h1, w1, 64, 1, dev)
    _conv_nb(P, "model.0", inp, 1, 4, 2, e0, act=FG_ACT_LRELU)
    ops.zero_border(e0)
    S = dict(inp=inp, e0=e0, groups=groups)
    prev = e0
    for conv, stride, c in (("model.2", 2, 128), ("model.5", 2, 256), ("model.8", 1, 512)):
        norm = DISC_NORMS[conv]
        hh, ww = PL.out_size(prev.h, 4, stride, 1), PL.out_size(prev.w, 4, stride, 1)
        e = Buf.empty(N, hh, ww, c, 0, dev)
        _conv_nb(P, conv, prev, 1, 4, stride, e, tag="p2p_d_model8_fwd" if conv == "model.8" else None)
        mean, invstd = _stats(B, norm, e, groups, training)
        a = Buf.zeros(N, hh, ww, c, 1, dev)
        ops.bn_apply(e, groups, mean, invstd, P[norm + ".weight"], P[norm + ".bias"], None, FG_ACT_LRELU, a)
        S[conv] = dict(x=prev, e=e, mean=mean, invstd=invstd, a=a)
        prev = a
    h5, w5 = PL.out_size(prev.h, 4, 1, 1), PL.out_size(prev.w, 4, 1, 1)
    pred = torch.empty(N, 1, h5, w5, dtype=torch.float32, device=dev)
    ops.conv_n1_fwd(prev, P["model.11.weight"], P["model.11.bias"], pred)
    return pred, (S if save else None)


def disc_backward(P, S, g_pred, param_grads=True, grads_into=None, input_grad=None, input_grad_channels=None,
                  input_grad_accumulate=False, ready=None):
    """Explicit backward of disc_forward (see executor.disc_backward for the arguments)."""
    ready = (ready if param_grads and ready is not None else (lambda name: None))
    inp, groups = S["inp"], S["groups"]
    N = inp.n
    dev = inp.t.device
    G = X._Grads(P, grads_into, device=dev)
    a3 = S["model.8"]["a"]
    h5, w5 = g_pred.shape[2], g_pred.shape[3]
    g11 = Buf.empty(N, h5, w5, 1, 3, dev)
    ops.pack_input(g_pred, 1, None, 0, g11, 0, N, FG_PAD_ZERO)
    if param_grads:
        w11 = P["model.11.weight"]
        G.off_path(lambda: ops.conv_n1_wgrad(a3, g11, PL.wmap_wgrad(w11.shape, True, a3.c, 4),
                                             G.get("model.11.weight")), (a3, g11), ("model.11.weight",))
        ops.channel_sum(g11, 1, G.get("model.11.bias"))
        G.ready(ready, "model.11")
    g_a = Buf.empty(N, a3.h, a3.w, 512, 0, dev)
    X._dgrad_s1(P, "model.11", g11, 2, 4, g_a)
    for conv, stride in (("model.8", 1), ("model.5", 2), ("model.2", 2)):
        norm = DISC_NORMS[conv]
        L = S[conv]
        e = L["e"]
        g_e = Buf.empty(N, e.h, e.w, e.c, 2 if stride == 1 else 1, dev)
        ops.bn_bwd(g_a, FG_ACT_LRELU, None, 0, e, groups, L["mean"], L["invstd"], P[norm + ".weight"],
                   P[norm + ".bias"], None, g_e, G.get(norm + ".weight") if param_grads else None,
                   G.get(norm + ".bias") if param_grads else None)
        ops.zero_border(g_e)
        if param_grads:
            X._wgrad_conv(P, G, conv, g_e, L["x"], 1, 4, stride)
            G.ready(ready, conv)
        xprev = L["x"]
        g_a = Buf.empty(N, xprev.h, xprev.w, xprev.c, 1 if conv == "model.2" else 0, dev)
        if stride == 1:
            X._dgrad_s1(P, conv, g_e, 2, 4, g_a)
        else:
            X._dgrad_s2(P, conv, g_e, 4, Y=g_a)
    e0 = S["e0"]
    g_e0 = g_a
    ops.zero_border(g_e0)
    ops.act_bwd(g_e0, e0, FG_ACT_LRELU)
    if param_grads:
        X._wgrad_conv(P, G, "model.0", g_e0, inp, 1, 4, 2)
        ops.channel_sum(g_e0, 64, G.get("model.0.bias"))
        G.ready(ready, "model.0")
    if input_grad is not None:
        c0, cn = input_grad_channels
        assert input_grad.is_contiguous() and input_grad.shape[1] >= cn
        X._dgrad_s2(P, "model.0", g_e0, 4, y_nchw=(input_grad.view(-1), input_grad.shape[1], inp.h, inp.w),
                    n_base=c0, n_out=cn, accumulate=int(input_grad_accumulate))
    G.join()
    return G.out


def disc_act_decisions(S, lo=0, hi=None):
    return {"model.0": X._decided(S["e0"], lo, hi), "model.2": X._decided(S["model.2"]["a"], lo, hi),
            "model.5": X._decided(S["model.5"]["a"], lo, hi), "model.8": X._decided(S["model.8"]["a"], lo, hi)}
