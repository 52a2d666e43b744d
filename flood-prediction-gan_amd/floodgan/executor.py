"""Native forward / backward executors of the PairedAttention generator and discriminator.

These run the whole network as a fixed sequence of libfloodgan kernels over NHWC buffers
(floodgan.plans.Buf), saving exactly the activations the explicit backward needs.  Both the
autograd-facing drop-in modules (floodgan.model_architectures) and the fused training step
(floodgan.model.paired_step) are built on them.

Reference: models/model_architectures.py:339-400 (generator forward), :412-418 (resnet
block), :424-441 (discriminator); backward = autograd of those graphs.
"""
import os

import torch

from . import _lib as L
from . import ops
from . import plans as PL
from ._lib import FG_ACT_LRELU, FG_ACT_NONE, FG_ACT_RELU, FG_PAD_REFLECT, FG_PAD_ZERO, require_device
from .plans import Buf

N_BLOCKS = 9
CONTENT_ALLOC = 32   # 27 content channels, padded for aligned NHWC rows
N_ATT = 10           # attention logits (deconv3_attention's output channels)
# the attention head's 1x1 conv and its gradients run as exact-fp32 FMA work (csrc/head1x1.hip; the implicit-GEMM
# engine path lost -0.13 ms per step, profiles/round2/r2ag_ab_head_1x1.log, and was retired in round 6).  Round 5: the attention head's 1x1 conv fused into the norm passes of its input (fg_in_apply_head / fg_in_bwd_head:
# the forward's logits formed by the apply pass, the backward's 64-channel input gradient formed in registers from the
# logits gradient by the statistics and apply passes) -- no conv1x1 forward / input-gradient launches and no re-read
# or materialisation of a 537-MB 64-channel tensor; bit-identical; interleaved A/B 45.95 -> 45.60 ms per step
# (profiles/round5/r5f_ab_fused_head.log).  FLOODGAN_FUSED_HEAD=0: the separate head1x1 kernels (the reference the
# fused passes are tested against, tests/test_gpu_northstar.py::test_fused_attention_head)
FUSED_HEAD = os.environ.get("FLOODGAN_FUSED_HEAD", "1") != "0"
ATT_ALLOC = 16       # 10 attention channels


def _blk(i, j):
    return f"resnet_blocks.{i}.conv{j}"


def generator_param_names():
    names = ["conv1", "conv2", "conv3"] + [_blk(i, j) for i in range(N_BLOCKS) for j in (1, 2)]
    names += ["deconv1_content", "deconv2_content", "deconv3_content",
              "deconv1_attention", "deconv2_attention", "deconv3_attention"]
    return names


DISC_LAYERS = ["model.0", "model.2", "model.5", "model.8", "model.11"]

# D's input gradient restricted to a few channels (the G step's dL/d(fake)) on its fp32 kernel (fg_d0_input_grad);
# FLOODGAN_D0_DGRAD=0: the restricted 4-phase transposed conv on the engine
D0_DGRAD = os.environ.get("FLOODGAN_D0_DGRAD", "1") != "0"


def disc_bucket_names():
    """the discriminator's gradient buckets (one per layer) in the order disc_backward completes them"""
    return [[f"{layer}.{k}" for k in ("weight", "bias")] for layer in reversed(DISC_LAYERS)]


class _Grads:
    """Destination of parameter gradients: either fresh tensors (autograd path) or
    preallocated .grad tensors (fused step).

    Every launch runs on the caller's (current) stream.  Weight gradients on a second stream beside the
    input-gradient chain were measured slower (profiles/round2/r2m_*: 57.3 vs 56.6 ms per step; the
    pipelined convs already hold every CU, so the overlapped kernels each slow down by the same factor)
    and that path was removed in round 5."""

    def __init__(self, params, into=None, accumulate=False, device=None):
        self.params, self.into = params, into
        self.acc = accumulate       # raise existing gradients (a network used several times per step)
        self.out = {}

    def get(self, name):
        if name not in self.out:
            p = self.params[name]
            if self.into is not None and name in self.into:
                self.out[name] = self.into[name]
            else:
                self.out[name] = torch.empty_like(p)
        return self.out[name]

    def off_path(self, fn, bufs, names=(), prepare=None):
        """run fn() (weight-gradient launches reading the Bufs `bufs`, writing the gradients `names`)"""
        for n in names:
            self.get(n)
        return fn()

    def wgrad(self, prob, wmap, name, bufs, tag=None):
        self.off_path(lambda: ops.wgrad(prob, wmap, self.get(name), accumulate=self.acc, tag=tag), bufs, (name,),
                      prepare=lambda: ops.prepare_wgrad(prob))

    def ready(self, ready, name):
        return ready(name)

    def join(self):
        pass


# ======================================================================================
# generator
# ======================================================================================

def _conv_fwd(P, name, X, pad, k, stride, Y, act=FG_ACT_NONE, tag=None, in_stats=False):
    """returns the InstanceNorm statistics of Y from the conv's epilogue when in_stats and available"""
    w = P[name + ".weight"]
    m = PL.wmap_conv_fwd(w.shape, X.c)
    return ops.conv([PL.conv_problem(X, pad, k, stride, ops.pack_weight(w, m), m, Y, bias=P[name + ".bias"],
                                     act=act)], tag=tag, in_stats=in_stats)


# round 5: the four output phases of a stride-2, 3-tap transposed op with 64 output channels as ONE problem (the quad
# form, plans.quad_map): each input pixel gathered once for all phases, zero segments skipped in the kernel.  The
# FLOODGAN_QUAD=0 switch was retired in round 6: the four-phase problems remain for every other shape, and
# tests/test_gpu_parity.py::test_quad_convT checks the quad form against fp64.
def _quad_ok(X, shape, k, Y):
    return (k == 3 and shape[1] == 64 and isinstance(Y, Buf) and Y.c == 64 and ops.is_presplit(X)
            and L.fwd_f16x3() and (Y.h, Y.w, Y.n) == (2 * X.h, 2 * X.w, X.n) and X.pad >= 1 and X.c % 32 == 0
            and X.c & (X.c - 1) == 0)


def _quad(P, name, X, Y, bias=None, in_stats=False):
    w = P[name + ".weight"]
    m, d0, mask = PL.quad_map(w.shape, 3, 1, X.c)
    return ops.conv([PL.quad_problem(X, m, d0, mask, ops.pack_weight(w, m), Y, bias=bias)], in_stats=in_stats)


def _convT_fwd(P, name, X, Y):
    w = P[name + ".weight"]
    if _quad_ok(X, w.shape, 3, Y):
        return _quad(P, name, X, Y, bias=P[name + ".bias"], in_stats=True)
    maps = PL.phase_maps(w.shape, 3, 1, X.c)
    wps = [ops.pack_weight(w, m) for m, _, _ in maps]
    return ops.conv(PL.phase_problems(X, w.shape, 3, 1, Y, wps, maps, bias=P[name + ".bias"]), in_stats=True)


def _norm(c, act, pad, mode, residual=None, stats=None, presplit=False, ps_copy=False, splitpix=False):
    """InstanceNorm + activation of conv output c; stats = (mean, rstd) from the conv's epilogue, or
    computed here.  presplit: the output is written in the FG_PRESPLIT format (read only by convs).  ps_copy: also a
    FG_PRESPLIT copy of the fp32 output (returned as a 4th value, None when the f16x3 pre-split path is off)"""
    mean, rstd = stats if stats is not None else ops.in_stats(c)
    out = Buf.empty(c.n, c.h, c.w, c.c, pad, c.t.device)
    ps = (Buf.empty(c.n, c.h, c.w, c.c, pad, c.t.device)
          if ps_copy and ops.presplit_on() and ops.PRESPLIT_RESID else None)
    if ps is not None and not ops.presplit_fits(ps):
        ps = None                  # beyond what the pre-split consumers take (ops.PRESPLIT_MAX_BYTES)
    ops.in_apply(c, mean, rstd, act, residual, out, mode, presplit=presplit, ps_copy=ps, splitpix=splitpix)
    return (mean, rstd, out, ps) if ps_copy else (mean, rstd, out)


# the content head's input is written in the window kernels' split layout by its norm pass (step 46.39 -> 46.19 ms,
# profiles/round4/r4e_ab_splitpix.log; the fp32 + fg_split_pixels alternative was retired in round 6)


def has_attention(P):
    """PairedAttention / AttentionGAN generators carry the attention head; CycleGAN's does not"""
    return "deconv3_attention.weight" in P


def gen_forward(P, x, save=True, x_extra=None):
    """x: [N, C, H, W] fp32 (any strides) on the device.  Returns (out [N,3,H,W], mask [N,H,W], saved).
    x_extra (optional [N, Ce, H, W]): the generator input is cat((x, x_extra), 1), packed without
    materialising the cat (the cycle path's `torch.cat((image, conditions), 1)`, models/model.py:682-689);
    x must then hold >= 3 channels (the tail composites input[:, :3]).
    The same graph serves the CycleGAN ResNet generator (models/model_architectures.py:91-120) when
    P has no attention head: one decoder and a tanh head (conv 7x7 64->3); mask is then None."""
    require_device(x, "generator input")
    N, Cin, H, W = x.shape
    Ce = 0
    if x_extra is not None:
        require_device(x_extra, "generator input")
        Ce = x_extra.shape[1]
        assert x_extra.shape[0] == N and tuple(x_extra.shape[2:]) == (H, W) and Cin >= 3
    if H % 4 or W % 4 or H < 8 or W < 8:
        raise RuntimeError(f"PairedAttentionGenerator needs H, W divisible by 4 and >= 8 (got {H}x{W})")
    dev = x.device
    S = {}
    X0 = Buf.empty(N, H, W, Cin + Ce, 3, dev)
    ops.pack_input(x, Cin, x_extra, Ce, X0, 0, N, FG_PAD_REFLECT)             # F.pad(input, 3, reflect)
    c1 = Buf.empty(N, H, W, 64, 0, dev)
    st = _conv_fwd(P, "conv1", X0, 3, 7, 1, c1, in_stats=True)
    ps = ops.presplit_on()     # norm outputs read only by pipelined convs / weight gradients: FG_PRESPLIT
    m1, r1, a1 = _norm(c1, FG_ACT_RELU, 1, FG_PAD_ZERO, stats=st, presplit=ps)
    c2 = Buf.empty(N, H // 2, W // 2, 128, 0, dev)
    st = _conv_fwd(P, "conv2", a1, 1, 3, 2, c2, in_stats=True)
    m2, r2, a2 = _norm(c2, FG_ACT_RELU, 1, FG_PAD_ZERO, stats=st, presplit=ps)
    c3 = Buf.empty(N, H // 4, W // 4, 256, 0, dev)
    st = _conv_fwd(P, "conv3", a2, 1, 3, 2, c3, in_stats=True)
    # block inputs / outputs: fp32 (the residual stream) and a pre-split copy for the convs that read them
    m3, r3, h, h_ps = _norm(c3, FG_ACT_RELU, 1, FG_PAD_REFLECT, stats=st, ps_copy=True)
    S.update(x=x, X0=X0, cin=Cin + Ce, c1=c1, m1=m1, r1=r1, a1=a1, c2=c2, m2=m2, r2=r2, a2=a2, c3=c3, m3=m3, r3=r3)
    blocks = []
    for i in range(N_BLOCKS):
        # block output feeds the next block (reflect pad) or the deconv heads (zero pad)
        mode = FG_PAD_REFLECT if i < N_BLOCKS - 1 else FG_PAD_ZERO
        h, h_ps, b = _block_fwd(P, f"resnet_blocks.{i}.", h, mode, h_ps)
        blocks.append(b)
    S.update(blocks=blocks, h=h, h_ps=h_ps)
    heads = {}
    attention = has_attention(P)
    for tag, pad2, mode2 in (("content", 3, FG_PAD_REFLECT), ("attention", 0, FG_PAD_ZERO))[:1 + attention]:
        d1 = Buf.empty(N, H // 2, W // 2, 128, 0, dev)
        st = _convT_fwd(P, f"deconv1_{tag}", h if h_ps is None else h_ps, d1)
        md1, rd1, ad1 = _norm(d1, FG_ACT_RELU, 1, FG_PAD_ZERO, stats=st, presplit=ps)
        d2 = Buf.empty(N, H, W, 64, 0, dev)
        st = _convT_fwd(P, f"deconv2_{tag}", ad1, d2)
        # the content head's ad2 is read only by the window conv and its weight gradient: written in their split
        # layout directly (no fp32 copy, no fg_split_pixels pass)
        # (when the window kernels take the head: output rows of >= 256 px, a multiple of 32; ops.win_eligible)
        spx = tag == "content" and ps and ops.USE_WIN and W >= 256 and W % 32 == 0
        if tag == "attention" and FUSED_HEAD:
            # the 1x1 head's logits from relu(IN(d2)) in the norm pass (fg_in_apply_head); the activation itself is
            # not written: the head's backward recomputes it from d2 for the weight gradient (round 5)
            md2, rd2 = st if st is not None else ops.in_stats(d2)
            ad2 = None
            al = Buf.empty(N, H, W, ATT_ALLOC, 0, dev)
            ops.in_apply_head(d2, md2, rd2, FG_ACT_RELU, None, FG_PAD_ZERO, P["deconv3_attention.weight"],
                              P["deconv3_attention.bias"], N_ATT, al)
        else:
            md2, rd2, ad2 = _norm(d2, FG_ACT_RELU, pad2, mode2, stats=st, splitpix=spx)
        heads[tag] = dict(d1=d1, md1=md1, rd1=rd1, ad1=ad1, d2=d2, md2=md2, rd2=rd2, ad2=ad2)
    cl = Buf.empty(N, H, W, CONTENT_ALLOC, 0, dev)
    _conv_fwd(P, "deconv3_content", heads["content"]["ad2"], 3, 7, 1, cl)
    out = torch.empty(N, 3, H, W, dtype=torch.float32, device=dev)
    if not attention:                                 # CycleGAN: nn.Tanh() on the 3 logits (:115-117)
        ops.tanh_head_fwd(cl, 3, out)
        S.update(heads=heads, cl=cl)
        return out, None, (S if save else None)
    if not FUSED_HEAD:
        al = Buf.empty(N, H, W, ATT_ALLOC, 0, dev)
        # 1x1 64 -> 10: a per-pixel matrix-vector product, fp32 FMA over LDS-staged tiles (csrc/head1x1.hip)
        ops.conv1x1_fwd(heads["attention"]["ad2"], P["deconv3_attention.weight"], P["deconv3_attention.bias"],
                        N_ATT, al)
    # (FUSED_HEAD: al was written by the attention head's norm pass above)
    mask = torch.empty(N, H, W, dtype=torch.float32, device=dev)
    ops.tail_fwd(cl, al, x, out, mask)
    S.update(heads=heads, cl=cl, al=al)
    return out, mask, (S if save else None)


def _block_fwd(P, pre, h, out_mode, h_ps=None):
    """PairedAttentionBlock (models/model_architectures.py:412-418) over h (reflect border 1; h_ps: its pre-split copy,
    which conv1 reads when given): returns (block output with `out_mode` border 1, its pre-split copy or None, saved
    tensors)."""
    N, Hh, Ww, Cc = h.n, h.h, h.w, h.c
    dev = h.t.device
    cb1 = Buf.empty(N, Hh, Ww, Cc, 0, dev)
    st = _conv_fwd(P, pre + "conv1", h if h_ps is None else h_ps, 1, 3, 1, cb1, tag="resblock_conv_fwd", in_stats=True)
    # rb is read only by conv2 and conv2's weight gradient: pre-split for both (ops.PRESPLIT)
    mb1, rb1, rb = _norm(cb1, FG_ACT_RELU, 1, FG_PAD_REFLECT, stats=st, presplit=ops.presplit_on())
    cb2 = Buf.empty(N, Hh, Ww, Cc, 0, dev)
    st = _conv_fwd(P, pre + "conv2", rb, 1, 3, 1, cb2, tag="resblock_conv_fwd", in_stats=True)
    if h_ps is None:          # a lone block (block_forward_nchw): no copies
        mb2, rb2, hn = _norm(cb2, FG_ACT_NONE, 1, out_mode, residual=h, stats=st)
        hn_ps = None
    else:
        mb2, rb2, hn, hn_ps = _norm(cb2, FG_ACT_NONE, 1, out_mode, residual=h, stats=st, ps_copy=True)
    return hn, hn_ps, dict(h=h, h_ps=h_ps, cb1=cb1, mb1=mb1, rb1=rb1, rb=rb, cb2=cb2, mb2=mb2, rb2=rb2)


def _block_bwd(P, pre, b, grad, G):
    """Backward of _block_fwd: grad = dL/d(block output) -> dL/d(block input), both as a lazy sum
    (gsrc, fold_pad, gadd): the gradient is fold(gsrc) + gadd -- the next block's input gradient is the
    reflect-pad adjoint of its conv1 input gradient plus the residual path's gradient, and its norm
    backward's statistics pass gathers that sum directly (and writes it out once, for this block's own
    residual path: gsum), so no separate fold + add pass runs.  The caller joins G's side stream."""
    gsrc, fold, gadd = grad
    cb2 = b["cb2"]
    N, Hh, Ww, Cc = cb2.n, cb2.h, cb2.w, cb2.c
    dev = cb2.t.device
    lazy = fold > 0 or gadd is not None
    g_h = Buf.empty(N, Hh, Ww, Cc, 0, dev) if lazy else gsrc
    g_cb2 = Buf.empty(N, Hh, Ww, Cc, 2, dev)          # zero border 2: full correlation of a 3x3
    # the conv-output gradients are read only by the input-gradient convs and the weight gradients: pre-split
    ps = ops.presplit_on()
    ops.in_bwd(gsrc, fold, gadd, cb2, b["mb2"], b["rb2"], FG_ACT_NONE, g_cb2, G.get(pre + "conv2.bias"), G.acc,
               gsum=g_h if lazy else None, presplit=ps)
    _wgrad_conv(P, G, pre + "conv2", g_cb2, b["rb"], 1, 3, 1, tag="resblock_conv_wgrad")
    g_rbp = _dgrad_s1_padded(P, pre + "conv2", g_cb2)  # gradient w.r.t. the reflect-padded relu output
    g_cb1 = Buf.empty(N, Hh, Ww, Cc, 2, dev)
    ops.in_bwd(g_rbp, 1, None, b["cb1"], b["mb1"], b["rb1"], FG_ACT_RELU, g_cb1, G.get(pre + "conv1.bias"), G.acc,
               presplit=ps)
    _wgrad_conv(P, G, pre + "conv1", g_cb1, b["h"] if b.get("h_ps") is None else b["h_ps"], 1, 3, 1,
                tag="resblock_conv_wgrad")
    g_hp = _dgrad_s1_padded(P, pre + "conv1", g_cb1)
    return g_hp, 1, g_h                               # reflect-pad adjoint + residual path, summed lazily


def _dgrad_s1_padded(P, name, gy):
    """Input gradient of a 3x3 stride-1 conv that read a reflect-padded (1) input: the gradient over the
    whole (H+2) x (W+2) padded domain, as an unpadded Buf of that extent (the layout in_bwd / fold_add
    fold).  Computed as the H x W interior -- an output grid of H-px rows, which the pipelined kernel's
    256-row tiles split evenly (the (H+2)-px grid at bs 8, 128^2 gives 529 tiles for 256 resident
    workgroups: 3 rounds instead of 2, +38 %, profiles/round2/r2n_diag_dgrad.log) -- plus the four
    one-pixel edge strips in a second launch.  gy's zero border leaves one kernel row (row strips) or
    column (column strips) there: K = 3 x C instead of 9 x C."""
    N, Hh, Ww, Cc = gy.n, gy.h, gy.w, gy.c
    assert gy.pad >= 2
    w = P[name + ".weight"]
    m = PL.wmap_conv_dgrad_s1(w.shape, gy.c)
    wp = ops.pack_weight(w, m)
    out = Buf.empty(N, Hh, Ww, Cc, 1, gy.t.device)     # interior = padded rows / cols 1..H
    ops.conv([PL.conv_problem(gy, 1, 3, 1, wp, m, out)], tag="resblock_conv_dgrad")
    # padded-domain position p reads gy rows / cols p-2 .. p (relative to gy's interior; rows -2, -1 and
    # H, H+1 are zero); out's interior origin is padded position 1.  Row strips: one row of the full
    # pack (gather row r at pack row r); column strips: packs of their single kernel column.
    strips = [PL.window_problem(gy, 0, -2, 1, Ww + 2, 1, 3, wp, m, out, -1, -1, w_row0=2),          # row 0
              PL.window_problem(gy, Hh - 1, -2, 1, Ww + 2, 1, 3, wp, m, out, Hh, -1, w_row0=0)]     # row H+1
    for col, x0, ox in ((2, 0, -1), (0, Ww - 1, Ww)):                                               # columns 0, W+1
        ms = PL.wmap_conv_dgrad_s1_taps(w.shape, gy.c, (0, 1, 2), (col,))
        strips.append(PL.window_problem(gy, -1, x0, Hh, 1, 3, 1, ops.pack_weight(w, ms), ms, out, 0, ox))
    # 24 k-steps of K = 768 per tile: ~31-33 us on every tile shape (128 x 64 auto, 128 x 128, 256 x 64, ...:
    # profiles/round6/r6m_ab_strip_tile_not_kept.log)
    ops.conv(strips, tag="resblock_dgrad_strips")
    return out.padded()


def _to_nchw(B):
    return B.interior().permute(0, 3, 1, 2)


def block_forward_nchw(x, params, save=True):
    """A lone PairedAttentionBlock on an NCHW tensor (params: w1, b1, w2, b2)."""
    require_device(x, "block input")
    N, Cc, Hh, Ww = x.shape
    P = {"conv1.weight": params["w1"], "conv1.bias": params["b1"],
         "conv2.weight": params["w2"], "conv2.bias": params["b2"]}
    h = Buf.empty(N, Hh, Ww, Cc, 1, x.device)
    ops.pack_input(x, Cc, None, 0, h, 0, N, FG_PAD_REFLECT)
    hn, _, b = _block_fwd(P, "", h, FG_PAD_ZERO)
    return _to_nchw(hn), (dict(P=P, b=b) if save else None)


def block_backward_nchw(S, g, need_input=True):
    N, Cc, Hh, Ww = g.shape
    gb = Buf.empty(N, Hh, Ww, Cc, 0, g.device)
    ops.pack_input(g, Cc, None, 0, gb, 0, N, FG_PAD_ZERO)
    G = _Grads(S["P"], device=g.device)
    g_hp, fold, g_res = _block_bwd(S["P"], "", S["b"], (gb, 0, None), G)
    g_new = Buf.empty(N, Hh, Ww, Cc, 0, g.device)
    ops.fold_add(g_hp, fold, g_res, g_new)
    G.join()
    grads = {"w1": G.out["conv1.weight"], "b1": G.out["conv1.bias"],
             "w2": G.out["conv2.weight"], "b2": G.out["conv2.bias"]}
    return (_to_nchw(g_new) if need_input else None), grads


def _wgrad_conv(P, G, name, gy, X, pad, k, stride, tag=None):
    w = P[name + ".weight"]
    G.wgrad(PL.wgrad_conv(gy, X, pad, k, stride, w.shape[0]), PL.wmap_wgrad(w.shape, True, X.c, k), name + ".weight",
            (gy, X), tag=tag)


def _dgrad_s1(P, name, gyp, pad_used, k, Y):
    w = P[name + ".weight"]
    m = PL.wmap_conv_dgrad_s1(w.shape, gyp.c)
    ops.conv([PL.conv_problem(gyp, pad_used, k, 1, ops.pack_weight(w, m), m, Y)])


def _dgrad_s2(P, name, gy, k, Y=None, y_nchw=None, n_base=0, n_out=None, accumulate=0):
    w = P[name + ".weight"]
    if y_nchw is None and not n_base and n_out is None and not accumulate and _quad_ok(gy, w.shape, k, Y):
        _quad(P, name, gy, Y)
        return
    maps = PL.phase_maps(w.shape, k, 1, gy.c, n_base=n_base, n_out=n_out)
    wps = [ops.pack_weight(w, m) for m, _, _ in maps]
    ops.conv(PL.phase_problems(gy, w.shape, k, 1, Y, wps, maps, y_nchw=y_nchw, accumulate=accumulate))


G_BUCKETS = ([f"{h}_{t}" for t in ("content", "attention") for h in ("deconv1", "deconv2", "deconv3")],) + \
    tuple([_blk(i, 1), _blk(i, 2)] for i in reversed(range(N_BLOCKS))) + (["conv1", "conv2", "conv3"],)


def gen_bucket_names(P=None):
    """the generator's gradient buckets in the order gen_backward completes them (parallel.FlatGrads);
    with P, only the layers P holds (the CycleGAN generator has no attention head)"""
    out = []
    for b in G_BUCKETS:
        names = [f"{layer}.{k}" for layer in b for k in ("weight", "bias")]
        if P is not None:
            names = [n for n in names if n in P]
        if names:
            out.append(names)
    return out


def gen_backward(P, S, g_out, grads_into=None, ready=None, input_grad=None, accumulate=False, g_mask=None):
    """Explicit backward of gen_forward.  g_out: [N,3,H,W] (any strides).  Returns
    {param name: grad} (written into grads_into[name] when given).  ready(layer name), when
    given, is called as soon as a gradient bucket (G_BUCKETS) is complete.  input_grad (optional
    [N,C,H,W] tensor, any strides) receives dL/d(input): the cycle path back-propagates through
    one generator into the other (models/model.py:677-706); the paired step never asks for it.
    accumulate: add into grads_into instead of overwriting (a generator applied several times in
    one cycle iteration).  g_mask (optional [N, H, W], any strides): dL/d(last_attention_mask), for a
    loss that reads the mask (models/model_architectures.py:396 keeps it in the autograd graph)."""
    ready = ready or (lambda name: None)
    x = S["x"]
    G = _Grads(P, grads_into, accumulate, device=x.device)
    assert not accumulate or grads_into is not None
    N, _, H, W = x.shape
    Cin = S["cin"]             # input channels, including a fused x_extra
    dev = x.device
    attention = has_attention(P)
    n_content = 27 if attention else 3
    # ---- tail: tanh / softmax / composite backward (models/model_architectures.py:352-399), or the
    # CycleGAN tanh head (:115-117)
    cl = S["cl"]
    gcl = Buf.empty(N, H, W, CONTENT_ALLOC, 6, dev)     # zero border 6 = full correlation of a 7x7
    hc = S["heads"]["content"]
    if attention:
        al = S["al"]
        gal = Buf.empty(N, H, W, ATT_ALLOC, 0, dev)
        ops.tail_bwd(cl, al, x, g_out, gcl, gal, gx=input_grad, g_mask=g_mask)   # input_grad[:, :3] = g_out * att10
        ha = S["heads"]["attention"]
    else:
        assert g_mask is None, "the CycleGAN generator has no attention mask"
        ops.tanh_head_bwd(cl, 3, g_out, gcl)
    # ---- deconv3_content: 7x7 over reflect-padded (3) ad2
    _wgrad_conv(P, G, "deconv3_content", gcl, hc["ad2"], 3, 7, 1)
    ops.channel_sum(gcl, n_content, G.get("deconv3_content.bias"), G.acc)
    g_ad2c = Buf.empty(N, H + 6, W + 6, 64, 0, dev)     # gradient w.r.t. the PADDED input
    _dgrad_s1(P, "deconv3_content", gcl, 6, 7, g_ad2c)
    heads = [("content", hc, g_ad2c, 3)]
    if attention:
        # ---- deconv3_attention: 1x1
        # the fused head: weight, bias and input gradients in its norm backward below (g_ad2a None)
        g_ad2a = None if FUSED_HEAD else Buf.empty(N, H, W, 64, 0, dev)
        if g_ad2a is not None:
            names = ("deconv3_attention.weight", "deconv3_attention.bias")
            G.off_path(lambda: ops.conv1x1_wgrad(gal, ha["ad2"], N_ATT, G.get(names[0]), G.get(names[1]), G.acc),
                       (gal, ha["ad2"]), names)
            ops.conv1x1_dgrad(gal, P["deconv3_attention.weight"], N_ATT, g_ad2a)
        heads.append(("attention", ha, g_ad2a, 0))
    # ---- deconv2 / deconv1 of both heads
    g_h = Buf.empty(N, H // 4, W // 4, 256, 0, dev)
    ps = ops.presplit_on()     # conv-output gradients read only by pipelined convs / weight gradients
    for idx, (tag, hd, g_ad2, fold) in enumerate(heads):
        g_d2 = Buf.empty(N, H, W, 64, 1, dev)
        if g_ad2 is None:        # the fused head: the input gradient w^T gal formed inside the norm passes, the head's
            # weight / bias gradients from the activation recomputed in the statistics pass
            ops.in_bwd_head(gal, P["deconv3_attention.weight"], N_ATT, hd["d2"], hd["md2"], hd["rd2"], FG_ACT_RELU,
                            g_d2, G.get(f"deconv2_{tag}.bias"), G.acc, presplit=ps,
                            wgrad=(G.get("deconv3_attention.weight"), G.get("deconv3_attention.bias"), G.acc))
        else:
            ops.in_bwd(g_ad2, fold, None, hd["d2"], hd["md2"], hd["rd2"], FG_ACT_RELU, g_d2,
                       G.get(f"deconv2_{tag}.bias"), G.acc, presplit=ps)
        name = f"deconv2_{tag}"
        w = P[name + ".weight"]
        G.wgrad(PL.wgrad_convT(hd["ad1"], g_d2, 3, 1, w.shape[0]), PL.wmap_wgrad(w.shape, True, g_d2.c, 3),
                name + ".weight", (hd["ad1"], g_d2))
        g_ad1 = Buf.empty(N, H // 2, W // 2, 128, 0, dev)
        m = PL.wmap_convT_dgrad(w.shape, g_d2.c)
        ops.conv([PL.conv_problem(g_d2, 1, 3, 2, ops.pack_weight(w, m), m, g_ad1)])
        g_d1 = Buf.empty(N, H // 2, W // 2, 128, 1, dev)
        ops.in_bwd(g_ad1, 0, None, hd["d1"], hd["md1"], hd["rd1"], FG_ACT_RELU, g_d1, G.get(f"deconv1_{tag}.bias"),
                   G.acc, presplit=ps)
        name = f"deconv1_{tag}"
        w = P[name + ".weight"]
        hx = S["h"] if S.get("h_ps") is None else S["h_ps"]
        G.wgrad(PL.wgrad_convT(hx, g_d1, 3, 1, w.shape[0]), PL.wmap_wgrad(w.shape, True, g_d1.c, 3),
                name + ".weight", (hx, g_d1))
        m = PL.wmap_convT_dgrad(w.shape, g_d1.c)
        ops.conv([PL.conv_problem(g_d1, 1, 3, 2, ops.pack_weight(w, m), m, g_h, accumulate=idx)])
    G.ready(ready, "deconv1_content")
    # ---- resnet blocks in reverse: out = h + IN(conv2(pad(relu(IN(conv1(pad(h)))))))
    grad = (g_h, 0, None)
    for i in reversed(range(N_BLOCKS)):
        grad = _block_bwd(P, f"resnet_blocks.{i}.", S["blocks"][i], grad, G)
        G.ready(ready, _blk(i, 1))
    # ---- encoder (the first block's input gradient, fold + residual, gathered by conv3's norm backward)
    g_c3 = Buf.empty(N, H // 4, W // 4, 256, 1, dev)
    ops.in_bwd(grad[0], grad[1], grad[2], S["c3"], S["m3"], S["r3"], FG_ACT_RELU, g_c3, G.get("conv3.bias"), G.acc,
               presplit=ps)
    _wgrad_conv(P, G, "conv3", g_c3, S["a2"], 1, 3, 2)
    g_a2 = Buf.empty(N, H // 2, W // 2, 128, 0, dev)
    _dgrad_s2(P, "conv3", g_c3, 3, Y=g_a2)
    g_c2 = Buf.empty(N, H // 2, W // 2, 128, 1, dev)
    ops.in_bwd(g_a2, 0, None, S["c2"], S["m2"], S["r2"], FG_ACT_RELU, g_c2, G.get("conv2.bias"), G.acc, presplit=ps)
    _wgrad_conv(P, G, "conv2", g_c2, S["a1"], 1, 3, 2)
    g_a1 = Buf.empty(N, H, W, 64, 0, dev)
    _dgrad_s2(P, "conv2", g_c2, 3, Y=g_a1)
    # zero border 6 = the full correlation of the 7x7 stem when the input gradient is wanted
    g_c1 = Buf.empty(N, H, W, 64, 0 if input_grad is None else 6, dev)
    ops.in_bwd(g_a1, 0, None, S["c1"], S["m1"], S["r1"], FG_ACT_RELU, g_c1, G.get("conv1.bias"), G.acc)
    _wgrad_conv(P, G, "conv1", g_c1, S["X0"], 3, 7, 1)
    G.ready(ready, "conv1")
    if input_grad is not None:
        # gradient of the reflect-padded input (9 -> 12 channels: aligned rows), then the pad's
        # adjoint into NCHW, accumulated onto the tail's x[:, :3] term
        g_x0 = Buf.empty(N, H + 6, W + 6, PL.rup(Cin, 4), 0, dev)
        _dgrad_s1(P, "conv1", g_c1, 6, 7, g_x0)
        ops.unfold_nchw(g_x0, 3, Cin, input_grad, acc_channels=3 if attention else 0)
    G.join()
    return G.out


def _decided(B, lo=0, hi=None, pre=None, mean=None):
    """activation decisions of an activation-output Buf (output > 0 <=> input > 0 for ReLU and
    LeakyReLU): NCHW bool on the host.  A pre-split output (FG_PRESPLIT) is decided from the norm's input
    `pre` and `mean` instead: act((c - mean) * rstd) > 0 <=> c > mean (rstd > 0; fp32 subtraction keeps the
    sign)."""
    if B is None or ops.is_presplit(B) or ops.is_splitpix(B):     # (None: the fused head's unwritten activation)
        d = pre.interior() > mean.view(pre.n, 1, 1, pre.c)
        return d[lo:hi].permute(0, 3, 1, 2).contiguous().cpu()
    return (B.interior()[lo:hi] > 0).permute(0, 3, 1, 2).contiguous().cpu()


def gen_act_decisions(S):
    """The generator's ReLU decisions in a saved forward, keyed by the oracle's layer names (test
    instrumentation: oracle ActDecisions teacher-forces them to compare gradients at full size)."""
    out = {"conv1": _decided(S["a1"], pre=S["c1"], mean=S["m1"]), "conv2": _decided(S["a2"], pre=S["c2"], mean=S["m2"]),
           "conv3": _decided(S["blocks"][0]["h"])}
    for i, b in enumerate(S["blocks"]):
        out[f"block{i}"] = _decided(b["rb"], pre=b["cb1"], mean=b["mb1"])
    for tag, hd in S["heads"].items():
        out[f"deconv1_{tag}"] = _decided(hd["ad1"], pre=hd["d1"], mean=hd["md1"])
        out[f"deconv2_{tag}"] = _decided(hd["ad2"], pre=hd["d2"], mean=hd["md2"])
    return out


def disc_act_decisions(S, lo=0, hi=None):
    """The discriminator's LeakyReLU decisions for images lo..hi of a saved forward (test instrumentation)"""
    return {"model.0": _decided(S["e0"], lo, hi), "model.2": _decided(S["a1"], lo, hi, S["e1"], S["m1"]),
            "model.5": _decided(S["a2"], lo, hi, S["e2"], S["m2"]), "model.8": _decided(S["a3"], lo, hi)}


# ======================================================================================
# discriminator
# ======================================================================================

def disc_pack(pairs, c_in_total):
    """Stack (a [N,Ca,H,W], b [N,Cb,H,W] or None) pairs along the batch into one zero-padded
    NHWC input buffer (torch.cat((a, b), 1) of models/model.py:616-617, fused)."""
    a0 = pairs[0][0]
    N = sum(a.shape[0] for a, _ in pairs)
    H, W = a0.shape[2], a0.shape[3]
    buf = Buf.empty(N, H, W, c_in_total, 1, a0.device)
    slot = ops.amax_slot(buf) if len(pairs) > 1 else None      # the parts raise one shared absmax slot
    img0 = 0
    for a, b in pairs:
        require_device(a, "discriminator input")
        cb = 0 if b is None else b.shape[1]
        ops.pack_input(a, a.shape[1], b, cb, buf, img0, a.shape[0], FG_PAD_ZERO, amax=slot)
        img0 += a.shape[0]
    return buf


def disc_prefix(buf, n):
    """The first n images of a disc_pack buffer as a Buf of their own (a view: the G step's D input (x, fake) is the
    D step's first half, so it is not packed again), with the buffer's absmax slot -- it bounds the whole buffer, so
    it bounds the prefix"""
    img = buf.t.numel() // buf.n
    v = Buf(buf.t[:n * img], n, buf.h, buf.w, buf.c, buf.pad)
    slot = getattr(buf.t, "_fg_amax", None)
    if slot is not None and getattr(buf.t, "_fg_amax_ver", None) == buf.t._version:
        v.t._fg_amax, v.t._fg_amax_ver = slot, v.t._version
    return v


def disc_forward(P, inp, save=True):
    """inp: Buf from disc_pack (zero border 1).  Returns (pred [N,1,ho,wo], saved)."""
    N, H, W = inp.n, inp.h, inp.w
    dev = inp.t.device
    if H < 24 or W < 24:
        raise RuntimeError(f"PairedAttentionDiscriminator needs H, W >= 24 (got {H}x{W})")
    h1, w1 = PL.out_size(H, 4, 2, 1), PL.out_size(W, 4, 2, 1)
    e0 = Buf.empty(N, h1, w1, 64, 1, dev)              # conv + bias + LeakyReLU fused, zero border
    _conv_fwd(P, "model.0", inp, 1, 4, 2, e0, act=FG_ACT_LRELU)
    ops.zero_border(e0)
    h2, w2 = PL.out_size(h1, 4, 2, 1), PL.out_size(w1, 4, 2, 1)
    e1 = Buf.empty(N, h2, w2, 128, 0, dev)
    st = _conv_fwd(P, "model.2", e0, 1, 4, 2, e1, in_stats=True)
    ps = ops.presplit_on()     # a1, a2 are read only by pipelined convs / weight gradients: FG_PRESPLIT
    m1, r1, a1 = _norm(e1, FG_ACT_LRELU, 1, FG_PAD_ZERO, stats=st, presplit=ps)
    h3, w3 = PL.out_size(h2, 4, 2, 1), PL.out_size(w2, 4, 2, 1)
    e2 = Buf.empty(N, h3, w3, 256, 0, dev)
    st = _conv_fwd(P, "model.5", a1, 1, 4, 2, e2, in_stats=True)
    m2, r2, a2 = _norm(e2, FG_ACT_LRELU, 1, FG_PAD_ZERO, stats=st, presplit=ps)
    h4, w4 = PL.out_size(h3, 4, 1, 1), PL.out_size(w3, 4, 1, 1)
    e3 = Buf.empty(N, h4, w4, 512, 0, dev)
    st = _conv_fwd(P, "model.8", a2, 1, 4, 1, e3, in_stats=True)
    m3, r3, a3 = _norm(e3, FG_ACT_LRELU, 1, FG_PAD_ZERO, stats=st)
    h5, w5 = PL.out_size(h4, 4, 1, 1), PL.out_size(w4, 4, 1, 1)
    pred = torch.empty(N, 1, h5, w5, dtype=torch.float32, device=dev)
    ops.conv_n1_fwd(a3, P["model.11.weight"], P["model.11.bias"], pred)      # GEMV-shaped: fp32 FMA kernel
    S = dict(inp=inp, e0=e0, e1=e1, m1=m1, r1=r1, a1=a1, e2=e2, m2=m2, r2=r2, a2=a2, e3=e3, m3=m3, r3=r3, a3=a3)
    return pred, (S if save else None)


def disc_backward(P, S, g_pred, param_grads=True, grads_into=None, input_grad=None, input_grad_channels=None,
                  input_grad_accumulate=False, ready=None):
    """Explicit backward of disc_forward.
    param_grads: compute weight / bias gradients (False in the generator step, where D is
    frozen: models/model.py:636-637).  input_grad: contiguous NCHW tensor whose channels 0 .. count
    receive dL/d(input channels input_grad_channels=(start, count)), written or accumulated.  ready(layer name), when
    given, is called as each layer's gradients are complete (parallel.FlatGrads buckets)."""
    ready = (ready if param_grads and ready is not None else (lambda name: None))
    inp = S["inp"]
    N = inp.n
    dev = inp.t.device
    G = _Grads(P, grads_into, device=dev)
    a3 = S["a3"]
    h5, w5 = g_pred.shape[2], g_pred.shape[3]
    g11 = Buf.empty(N, h5, w5, 1, 3, dev)              # zero border 3: the n1 weight-gradient kernel's reach
    ops.pack_input(g_pred, 1, None, 0, g11, 0, N, FG_PAD_ZERO)
    if param_grads:
        w11 = P["model.11.weight"]
        G.off_path(lambda: ops.conv_n1_wgrad(a3, g11, PL.wmap_wgrad(w11.shape, True, a3.c, 4),
                                             G.get("model.11.weight")), (a3, g11), ("model.11.weight",))   # fp32
        ops.channel_sum(g11, 1, G.get("model.11.bias"))
        G.ready(ready, "model.11")
    g_a3 = Buf.empty(N, a3.h, a3.w, 512, 0, dev)
    _dgrad_s1(P, "model.11", g11, 2, 4, g_a3)
    # model.8 (k4 s1 p1) + IN + LReLU
    g_e3 = Buf.empty(N, a3.h, a3.w, 512, 2, dev)
    ps = ops.presplit_on()     # the conv-output gradients feed only pipelined convs / weight gradients
    ops.in_bwd(g_a3, 0, None, S["e3"], S["m3"], S["r3"], FG_ACT_LRELU, g_e3,
               G.get("model.8.bias") if param_grads else None, presplit=ps)
    a2 = S["a2"]
    if param_grads:
        _wgrad_conv(P, G, "model.8", g_e3, a2, 1, 4, 1)
        G.ready(ready, "model.8")
    g_a2 = Buf.empty(N, a2.h, a2.w, 256, 0, dev)
    _dgrad_s1(P, "model.8", g_e3, 2, 4, g_a2)
    # model.5 (k4 s2 p1)
    g_e2 = Buf.empty(N, a2.h, a2.w, 256, 1, dev)
    ops.in_bwd(g_a2, 0, None, S["e2"], S["m2"], S["r2"], FG_ACT_LRELU, g_e2,
               G.get("model.5.bias") if param_grads else None, presplit=ps)
    a1 = S["a1"]
    if param_grads:
        _wgrad_conv(P, G, "model.5", g_e2, a1, 1, 4, 2)
        G.ready(ready, "model.5")
    g_a1 = Buf.empty(N, a1.h, a1.w, 128, 0, dev)
    _dgrad_s2(P, "model.5", g_e2, 4, Y=g_a1)
    # model.2
    g_e1 = Buf.empty(N, a1.h, a1.w, 128, 1, dev)
    ops.in_bwd(g_a1, 0, None, S["e1"], S["m1"], S["r1"], FG_ACT_LRELU, g_e1,
               G.get("model.2.bias") if param_grads else None, presplit=ps)
    e0 = S["e0"]
    if param_grads:
        _wgrad_conv(P, G, "model.2", g_e1, e0, 1, 4, 2)
        G.ready(ready, "model.2")
    g_e0 = Buf.empty(N, e0.h, e0.w, 64, 1, dev)
    _dgrad_s2(P, "model.2", g_e1, 4, Y=g_e0)
    ops.zero_border(g_e0)
    ops.act_bwd(Buf(g_e0.t, N, e0.h, e0.w, 64, 1), e0, FG_ACT_LRELU, border_zero=True)   # LeakyReLU of model.1
    if param_grads:
        _wgrad_conv(P, G, "model.0", g_e0, inp, 1, 4, 2)
        ops.channel_sum(g_e0, 64, G.get("model.0.bias"))
        G.ready(ready, "model.0")
    if input_grad is not None:
        c0, cn = input_grad_channels
        # input_grad: contiguous [N, Ctot, H, W]; D-input channels c0 .. c0+cn land in its channels 0 .. cn
        assert input_grad.is_contiguous() and input_grad.shape[1] >= cn
        if D0_DGRAD and ops.d0_input_grad_ok(g_e0, c0, cn, inp.h, inp.w):
            ops.d0_input_grad(g_e0, P["model.0.weight"], c0, cn, input_grad, input_grad_accumulate)
        else:
            _dgrad_s2(P, "model.0", g_e0, 4, y_nchw=(input_grad.view(-1), input_grad.shape[1], inp.h, inp.w),
                      n_base=c0, n_out=cn, accumulate=int(input_grad_accumulate))
    G.join()
    return G.out
