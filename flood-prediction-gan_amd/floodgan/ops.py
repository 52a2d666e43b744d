"""Thin device-op layer: turns plans / buffers into C-ABI calls on the current HIP stream.

Every function here launches HIP kernels from libfloodgan.so; nothing falls back to ATen.
"""
import ctypes as C

import torch

from . import _lib as L
from .plans import Buf, packed_numel, slab_numel

EPS = 1e-5


def _lib():
    return L.load()


def _dev(t):
    return t.t.device if isinstance(t, Buf) else t.device


def _addr(ref):
    """(Buf|tensor, element offset) -> device address"""
    obj, off = ref
    t = obj.t if isinstance(obj, Buf) else obj
    return t.data_ptr() + 4 * off


def view(B):
    if B is None:
        return L.fg_view(None, 0, 0, 0, 0, 0)
    return L.fg_view(B.t.data_ptr(), B.n, B.h, B.w, B.c, B.pad)


def sview(t):
    """4-D [N, C, H, W] tensor (any strides) -> fg_sview"""
    if t is None:
        return L.fg_sview(None, 0, 0, 0, 0)
    sn, sc, sy, sx = t.stride()
    return L.fg_sview(t.data_ptr(), sn, sc, sy, sx)


def wmap_struct(m):
    s = L.fg_weight_map()
    for k in ("n_out", "kh", "kw", "c", "c_valid", "jp", "dim0_is_n", "d0", "d1", "KH", "KW", "n_base"):
        setattr(s, k, int(m[k]))
    for i in range(8):
        s.rtab[i] = int(m["rtab"][i]) if i < len(m["rtab"]) else 0
        s.stab[i] = int(m["stab"][i]) if i < len(m["stab"]) else 0
    return s


# ------------------------------------------------------------------ conv engine

def pack_weight(w, m, split=None):
    """Packed weight for the conv engine: fp32 [n][kh*jp], or (split, the default under the
    bf16x6 forward math) the pre-split bf16 h/m/l layout of fg_pack_weight_split, returned as a
    bfloat16 tensor (conv problems built on it carry w_split = 1)."""
    L.require_device(w, "weight")
    w = w.contiguous()
    s = wmap_struct(m)
    if split is None:
        split = L.fwd_x6()
    if split:
        wp = torch.empty(3 * packed_numel(m), dtype=torch.bfloat16, device=w.device)
        L.check(_lib().fg_pack_weight_split(L.ptr(w), C.byref(s), L.ptr(wp), L.stream_handle()), "pack_weight_split")
        return wp
    wp = torch.empty(packed_numel(m), dtype=torch.float32, device=w.device)
    L.check(_lib().fg_pack_weight(L.ptr(w), C.byref(s), L.ptr(wp), L.stream_handle()), "pack_weight")
    return wp


_CONV_FIELDS = ("sxn", "sxa", "sxb", "sxr", "syn", "sya", "syb", "syc", "m_img", "m_a", "m_b", "kh", "j_valid",
                "jp", "n_out", "ldw", "act", "accumulate")


class KernelTimer:
    """HIP-event timing of tagged launches on the current stream (used by bench.py to time the
    dominant kernel live inside the timed region)."""

    def __init__(self, tags):
        self.tags = set(tags)
        self.events = {t: [] for t in tags}

    def __enter__(self):
        global _TIMER
        self._prev, _TIMER = _TIMER, self
        return self

    def __exit__(self, *exc):
        global _TIMER
        _TIMER = self._prev

    def durations_ms(self):
        torch.cuda.synchronize()
        return {t: [s.elapsed_time(e) for s, e in ev] for t, ev in self.events.items()}


_TIMER = None


def conv(probs, tag=None):
    """Launch 1-4 fg_conv_problem dicts (plans.conv_problem / phase_problems) in one kernel."""
    if _TIMER is not None and tag in _TIMER.tags:
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        _conv(probs)
        e.record()
        _TIMER.events[tag].append((s, e))
    else:
        _conv(probs)


def _conv(probs):
    arr = (L.fg_conv_problem * len(probs))()
    for i, p in enumerate(probs):
        s = arr[i]
        s.x, s.w, s.y = _addr(p["x"]), _addr(p["w"]), _addr(p["y"])
        s.w_split = int(p["w"][0].dtype == torch.bfloat16)
        s.bias = p["bias"].data_ptr() if p["bias"] is not None else None
        for k in _CONV_FIELDS:
            setattr(s, k, int(p[k]))
    L.check(_lib().fg_conv_fwd(arr, len(probs), L.stream_handle()), "conv_fwd")


_WG_FIELDS = ("spn", "spa", "spb", "sxn", "sxa", "sxb", "sxr", "m_img", "m_a", "m_b", "n_a", "kh", "j_valid",
              "splits", "m_chunk")


def wgrad(prob, wmap, dw, accumulate=False):
    """weight gradient into the PyTorch-layout tensor dw (overwritten, or += if accumulate)"""
    dev = _dev(prob["p"][0])
    slab = torch.empty(slab_numel(prob), dtype=torch.float32, device=dev)
    s = L.fg_wgrad_problem()
    s.p, s.x, s.out = _addr(prob["p"]), _addr(prob["x"]), slab.data_ptr()
    for k in _WG_FIELDS:
        setattr(s, k, int(prob[k]))
    st = L.stream_handle()
    L.check(_lib().fg_conv_wgrad(C.byref(s), st), "conv_wgrad")
    m = wmap_struct(wmap)
    L.check(_lib().fg_wgrad_reduce(L.ptr(slab), int(prob["splits"]), C.byref(m), L.ptr(dw), int(accumulate), st),
            "wgrad_reduce")


# ------------------------------------------------------------------ layout

def pack_input(a, ca, b, cb, dst, img0, nimg, pad_mode):
    L.check(_lib().fg_pack_input(sview(a), ca, sview(b), cb, view(dst), img0, nimg, pad_mode, L.stream_handle()),
            "pack_input")


def zero_border(B):
    L.check(_lib().fg_zero_border(view(B), L.stream_handle()), "zero_border")


def fold_add(gpad, fold_pad, add, dst):
    L.check(_lib().fg_fold_add(view(gpad), fold_pad, view(add), view(dst), L.stream_handle()), "fold_add")


# ------------------------------------------------------------------ instance norm

def _work(n, c, dev):
    return torch.empty(int(_lib().fg_in_workspace_doubles(n, c)), dtype=torch.float64, device=dev)


def in_stats(src):
    dev = src.t.device
    mean = torch.empty(src.n * src.c, dtype=torch.float32, device=dev)
    rstd = torch.empty_like(mean)
    L.check(_lib().fg_in_stats(view(src), C.c_float(EPS), L.ptr(mean), L.ptr(rstd), L.ptr(_work(src.n, src.c, dev)),
                               L.stream_handle()), "in_stats")
    return mean, rstd


def in_apply(src, mean, rstd, act, residual, dst, pad_mode):
    L.check(_lib().fg_in_apply(view(src), L.ptr(mean), L.ptr(rstd), act, view(residual), view(dst), pad_mode,
                               L.stream_handle()), "in_apply")


def in_bwd(gsrc, fold_pad, gadd, src, mean, rstd, act, dst, bias_grad=None):
    L.check(_lib().fg_in_bwd(view(gsrc), fold_pad, view(gadd), view(src), L.ptr(mean), L.ptr(rstd), act, view(dst),
                             L.ptr(bias_grad), L.ptr(_work(src.n, src.c, src.t.device)), L.stream_handle()),
            "in_bwd")


def act_bwd(g, y, act):
    L.check(_lib().fg_act_bwd(view(g), view(y), act, L.stream_handle()), "act_bwd")


def channel_sum(src, c_valid, out, accumulate=False):
    work = torch.empty(256 * c_valid + 64, dtype=torch.float64, device=src.t.device)
    L.check(_lib().fg_channel_sum(view(src), c_valid, L.ptr(out), int(accumulate), L.ptr(work), L.stream_handle()),
            "channel_sum")


# ------------------------------------------------------------------ tail / losses / adam

def tail_fwd(cl, al, x, out, mask):
    L.check(_lib().fg_tail_fwd(view(cl), view(al), sview(x), L.ptr(out), L.ptr(mask), L.stream_handle()), "tail_fwd")


def tail_bwd(cl, al, x, g_out, gc, ga):
    L.check(_lib().fg_tail_bwd(view(cl), view(al), sview(x), sview(g_out), view(gc), view(ga), L.stream_handle()),
            "tail_bwd")


def mse_const(p, target, gscale, loss_out, g=None):
    """loss_out[0] = mean((p - target)^2); g = gscale * dL/dp (optional)"""
    work = torch.empty(1024, dtype=torch.float64, device=p.device)
    L.check(_lib().fg_mse_const(L.ptr(p), p.numel(), C.c_float(target), C.c_float(gscale), L.ptr(loss_out),
                                L.ptr(g), L.ptr(work), L.stream_handle()), "mse")


def l1(a, b, gscale, loss_out, g=None, accumulate=False):
    """loss_out[0] = mean|a - b| over [N,C,H,W]; g (contiguous NCHW) = gscale * dL/da"""
    N, Cc, H, W = a.shape
    work = torch.empty(1024, dtype=torch.float64, device=a.device)
    L.check(_lib().fg_l1(sview(a), sview(b), N, Cc, H, W, C.c_float(gscale), L.ptr(loss_out), L.ptr(g),
                         int(accumulate), L.ptr(work), L.stream_handle()), "l1")


def adam_step(entries, lr, beta1, beta2, eps, step):
    """entries: list of (param, grad, exp_avg, exp_avg_sq) tensors sharing `step`"""
    if not entries:
        return
    arr = (L.fg_adam_tensor * len(entries))()
    for i, (p, g, m, v) in enumerate(entries):
        arr[i].param, arr[i].grad, arr[i].exp_avg, arr[i].exp_avg_sq = (
            p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr())
        arr[i].numel = p.numel()
    L.check(_lib().fg_adam_step(arr, len(entries), float(lr), float(beta1), float(beta2), float(eps), int(step),
                                L.stream_handle()), "adam_step")
