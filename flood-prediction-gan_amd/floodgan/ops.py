"""Thin device-op layer: turns plans / buffers into C-ABI calls on the current HIP stream.

Every function here launches HIP kernels from libfloodgan.so; nothing falls back to ATen.
"""
import ctypes as C
import os

import torch

from . import _lib as L
from .plans import Buf, Slice, f3_wgrad_eligible, packed_numel, slab_numel, stem_wgrad_layout, wgrad_splits

EPS = 1e-5


def _lib():
    return L.load()


def _dev(t):
    return t.t.device if isinstance(t, (Buf, Slice)) else t.device


def _addr(ref):
    """(Buf|tensor, element offset) -> device address"""
    obj, off = ref
    t = obj.t if isinstance(obj, Buf) else obj
    return t.data_ptr() + 4 * off


def view(B):
    if B is None:
        return L.fg_view(None, 0, 0, 0, 0, 0)
    if isinstance(B, Slice):
        b = B.buf
        return L.fg_view(b.t.data_ptr() + 4 * B.c0, b.n, b.h, b.w, b.c, b.pad)
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
    s.q_n = int(m.get("q_n", 0))
    return s


# ------------------------------------------------------------------ conv engine

# ------------------------------------------------------------------ f16x3 operand scales
#
# The f16x3 conv math scales each operand by a power of two derived from a device scalar >=
# max |operand|.  Those scalars live in slots of a zero-initialised pool (one fill per 4096
# slots).  Producers that already touch every element (IN apply / backward) raise their
# output's slot for free; otherwise the conv computes one with fg_absmax.  The slot is cached
# on the tensor object and dropped by every op that writes that tensor (a stale slot is only
# safe while it still bounds the contents).


SHARDS = 64     # FG_AMAX_SHARDS: floats per absmax slot


class _SlotPool:
    SIZE = 4096     # slots per zero-filled pool

    def __init__(self):
        self.t, self.i = None, 0

    def take(self, device):
        if self.t is None or self.i >= self.SIZE or self.t.device != torch.device(device):
            self.t, self.i = torch.zeros(self.SIZE * SHARDS, dtype=torch.float32, device=device), 0
        self.i += 1
        return self.t[(self.i - 1) * SHARDS:self.i * SHARDS]


_SLOTS = _SlotPool()


def _tensor(obj):
    return obj.t if isinstance(obj, (Buf, Slice)) else obj


def _wrote(*objs):
    """an op wrote these buffers: forget their cached absmax slots, split copies and pre-split format"""
    for o in objs:
        if o is not None:
            t = _tensor(o)
            if getattr(t, "_fg_amax", None) is not None:
                t._fg_amax = None
            if getattr(t, "_fg_split", None) is not None:
                t._fg_split = None
            if getattr(t, "_fg_presplit", False):
                t._fg_presplit = False
            if getattr(t, "_fg_splitpix", False):
                t._fg_splitpix = False


# Pre-split operands (FG_PRESPLIT, include/floodgan.h): the norm passes that feed a resblock conv write its
# operand as the fp16 (h, l) pieces the f16x3 kernels would otherwise split on the fly (FLOODGAN_PRESPLIT=0:
# off).  The format is recorded on the tensor with its version counter: only the pipelined kernels read it.
PRESPLIT = os.environ.get("FLOODGAN_PRESPLIT", "1") != "0"


# the resblock chain's block inputs / outputs also get a pre-split copy beside the fp32 residual stream
# (fg_in_apply_dual; FLOODGAN_PRESPLIT_RESID=0: off)
PRESPLIT_RESID = os.environ.get("FLOODGAN_PRESPLIT_RESID", "1") != "0"


def presplit_on():
    return PRESPLIT and L.fwd_f16x3() and L.wgrad_f16x3() and L.wgrad_f3_on()


# Only the pipelined kernels read FG_PRESPLIT operands, and they address their outputs with 31-bit byte offsets
# (conv_f3.hip f3_takes): a consumer of a larger operand would produce an output the kernel declines.  Producers
# therefore write a buffer beyond this size in fp32 (every kernel reads that) -- at bs 8, 512^2 the largest
# pre-split buffer (64 channels at 512^2) is 0.55 GB.  The other geometry the pipelined kernels need (packed row
# run jp % 32 == 0, channel groups of 8, more than 32 output channels -- conv_f3.hip f3_takes / presplit_ok) holds
# at every producer call site for any batch size and resolution: each pre-split buffer has 64..512 channels and
# feeds only 3x3 / 4x4 convs and weight gradients with 64..512 outputs.  A consumer that still declines a pre-split
# operand fails with FG_ERR_INVALID (it never reads it as fp32).
PRESPLIT_MAX_BYTES = (1 << 31) - (1 << 24)


def presplit_fits(buf):
    return buf is not None and 4 * _tensor(buf).numel() <= PRESPLIT_MAX_BYTES


def is_presplit(obj):
    t = _tensor(obj)
    if not getattr(t, "_fg_presplit", False):
        return False
    if getattr(t, "_fg_presplit_ver", None) != t._version:
        raise RuntimeError("a pre-split (FG_PRESPLIT) buffer was written by torch since its producer ran")
    return True


def is_splitpix(obj):
    """the buffer holds the fg_split_pixels layout written by its producer (in_apply(splitpix=True)), not fp32"""
    t = _tensor(obj)
    if not getattr(t, "_fg_splitpix", False):
        return False
    if getattr(t, "_fg_splitpix_ver", None) != t._version:
        raise RuntimeError("a split-pixels buffer was written by torch since its producer ran")
    return True


def _mark_presplit(dst):
    t = _tensor(dst)
    t._fg_presplit, t._fg_presplit_ver = True, t._version


# Self-checking scale caches (FLOODGAN_CHECK_SCALES=1, a debug mode: one device reduction and a host sync per
# operand).  Before every f16x3 launch the operands are re-measured and the launch is refused unless the absmax
# slot it will derive its power-of-two scale from still bounds them: fp32 operands max |v| <= slot; pre-split
# operands |h| <= 2^14 (the producer split v * s with s = 2^(14-e) from the same slot, so a slot that no longer
# bounds v shows as an h piece beyond 2^14, inf or NaN); cached weight packs and window-kernel split copies are
# rebuilt and compared bit for bit with the cached ones.  SCALE_CHECKS counts the checks per kind.
CHECK_SCALES = os.environ.get("FLOODGAN_CHECK_SCALES", "0") != "0"
SCALE_CHECKS = {}


def _count_check(kind):
    SCALE_CHECKS[kind] = SCALE_CHECKS.get(kind, 0) + 1


def _region(obj):
    """what a gather can read: the padded extent of a Buf (a Slice's whole buffer), else the tensor"""
    if isinstance(obj, Slice):
        obj = obj.buf
    return obj.nhwc() if isinstance(obj, Buf) else obj


def check_scale(obj, slot, what):
    """FLOODGAN_CHECK_SCALES: raise unless `slot` (the absmax slot a launch scales obj by) bounds obj"""
    reg = _region(obj)
    if is_presplit(obj):
        pieces = reg.reshape(-1, 8).view(torch.float16).view(-1, 2, 8)[:, 0]
        worst = float(pieces.abs().float().max()) if pieces.numel() else 0.0
        ok = worst <= 2.0 ** 14
        kind = "presplit"
    else:
        worst = float(reg.abs().max()) if reg.numel() else 0.0
        bound = float(slot.max())
        ok = worst <= bound
        kind = "fp32"
    if not ok:
        raise RuntimeError(f"FLOODGAN_CHECK_SCALES: the {kind} operand '{what}' is not bounded by its cached scale "
                           f"slot (max {worst!r}" + (f" > slot {bound!r})" if kind == "fp32" else " > 2^14 in h)"))
    _count_check(kind)


def absmax(t):
    """Device scalar >= max |t| (the f16x3 operand-scale source), over the whole storage of a
    tensor or of a Buf (border and padding channels included: everything a gather can read);
    cached on the tensor until an op writes it."""
    t = _tensor(t)
    if getattr(t, "_fg_splitpix", False) and getattr(t, "_fg_splitpix_ver", None) == t._version:
        raise RuntimeError("absmax of a split-pixels buffer (it holds fp16 pieces, read only by the window kernels)")
    if getattr(t, "_fg_presplit", False) and getattr(t, "_fg_presplit_ver", None) == t._version:
        # the producer's scale slot is the only valid scale source of a pre-split buffer
        if getattr(t, "_fg_amax", None) is None or getattr(t, "_fg_amax_ver", None) != t._version:
            raise RuntimeError("pre-split buffer without its producer's scale slot")
        return t._fg_amax
    cached = getattr(t, "_fg_amax", None)
    # a slot is valid only together with the version counter it was recorded at: an in-place torch
    # write since then (or a slot recorded without a version) means it may no longer bound t
    if cached is not None and getattr(t, "_fg_amax_ver", None) == t._version:
        return cached
    out = _SLOTS.take(t.device)
    L.check(_lib().fg_absmax(L.ptr(t), t.numel(), L.ptr(out), L.stream_handle()), "absmax")
    t._fg_amax, t._fg_amax_ver = out, t._version
    return out


def _amax_out(dst):
    """slot for a producer to raise to max |dst| (f16x3 only), recorded on dst"""
    _wrote(dst)
    if not L.fwd_f16x3() and not L.wgrad_f16x3():
        return None
    slot = _SLOTS.take(_dev(dst))
    t = _tensor(dst)
    # the kernel writes through a raw pointer (torch's counter does not move): record the version
    # now, so a later in-place torch write invalidates the slot
    t._fg_amax, t._fg_amax_ver = slot, t._version
    return slot


def _weight_absmax(w):
    """absmax slot of a parameter: the one FusedAdam's kernel raised with the last update while the
    tensor's version counter shows no torch write since, else a fresh fg_absmax pass (recorded
    with the version so the other packs of the same weights reuse it)"""
    slot = getattr(w, "_fg_amax", None)
    if slot is not None and getattr(w, "_fg_amax_ver", None) == w._version:
        return slot
    slot = _SLOTS.take(w.device)
    L.check(_lib().fg_absmax(L.ptr(w), w.numel(), L.ptr(slot), L.stream_handle()), "absmax")
    w._fg_amax, w._fg_amax_ver = slot, w._version
    return slot


# Pack cache (f16x3): each parameter keeps its packed layouts (one per weight map) with the absmax slot
# they were scaled by; a pack is current while that slot is the parameter's current one (a torch write
# moves the version counter, an adam_step installs a new slot AND re-packs every cached layout of the
# parameters it updated in batched launches), so a training step packs nothing itself.
# FLOODGAN_PACK_CACHE=0: pack at every use.
PACK_CACHE = os.environ.get("FLOODGAN_PACK_CACHE", "1") != "0"


def _repack(params):
    """re-pack every cached f16x3 layout of `params` with their current absmax slots (after an update)"""
    jobs = []
    for p in params:
        packs = p.__dict__.get("_fg_packs")
        if not packs:
            continue
        slot = _weight_absmax(p)
        for wp in packs.values():
            j = L.fg_pack_job()
            j.w, j.w_absmax, j.dst, j.map = p.data_ptr(), slot.data_ptr(), wp.data_ptr(), wp._fg_map
            jobs.append(j)
            wp.absmax = slot
    for i in range(0, len(jobs), L.FG_PACK_BATCH_MAX):
        part = jobs[i:i + L.FG_PACK_BATCH_MAX]
        arr = (L.fg_pack_job * len(part))(*part)
        L.check(_lib().fg_pack_weight_f16_batch(arr, len(part), L.stream_handle()), "pack_weight_f16_batch")


def pack_weight(w, m, split=None):
    """Packed weight for the conv engine: fp32 [n][kh*jp]; or, by default under a split forward
    math, the pre-split layout -- bf16 h/m/l pieces (bf16x6, fg_pack_weight_split) or scaled fp16
    h/l pieces (f16x3, fg_pack_weight_f16; the tensor carries its scale source as `.absmax`).
    Conv problems built on it carry w_split = 1 or 2 accordingly."""
    L.require_device(w, "weight")
    w = w.contiguous()
    s = wmap_struct(m)
    if split is None:
        split = "f16x3" if L.fwd_f16x3() else ("bf16x6" if L.fwd_x6() else None)
    elif split is True:
        split = "f16x3" if L.fwd_f16x3() else "bf16x6"
    if split == "f16x3":
        amax = _weight_absmax(w)
        packs = w.__dict__.setdefault("_fg_packs", {}) if PACK_CACHE else None
        key = bytes(s)
        if packs is not None and key in packs and packs[key].absmax is amax:
            if CHECK_SCALES:
                _check_pack(w, s, amax, packs[key])
            return packs[key]          # packed from the current values (re-packed by the last adam_step)
        if CHECK_SCALES:
            check_scale(w, amax, "weight")
        wp = torch.empty(2 * packed_numel(m), dtype=torch.float16, device=w.device)
        L.check(_lib().fg_pack_weight_f16(L.ptr(w), C.byref(s), L.ptr(amax), L.ptr(wp), L.stream_handle()),
                "pack_weight_f16")
        wp.absmax = amax
        if packs is not None:
            wp._fg_map = s
            packs[key] = wp
        return wp
    if split == "bf16x6":
        wp = torch.empty(3 * packed_numel(m), dtype=torch.bfloat16, device=w.device)
        L.check(_lib().fg_pack_weight_split(L.ptr(w), C.byref(s), L.ptr(wp), L.stream_handle()), "pack_weight_split")
        return wp
    wp = torch.empty(packed_numel(m), dtype=torch.float32, device=w.device)
    L.check(_lib().fg_pack_weight(L.ptr(w), C.byref(s), L.ptr(wp), L.stream_handle()), "pack_weight")
    return wp


def _check_pack(w, s, amax, cached):
    """FLOODGAN_CHECK_SCALES: a cached f16x3 pack must equal a fresh pack of the current weights by a slot
    that bounds them"""
    check_scale(w, amax, "weight")
    fresh = torch.empty_like(cached)
    L.check(_lib().fg_pack_weight_f16(L.ptr(w), C.byref(s), L.ptr(amax), L.ptr(fresh), L.stream_handle()),
            "pack_weight_f16")
    if not torch.equal(fresh.view(torch.int16), cached.view(torch.int16)):
        raise RuntimeError("FLOODGAN_CHECK_SCALES: a cached weight pack differs from a fresh pack of the weights")
    _count_check("pack")


_CONV_FIELDS = ("sxn", "sxa", "sxb", "sxr", "syn", "sya", "syb", "syc", "m_img", "m_a", "m_b", "kh", "j_valid",
                "jp", "n_out", "ldw", "act", "accumulate")


TIMER_EVENTS = {"system": 0, "device": 1, "none": 2, "dispatch": 2}


class KernelTimer:
    """HIP-event timing of tagged launches on the current stream (used by bench.py to time the
    dominant kernel live inside the timed region).

    events: "dispatch" (default) attaches the start / stop events to the timed kernel's own dispatch packet
    (fg_timing_arm -> hipExtLaunchKernel: the pipelined conv / weight-gradient launch of the tagged call), so the
    stream carries no extra packet.  "system" / "device" / "none" record marker events around the tagged call with
    that release scope; "system" is torch.cuda.Event's: every record writes back and invalidates L2, ~6 us per
    event at the step's kernel boundaries, which the timed step then carries (profiles/round6/r6k_*)."""

    def __init__(self, tags, events="dispatch"):
        self.tags = set(tags)
        self.dispatch = events == "dispatch"
        self.mode = TIMER_EVENTS[events]
        self.events = {t: [] for t in tags}

    def __enter__(self):
        global _TIMER
        self._prev, _TIMER = _TIMER, self
        return self

    def __exit__(self, *exc):
        global _TIMER
        _TIMER = self._prev

    def _event(self):
        ev = C.c_void_p()
        L.check(_lib().fg_timing_event_create(self.mode, C.byref(ev)), "timing_event_create")
        return ev

    def record_pair(self, tag, fn):
        s, e = self._event(), self._event()
        if self.dispatch:
            L.check(_lib().fg_timing_arm(s, e), "timing_arm")
            try:
                out = fn()
            finally:
                pending = _lib().fg_timing_disarm()
            if pending:
                raise RuntimeError(f"KernelTimer: the call tagged {tag} launched no timed kernel")
        else:
            st = L.stream_handle()
            L.check(_lib().fg_timing_event_record(s, st), "timing_event_record")
            out = fn()
            L.check(_lib().fg_timing_event_record(e, st), "timing_event_record")
        self.events[tag].append((s, e))
        return out

    def durations_ms(self):
        """waits for the recorded launches; returns {tag: [ms per launch]} and releases the events"""
        out = {}
        ms = C.c_float()
        for t, ev in self.events.items():
            out[t] = []
            for s, e in ev:
                L.check(_lib().fg_timing_event_elapsed(s, e, C.byref(ms)), "timing_event_elapsed")
                out[t].append(ms.value)
                L.check(_lib().fg_timing_event_destroy(s), "timing_event_destroy")
                L.check(_lib().fg_timing_event_destroy(e), "timing_event_destroy")
        self.events = {t: [] for t in self.tags}
        return out


_TIMER = None


def _timed(tag, fn):
    """run fn (one launch on the current stream), bracketed by HIP events when the active KernelTimer
    collects `tag`"""
    if _TIMER is None or tag not in _TIMER.tags:
        return fn()
    return _TIMER.record_pair(tag, fn)


USE_WIN = True   # route eligible single convs to the row-strip kernel (fg_conv_win)


# InstanceNorm statistics from the pipelined kernel's epilogue where it runs (FLOODGAN_FUSED_IN_STATS=0: off)
FUSED_IN_STATS = os.environ.get("FLOODGAN_FUSED_IN_STATS", "1") != "0"


LAST_CONV_KERNEL = None    # the kernel family the last conv() launch ran (fg_last_launch; tests)


def conv(probs, tag=None, in_stats=False):
    """Launch 1-4 fg_conv_problem dicts (plans.conv_problem / phase_problems) in one kernel
    (the row-strip window kernel for a lone eligible 7x7 conv, see win_eligible).  in_stats=True:
    the problems all write one output Buf (the 4 phases of a transposed conv, or a single conv) that an
    InstanceNorm reads next; when the pipelined kernel takes them, its epilogue also emits the norm's
    statistics partials and conv returns (mean, rstd) per (image, channel), else None."""
    if USE_WIN and len(probs) == 1 and win_eligible(probs[0]):
        return conv_win(probs[0], tag)
    stats = _conv(probs, in_stats, tag)
    return None if stats is None else _merge_stats(*stats)


def _conv(probs, in_stats=False, tag=None):
    arr = (L.fg_conv_problem * len(probs))()
    f16 = L.fwd_f16x3()
    keep = {}
    for i, p in enumerate(probs):
        s = arr[i]
        s.x, s.w, s.y = _addr(p["x"]), _addr(p["w"]), _addr(p["y"])
        wt = p["w"][0]
        s.w_split = {torch.bfloat16: 1, torch.float16: 2}.get(wt.dtype, 0)
        s.bias = p["bias"].data_ptr() if p["bias"] is not None else None
        for k in _CONV_FIELDS:
            setattr(s, k, int(p[k]))
        s.jc = getattr(p["x"][0], "c", 0)
        s.x_presplit = int(is_presplit(p["x"][0]))
        if p.get("q_n"):
            s.q_n, s.q_mask = int(p["q_n"]), int(p["q_mask"])
            for q in range(4):
                s.q_yoff[q] = int(p["q_yoff"][q])
        if f16:
            xb = p["x"][0]
            if id(xb) not in keep:
                keep[id(xb)] = absmax(xb)
            s.x_absmax = keep[id(xb)].data_ptr()
            if CHECK_SCALES:
                check_scale(xb, keep[id(xb)], "conv input")
            wa = getattr(wt, "absmax", None)
            if wa is None:              # fp32 weights split on the fly: scale from their own max
                if ("w", id(wt)) not in keep:
                    keep[("w", id(wt))] = _SLOTS.take(wt.device)
                    L.check(_lib().fg_absmax(L.ptr(wt), wt.numel(), L.ptr(keep[("w", id(wt))]),
                                             L.stream_handle()), "absmax")
                wa = keep[("w", id(wt))]
            s.w_absmax = wa.data_ptr()
            if CHECK_SCALES and wt.dtype == torch.float32:
                check_scale(wt, wa, "fp32 weight")
    stats = _stats_partials(probs, arr) if (in_stats and FUSED_IN_STATS) else None
    _timed(tag, lambda: L.check(_lib().fg_conv_fwd(arr, len(probs), L.stream_handle()), "conv_fwd"))
    global LAST_CONV_KERNEL
    LAST_CONV_KERNEL = L.last_launch()
    _wrote(*[p["y"][0] for p in probs])
    return stats


def _merge_stats(nprob, buf, n_img, rb, c):
    """(mean, rstd) per (image, channel) from the epilogue partials of one conv launch"""
    mean = torch.empty(n_img * c, dtype=torch.float32, device=buf.device)
    rstd = torch.empty_like(mean)
    work = torch.empty(int(_lib().fg_in_partials_workspace_doubles(n_img, c)), dtype=torch.float64,
                       device=buf.device)
    L.check(_lib().fg_in_stats_partials(L.ptr(buf), nprob, n_img, rb, c, C.c_float(EPS), L.ptr(mean),
                                        L.ptr(rstd), L.ptr(work), L.stream_handle()), "in_stats_partials")
    return mean, rstd


def _stats_partials(probs, arr):
    """attach epilogue-statistics buffers to the problem structs when the pipelined kernel takes them:
    (regions, buffer, images, 32-row blocks per image and region, channels) or None -- one region per problem, or
    per column group of a quad-form problem"""
    Y = probs[0]["y"][0]
    if not isinstance(Y, Buf) or any(p["y"][0] is not Y for p in probs):
        return None
    if probs[0].get("q_n"):           # the quad form: one region per column group (= phase), merged like 4 problems
        p, ng, c = probs[0], probs[0]["n_out"] // probs[0]["q_n"], probs[0]["q_n"]
        if c != Y.c or (p["m_a"] * p["m_b"]) % 32 or not _lib().fg_conv_stats_ok(arr, 1):
            return None
        rb = p["m_a"] * p["m_b"] // 32
        buf = torch.empty(ng * Y.n * rb * c * 2, dtype=torch.float32, device=Y.t.device)
        arr[0].in_stats = buf.data_ptr()
        arr[0].q_soff = Y.n * rb * c * 2
        return ng, buf, Y.n, rb, c
    rows = {p["m_a"] * p["m_b"] for p in probs}
    c = probs[0]["n_out"]
    if len(rows) != 1 or c != Y.c or any(p["n_out"] != c or p["m_img"] != Y.n for p in probs):
        return None
    r = rows.pop()
    if r % 32 or not _lib().fg_conv_stats_ok(arr, len(probs)):
        return None
    rb = r // 32
    buf = torch.empty(len(probs) * Y.n * rb * c * 2, dtype=torch.float32, device=Y.t.device)
    for i in range(len(probs)):
        arr[i].in_stats = buf.data_ptr() + 4 * i * Y.n * rb * c * 2
    return len(probs), buf, Y.n, rb, c


def split_pixels(X):
    """fg_split_pixels copy of a Buf (32 or 64 channels): fp16 h/l pieces of the scaled values,
    the window-conv operand.  Cached on the buffer's tensor until an op writes it."""
    t = X.t
    if is_presplit(X):
        raise RuntimeError("split_pixels of a pre-split buffer")
    if is_splitpix(X):
        return t._fg_split              # the producer wrote the split layout itself (in_apply(splitpix=True))
    cached = getattr(t, "_fg_split", None)
    if cached is not None and getattr(t, "_fg_split_ver", None) == t._version:
        if CHECK_SCALES:
            check_scale(X, cached.absmax, "split-copy source")
            if cached.absmax is not absmax(t):
                raise RuntimeError("FLOODGAN_CHECK_SCALES: a cached split copy was scaled by another slot")
            fresh = torch.empty_like(cached)
            L.check(_lib().fg_split_pixels(L.ptr(t), X.n * X.hp * X.wp, X.c, X.wp, L.ptr(cached.absmax), L.ptr(fresh),
                                           L.stream_handle()), "split_pixels")
            if not torch.equal(fresh.view(torch.int16), cached.view(torch.int16)):
                raise RuntimeError("FLOODGAN_CHECK_SCALES: a cached split copy differs from its source")
            _count_check("split_copy")
        return cached
    npix = X.n * X.hp * X.wp
    out = torch.empty(npix * 2 * X.c, dtype=torch.float16, device=t.device)
    if CHECK_SCALES:
        check_scale(X, absmax(t), "split-copy source")
    L.check(_lib().fg_split_pixels(L.ptr(t), npix, X.c, X.wp, L.ptr(absmax(t)), L.ptr(out), L.stream_handle()),
            "split_pixels")
    out.absmax = absmax(t)
    t._fg_split, t._fg_split_ver = out, t._version
    return out


def win_eligible(prob):
    """True when fg_conv_win takes this conv (stride-1 7x7 over a 32/64-channel Buf whose full
    border is the conv's padding, n_out within one 32/64-column tile, output rows >= 256 px)"""
    X, off = prob["x"]
    if not L.fwd_f16x3() or not isinstance(X, Buf) or X.c not in (32, 64):
        return False
    # C = 32 is the content head's input gradient (27(32) -> 64): its split copy is the one the content
    # weight gradient already made, and the strip form beats the pipelined kernel's per-tap re-gather
    # (1.58 vs 1.67 ms at bs 8, profiles/round2/r2v_content_dgrad_win.log)
    return (prob["kh"] == 7 and prob["j_valid"] == 7 * X.c and prob["jp"] == prob["j_valid"]
            and prob["sxb"] == X.c and prob["sxa"] == prob["sxr"] == X.s_row and off == 0
            and prob["n_out"] <= (32 if X.c == 64 else 64) and prob["m_b"] >= 256
            and prob["w"][0].dtype == torch.float16)


def conv_win(prob, tag=None):
    """The row-strip window conv (fg_conv_win) of one plans.conv_problem."""
    X, off = prob["x"]
    xs = split_pixels(X)
    arr = (L.fg_conv_problem * 1)()
    s = arr[0]
    s.x, s.w, s.y = _addr(prob["x"]), _addr(prob["w"]), _addr(prob["y"])
    s.w_split = 2
    s.bias = prob["bias"].data_ptr() if prob["bias"] is not None else None
    for k in _CONV_FIELDS:
        setattr(s, k, int(prob[k]))
    s.x_absmax = xs.absmax.data_ptr()
    s.w_absmax = prob["w"][0].absmax.data_ptr()

    _timed(tag, lambda: L.check(_lib().fg_conv_win(arr, L.ptr(xs), off // X.c, L.stream_handle()), "conv_win"))
    _wrote(prob["y"][0])


WIN_WGRAD_SPLITS = 216   # x 7 kernel rows = 1512 workgroups of 4 waves (several resident per CU); a multiple of 8:
#                          the 7 workgroups of a split then share an XCD (conv_wgrad_win.hip).  bs 8, 512^2:
#                          72 / 144 / 216 / 288 splits 1218 / 1290 / 1065 / 1085 us (profiles/round3/r3ar_*)


def wgrad_win_eligible(prob):
    """the content-head weight gradient fg_conv_wgrad_win takes: 7x7 over a 64-channel Buf gathered
    from a padded-row start, gradient a 32-channel Buf, n_a <= 32, output rows a multiple of 32 px"""
    P, poff = prob["p"]
    X, xoff = prob["x"]
    return (isinstance(P, Buf) and isinstance(X, Buf) and P.c == 32 and X.c == 64 and prob["kh"] == 7
            and prob["j_valid"] == 7 * 64 and prob["sxb"] == 64 and prob["sxa"] == prob["sxr"] == X.s_row
            and prob["spb"] == 32 and prob["spa"] == P.s_row and prob["n_a"] <= 32 and prob["m_b"] % 32 == 0
            and (xoff // X.c) % X.wp == 0 and xoff % X.c == 0 and poff % P.c == 0)


def _wgrad_win(prob, wmap, dw, accumulate):
    P, poff = prob["p"]
    X, xoff = prob["x"]
    ps, xs = split_pixels(P), split_pixels(X)
    prob = dict(prob, splits=WIN_WGRAD_SPLITS, m_chunk=1)
    slab = torch.empty(slab_numel(prob), dtype=torch.float32, device=P.t.device)
    s = L.fg_wgrad_problem()
    s.p, s.x, s.out = _addr(prob["p"]), _addr(prob["x"]), slab.data_ptr()
    for k in _WG_FIELDS:
        setattr(s, k, int(prob[k]))
    s.p_absmax, s.x_absmax = ps.absmax.data_ptr(), xs.absmax.data_ptr()
    st = L.stream_handle()
    p_pix0 = poff // P.c
    L.check(_lib().fg_conv_wgrad_win(C.byref(s), L.ptr(ps), p_pix0, p_pix0 % P.wp, P.wp, L.ptr(xs), xoff // X.c,
                                     X.wp, st), "conv_wgrad_win")
    m = wmap_struct(wmap)
    L.check(_lib().fg_wgrad_reduce(L.ptr(slab), int(prob["splits"]), C.byref(m), L.ptr(dw), int(accumulate), st),
            "wgrad_reduce")


LAST_WGRAD_KERNEL = None   # the kernel family the last wgrad() launch ran (fg_last_launch; tests)

_WG_FIELDS = ("spn", "spa", "spb", "sxn", "sxa", "sxb", "sxr", "m_img", "m_a", "m_b", "n_a", "kh", "j_valid",
              "splits", "m_chunk")


def prepare_wgrad(prob):
    """fill the operand caches a wgrad(prob) launch reads (f16x3 scale slots; the window kernel's split
    copies) on the current stream, ahead of running wgrad on another stream"""
    if not L.wgrad_f16x3():
        return
    if USE_WIN and wgrad_win_eligible(prob):
        split_pixels(prob["p"][0])
        split_pixels(prob["x"][0])
    else:
        absmax(prob["p"][0])
        absmax(prob["x"][0])


def wgrad(prob, wmap, dw, accumulate=False, tag=None):
    """weight gradient into the PyTorch-layout tensor dw (overwritten, or += if accumulate); `tag` times the
    weight-gradient launch itself (not the split reduction) under a KernelTimer"""
    dev = _dev(prob["p"][0])
    if USE_WIN and L.wgrad_f16x3() and wgrad_win_eligible(prob):
        return _wgrad_win(prob, wmap, dw, accumulate)
    stem = stem_wgrad_layout(prob) if L.wgrad_f16x3() else None
    if stem is not None and not (is_presplit(prob["p"][0]) or is_presplit(prob["x"][0])):
        # the stem's strip kernel (conv_stem.hip) defines its own splits: 64-px strips of m_chunk / 64 rows
        prob = dict(prob, splits=stem[0], m_chunk=stem[1])
    elif L.wgrad_f16x3() and L.wgrad_f3_on() and f3_wgrad_eligible(prob):
        # re-split the pixel range for the pipelined kernel's tiles (one workgroup per CU)
        splits, chunk = wgrad_splits(prob["n_a"], prob["kh"] * prob["j_valid"],
                                     prob["m_img"] * prob["m_a"] * prob["m_b"], f3=True)
        prob = dict(prob, splits=splits, m_chunk=chunk)
    slab = torch.empty(slab_numel(prob), dtype=torch.float32, device=dev)
    s = L.fg_wgrad_problem()
    s.p, s.x, s.out = _addr(prob["p"]), _addr(prob["x"]), slab.data_ptr()
    for k in _WG_FIELDS:
        setattr(s, k, int(prob[k]))
    if L.wgrad_f16x3():
        pa, xa = absmax(prob["p"][0]), absmax(prob["x"][0])
        s.p_absmax, s.x_absmax = pa.data_ptr(), xa.data_ptr()
        if CHECK_SCALES:
            check_scale(prob["p"][0], pa, "wgrad gradient")
            check_scale(prob["x"][0], xa, "wgrad input")
    s.p_presplit, s.x_presplit = int(is_presplit(prob["p"][0])), int(is_presplit(prob["x"][0]))
    st = L.stream_handle()
    _timed(tag, lambda: L.check(_lib().fg_conv_wgrad(C.byref(s), st), "conv_wgrad"))
    global LAST_WGRAD_KERNEL
    LAST_WGRAD_KERNEL = L.last_launch()
    m = wmap_struct(wmap)
    L.check(_lib().fg_wgrad_reduce(L.ptr(slab), int(prob["splits"]), C.byref(m), L.ptr(dw), int(accumulate), st),
            "wgrad_reduce")


# ------------------------------------------------------------------ discriminator head (model.11)

N1_ROWS = 5   # input rows per weight-gradient block


def conv_n1_fwd(X, w, b, y):
    """model.11 forward: X Buf (512 ch, border 1), w (1, 512, 4, 4), y [N, 1, h-1, w-1] contiguous"""
    _wrote(y)
    L.check(_lib().fg_conv_n1_fwd(L.ptr(X.t), X.n, X.hp, X.wp, X.c, L.ptr(w.contiguous()), L.ptr(b), L.ptr(y),
                                  y.shape[2], y.shape[3], L.stream_handle()), "conv_n1_fwd")


def conv_n1_wgrad(X, G, wmap, dw):
    """model.11 weight gradient: X Buf (512 ch, border 1), G output-gradient Buf (1 ch, border 3)"""
    blocks = int(_lib().fg_conv_n1_wgrad_blocks(X.n, X.hp, N1_ROWS))
    slab = torch.empty(blocks * 16 * X.c, dtype=torch.float32, device=X.t.device)
    st = L.stream_handle()
    L.check(_lib().fg_conv_n1_wgrad(L.ptr(X.t), X.n, X.hp, X.wp, X.c, L.ptr(G.t), G.hp, G.wp, N1_ROWS, L.ptr(slab),
                                    st), "conv_n1_wgrad")
    m = wmap_struct(wmap)
    L.check(_lib().fg_wgrad_reduce(L.ptr(slab), blocks, C.byref(m), L.ptr(dw), 0, st), "wgrad_reduce")


def d0_input_grad_ok(G, c0, cn, H, W):
    return G.c == 64 and G.pad >= 1 and H % 2 == 0 and W % 2 == 0 and G.h == H // 2 and G.w == W // 2 and 1 <= cn <= 4


def d0_input_grad(G, w, c0, cn, y, accumulate):
    """dL/d(D input channels c0 .. c0+cn-1) of model.0 (4x4 s2 p1, 64 outputs) from its output gradient G (Buf, 64 ch,
    zero border >= 1) into y [N, >= cn, H, W] contiguous NCHW channels 0 .. cn-1 (fg_d0_input_grad, exact fp32)"""
    assert y.is_contiguous() and w.is_contiguous()
    _wrote(y)
    L.check(_lib().fg_d0_input_grad(view(G), L.ptr(w), w.shape[1], c0, cn, L.ptr(y), y.shape[1], y.shape[2],
                                    y.shape[3], int(accumulate), L.stream_handle()), "d0_input_grad")


# ------------------------------------------------------------------ layout

def pack_input(a, ca, b, cb, dst, img0, nimg, pad_mode, amax=None):
    """F.pad + torch.cat into the NHWC Buf dst (fg_pack_input).  The kernel raises dst's absmax slot: a pack
    of all of dst's images takes a fresh one; packs that fill dst in parts pass the slot they share
    (amax_slot(dst), taken before the first part)."""
    if amax is None:
        full = img0 == 0 and nimg == dst.n
        slot = _amax_out(dst) if full else None
        if slot is None:
            _wrote(dst)
    else:
        # a part of a multi-launch fill: the slot must be the one amax_slot(dst) recorded on dst, at dst's
        # current version (the kernels write through raw pointers, so the counter has not moved since)
        slot = amax
        t = _tensor(dst)
        if getattr(t, "_fg_amax", None) is not amax or getattr(t, "_fg_amax_ver", None) != t._version:
            raise RuntimeError("pack_input: the shared absmax slot is not the one amax_slot(dst) recorded on dst "
                               "(or dst was written by torch since)")
        t._fg_split = None
        t._fg_presplit = False
    L.check(_lib().fg_pack_input(sview(a), ca, sview(b), cb, view(dst), img0, nimg, pad_mode, L.ptr(slot),
                                 L.stream_handle()), "pack_input")


def amax_slot(dst):
    """a fresh absmax slot recorded on dst, for producers that write dst in several launches"""
    return _amax_out(dst)


def conv1x1_fwd(X, w, b, n_out, Y):
    """the attention head's 1x1 conv (fp32 FMA, fg_conv1x1_fwd): Y[..., :n_out] = w X + b, Y's other
    channels 0"""
    _wrote(Y)
    L.check(_lib().fg_conv1x1_fwd(view(X), L.ptr(w), L.ptr(b), n_out, view(Y), L.stream_handle()), "conv1x1_fwd")


def conv1x1_dgrad(GY, w, n_out, GX):
    _wrote(GX)
    L.check(_lib().fg_conv1x1_dgrad(view(GY), L.ptr(w), n_out, view(GX), L.stream_handle()), "conv1x1_dgrad")


def conv1x1_wgrad(GY, X, n_out, dw, db, accumulate=False):
    work = torch.empty(int(_lib().fg_conv1x1_wgrad_workspace_floats(n_out)), dtype=torch.float32, device=dw.device)
    L.check(_lib().fg_conv1x1_wgrad(view(GY), view(X), n_out, L.ptr(dw), L.ptr(db), int(accumulate), L.ptr(work),
                                    L.stream_handle()), "conv1x1_wgrad")


def zero_border(B):
    _wrote(B)
    L.check(_lib().fg_zero_border(view(B), L.stream_handle()), "zero_border")


def fold_add(gpad, fold_pad, add, dst):
    _wrote(dst)
    L.check(_lib().fg_fold_add(view(gpad), fold_pad, view(add), view(dst), L.stream_handle()), "fold_add")


def unfold_nchw(gpad, fold_pad, c, dst, acc_channels=0):
    """dst [N, c', H, W] (any strides): channels < c get the reflect-pad adjoint of gpad (accumulated for
    channels < acc_channels)"""
    _wrote(dst)
    N, _, H, W = dst.shape
    assert gpad.n == N and dst.shape[1] >= c
    L.check(_lib().fg_unfold_nchw(view(gpad), fold_pad, c, sview(dst), H, W, acc_channels, L.stream_handle()),
            "unfold_nchw")


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


def in_apply(src, mean, rstd, act, residual, dst, pad_mode, presplit=False, ps_copy=None, splitpix=False):
    """presplit: dst is written in the FG_PRESPLIT format (no residual; the f16x3 math).  ps_copy (Buf of dst's
    geometry): dst in fp32 AND a FG_PRESPLIT copy there (fg_in_apply_dual).  splitpix: dst (C 32 / 64) is written
    in the fg_split_pixels layout the window kernels read (split_pixels(dst) then returns it; no fp32 values)"""
    if splitpix:
        assert residual is None and not presplit and ps_copy is None and L.fwd_f16x3() and L.wgrad_f16x3()
        slot = _amax_out(dst)
        L.check(_lib().fg_in_apply_splitpix(view(src), L.ptr(mean), L.ptr(rstd), act, view(dst), pad_mode,
                                            L.ptr(slot), L.stream_handle()), "in_apply_splitpix")
        t = _tensor(dst)
        split = t.view(torch.float16)
        split.absmax = slot
        t._fg_split, t._fg_split_ver = split, t._version
        t._fg_splitpix, t._fg_splitpix_ver = True, t._version
        return
    presplit = presplit and presplit_fits(dst)
    if ps_copy is not None:
        assert presplit_fits(ps_copy), "pre-split copy beyond PRESPLIT_MAX_BYTES (the caller checks presplit_fits)"
        assert not presplit and L.fwd_f16x3()
        ra = absmax(residual) if residual is not None else None
        slot, ps_slot = _amax_out(dst), _amax_out(ps_copy)
        L.check(_lib().fg_in_apply_dual(view(src), L.ptr(mean), L.ptr(rstd), act, view(residual), L.ptr(ra), view(dst),
                                        pad_mode, L.ptr(slot), L.ptr(ps_copy.t), L.ptr(ps_slot), L.stream_handle()),
                "in_apply_dual")
        _mark_presplit(ps_copy)
        return
    if presplit:
        assert residual is None and L.fwd_f16x3()
        slot = _amax_out(dst)
        L.check(_lib().fg_in_apply_presplit(view(src), L.ptr(mean), L.ptr(rstd), act, view(dst), pad_mode,
                                            L.ptr(slot), L.stream_handle()), "in_apply_presplit")
        _mark_presplit(dst)
        return
    L.check(_lib().fg_in_apply(view(src), L.ptr(mean), L.ptr(rstd), act, view(residual), view(dst), pad_mode,
                               L.ptr(_amax_out(dst)), L.stream_handle()), "in_apply")


def in_bwd(gsrc, fold_pad, gadd, src, mean, rstd, act, dst, bias_grad=None, bias_accumulate=False, gsum=None,
           presplit=False):
    """InstanceNorm (+ activation, reflect-pad fold, residual gradient gadd) backward into dst.  gsum (Buf): also
    receives the gathered gradient fold(gsrc) + gadd (written by the statistics pass that reads it anyway).
    presplit: dst is written in the FG_PRESPLIT format (the f16x3 math)."""
    work = _work(src.n, src.c, src.t.device)
    _wrote(gsum)
    if presplit and presplit_fits(dst):
        assert L.fwd_f16x3()
        slot = _amax_out(dst)
        L.check(_lib().fg_in_bwd_presplit(view(gsrc), fold_pad, view(gadd), view(src), L.ptr(mean), L.ptr(rstd), act,
                                          view(dst), L.ptr(bias_grad), int(bias_accumulate), view(gsum), L.ptr(work),
                                          L.ptr(slot), L.stream_handle()), "in_bwd_presplit")
        _mark_presplit(dst)
        return
    L.check(_lib().fg_in_bwd(view(gsrc), fold_pad, view(gadd), view(src), L.ptr(mean), L.ptr(rstd), act, view(dst),
                             L.ptr(bias_grad), int(bias_accumulate), view(gsum), L.ptr(work),
                             L.ptr(_amax_out(dst)), L.stream_handle()), "in_bwd")


def in_apply_head(src, mean, rstd, act, dst, pad_mode, w, b, n_out, Y):
    """fg_in_apply_head: dst = act(IN(src)) (fp32, unpadded; absmax slot raised) AND the attention head's 1x1 logits
    Y[..., :n_out] = w dst + b (Y's other channels 0), bit-identical to in_apply + conv1x1_fwd.  dst None: only the
    logits (the fused backward, in_bwd_head with wgrad, recomputes the activation)"""
    if dst is None:
        _wrote(Y)
        dv = L.fg_view(None, src.n, src.h, src.w, src.c, 0)
        amax = None
    else:
        _wrote(dst, Y)
        dv, amax = view(dst), L.ptr(_amax_out(dst))
    L.check(_lib().fg_in_apply_head(view(src), L.ptr(mean), L.ptr(rstd), act, dv, pad_mode, amax,
                                    L.ptr(w.contiguous()), L.ptr(b), n_out, view(Y), L.stream_handle()),
            "in_apply_head")


def in_bwd_head(GY, w, n_out, src, mean, rstd, act, dst, bias_grad=None, bias_accumulate=False, presplit=False,
                wgrad=None):
    """fg_in_bwd_head: the norm backward of the attention head's input with the incoming gradient w^T GY formed from
    the logits gradient GY in registers (bit-identical to conv1x1_dgrad + in_bwd; no 64-channel gradient buffer).
    wgrad = (dw, db, accumulate): also the head's weight / bias gradients (the replaced conv1x1_wgrad), from the
    activation recomputed inside the statistics pass"""
    work = _work(src.n, src.c, src.t.device)
    dw = db = wg_work = None
    acc = 0
    if wgrad is not None:
        dw, db, acc = wgrad
        nf = int(_lib().fg_in_head_wgrad_workspace_floats(src.n, src.h, src.w, n_out))
        wg_work = torch.empty(nf, dtype=torch.float32, device=src.t.device)
    tail = (L.ptr(dw), L.ptr(db), int(acc), L.ptr(wg_work), L.stream_handle())
    if presplit and presplit_fits(dst):
        assert L.fwd_f16x3()
        slot = _amax_out(dst)
        L.check(_lib().fg_in_bwd_head(view(GY), L.ptr(w.contiguous()), n_out, view(src), L.ptr(mean), L.ptr(rstd), act,
                                      view(dst), L.ptr(bias_grad), int(bias_accumulate), L.ptr(work), None, L.ptr(slot),
                                      *tail), "in_bwd_head")
        _mark_presplit(dst)
        return
    _wrote(dst)
    L.check(_lib().fg_in_bwd_head(view(GY), L.ptr(w.contiguous()), n_out, view(src), L.ptr(mean), L.ptr(rstd), act,
                                  view(dst), L.ptr(bias_grad), int(bias_accumulate), L.ptr(work),
                                  L.ptr(_amax_out(dst)), None, *tail), "in_bwd_head")


def act_bwd(g, y, act, border_zero=False):
    # in place g *= act'(y) with act' in {0, 0.2, 1}: |g| cannot grow, so a cached absmax slot still
    # bounds it and is kept; a cached pre-split copy no longer matches the contents and is dropped.  Without a
    # cached slot, border_zero=True (g's border holds zeros) lets the kernel raise a fresh one over the interior.
    t = _tensor(g)
    slot, ver = getattr(t, "_fg_amax", None), getattr(t, "_fg_amax_ver", None)
    valid = slot is not None and ver == t._version
    _wrote(g)
    raise_slot = None
    if valid:
        t._fg_amax, t._fg_amax_ver = slot, ver
    elif border_zero:
        raise_slot = _amax_out(g)
    L.check(_lib().fg_act_bwd(view(g), view(y), act, L.ptr(raise_slot), L.stream_handle()), "act_bwd")


def channel_sum(src, c_valid, out, accumulate=False):
    work = torch.empty(_lib().fg_channel_sum_workspace_doubles(src.c), dtype=torch.float64, device=src.t.device)
    L.check(_lib().fg_channel_sum(view(src), c_valid, L.ptr(out), int(accumulate), L.ptr(work), L.stream_handle()),
            "channel_sum")


# ------------------------------------------------------------------ batch norm

BN_MOMENTUM = 0.1


def _bn_work(n, c, dev):
    return torch.empty(int(_lib().fg_bn_workspace_doubles(n, c)), dtype=torch.float64, device=dev)


def _dst_slot(dst, slot):
    """absmax slot a producer raises for dst: the caller's (a buffer several producers write in
    channel slices shares one slot, taken once with _amax_out(buffer)), else a fresh one for a whole
    Buf; a Slice without a slot only invalidates its buffer's caches"""
    if dst is None:
        return None
    if slot is not None:
        return slot
    if isinstance(dst, Slice):
        _wrote(dst)
        return None
    return _amax_out(dst)


def bn_stats(src, groups=1, running=None, eps=EPS, momentum=BN_MOMENTUM):
    """nn.BatchNorm2d(train) statistics of src's interior, per group of src.n / groups images ->
    (mean, invstd) [groups * C]; running = (running_mean, running_var[, num_batches_tracked]) updated
    once per group"""
    dev = src.t.device
    mean = torch.empty(groups * src.c, dtype=torch.float32, device=dev)
    invstd = torch.empty_like(mean)
    rm, rv, nbt = (tuple(running) + (None,))[:3] if running is not None else (None, None, None)
    L.check(_lib().fg_bn_stats(view(src), groups, C.c_float(eps), C.c_float(momentum), L.ptr(mean), L.ptr(invstd),
                               L.ptr(rm), L.ptr(rv), L.ptr(nbt), L.ptr(_bn_work(src.n, src.c, dev)),
                               L.stream_handle()), "bn_stats")
    return mean, invstd


def bn_eval_stats(running_mean, running_var, eps=EPS):
    """module.eval(): (running_mean, 1 / sqrt(running_var + eps))"""
    mean, invstd = torch.empty_like(running_mean), torch.empty_like(running_var)
    L.check(_lib().fg_bn_eval_stats(running_mean.numel(), L.ptr(running_mean), L.ptr(running_var), C.c_float(eps),
                                    L.ptr(mean), L.ptr(invstd), L.stream_handle()), "bn_eval_stats")
    return mean, invstd


DROP_SCALE = 2.0      # nn.Dropout(0.5): kept elements x 1 / (1 - p)


def _drop_args(drop):
    """drop: None, a 0/1 NCHW mask tensor, or an int seed (device-hashed keep decisions)"""
    if drop is None:
        return C.c_void_p(0), 0
    if isinstance(drop, int):
        assert drop > 0
        return C.c_void_p(0), drop
    return L.ptr(drop), 0


def bn_apply(src, groups, mean, invstd, gamma, beta, drop, act0, dst0, act1=0, dst1=None, slots=(None, None)):
    """dst0 = act0(BN(src) * keep * 2), dst1 = act1(same) (interiors; Buf or Slice destinations);
    mean None = no normalisation; drop: None, a 0/1 mask tensor or a seed (see _drop_args)"""
    s0, s1 = _dst_slot(dst0, slots[0]), _dst_slot(dst1, slots[1])
    mask, seed = _drop_args(drop)
    L.check(_lib().fg_bn_apply(view(src), groups, L.ptr(mean), L.ptr(invstd), L.ptr(gamma), L.ptr(beta), mask,
                               C.c_float(DROP_SCALE), seed, act0, view(dst0), L.ptr(s0), act1, view(dst1), L.ptr(s1),
                               L.stream_handle()), "bn_apply")


def bn_bwd(gA, actA, gB, actB, src, groups, mean, invstd, gamma, beta, drop, dst, gamma_grad=None, beta_grad=None,
           accumulate=False):
    """dst = dL/dsrc of bn_apply, the incoming gradient being gA * actA'(u) (+ gB * actB'(u))"""
    slot = _dst_slot(dst, None)
    mask, seed = _drop_args(drop)
    L.check(_lib().fg_bn_bwd(view(gA), actA, view(gB), actB, view(src), groups, L.ptr(mean), L.ptr(invstd),
                             L.ptr(gamma), L.ptr(beta), mask, C.c_float(DROP_SCALE), seed, view(dst),
                             L.ptr(gamma_grad), L.ptr(beta_grad), int(accumulate),
                             L.ptr(_bn_work(src.n, src.c, src.t.device)), L.ptr(slot), L.stream_handle()), "bn_bwd")


def dropout_mask(seed, shape, device):
    """the 0/1 keep decisions bn_apply makes for `seed` over a tensor of NCHW `shape` (float32, device)"""
    out = torch.empty(shape, dtype=torch.float32, device=device)
    L.check(_lib().fg_dropout_mask(seed, C.c_float(1.0 / DROP_SCALE), out.numel(), L.ptr(out), L.stream_handle()),
            "dropout_mask")
    return out


def maxpool2(src, dst):
    _wrote(dst)
    L.check(_lib().fg_maxpool2(view(src), view(dst), L.stream_handle()), "maxpool2")


# ------------------------------------------------------------------ tail / losses / adam

def tail_fwd(cl, al, x, out, mask):
    _wrote(out, mask)
    L.check(_lib().fg_tail_fwd(view(cl), view(al), sview(x), L.ptr(out), L.ptr(mask), L.stream_handle()), "tail_fwd")


def tail_bwd(cl, al, x, g_out, gc, ga, gx=None, g_mask=None):
    """gx (optional [N, C, H, W] tensor): channels 0..2 receive the background term's input gradient;
    g_mask (optional [N, H, W]): dL/d(last_attention_mask), added to attention channel 9's gradient"""
    _wrote(gx)
    gm = None if g_mask is None else g_mask.unsqueeze(1)
    L.check(_lib().fg_tail_bwd(view(cl), view(al), sview(x), sview(g_out), sview(gm), view(gc), view(ga), sview(gx),
                               L.ptr(_amax_out(gc)), L.ptr(_amax_out(ga)), L.stream_handle()), "tail_bwd")


def tanh_head_fwd(logits, c, out):
    _wrote(out)
    L.check(_lib().fg_tanh_head_fwd(view(logits), c, sview(out), L.stream_handle()), "tanh_head_fwd")


def tanh_head_bwd(logits, c, g_out, g_logits):
    _wrote(g_logits)
    L.check(_lib().fg_tanh_head_bwd(view(logits), c, sview(g_out), view(g_logits), L.stream_handle()),
            "tanh_head_bwd")


def mse_const(p, target, gscale, loss_out, g=None):
    """loss_out[0] = mean((p - target)^2); g = gscale * dL/dp (optional)"""
    work = torch.empty(1024, dtype=torch.float64, device=p.device)
    _wrote(g)
    L.check(_lib().fg_mse_const(L.ptr(p), p.numel(), C.c_float(target), C.c_float(gscale), L.ptr(loss_out),
                                L.ptr(g), L.ptr(work), L.stream_handle()), "mse")


def l1(a, b, gscale, loss_out, g=None, accumulate=False, loss_scale=1.0):
    """loss_out[0] = loss_scale * mean|a - b| over [N,C,H,W]; g (contiguous NCHW) = gscale * dL/da"""
    N, Cc, H, W = a.shape
    work = torch.empty(1024, dtype=torch.float64, device=a.device)
    _wrote(g)
    L.check(_lib().fg_l1(sview(a), sview(b), N, Cc, H, W, C.c_float(gscale), C.c_float(loss_scale), L.ptr(loss_out),
                         L.ptr(g),
                         int(accumulate), L.ptr(work), L.stream_handle()), "l1")


def adam_step(entries, lr, beta1, beta2, eps, step):
    """entries: list of (param, grad, exp_avg, exp_avg_sq) tensors sharing `step`.  The kernel
    also raises a fresh absmax slot per parameter (the next weight packing's scale source),
    cached on the parameter with its version counter (see absmax)."""
    if not entries:
        return
    arr = (L.fg_adam_tensor * len(entries))()
    slots = []
    for i, (p, g, m, v) in enumerate(entries):
        arr[i].param, arr[i].grad, arr[i].exp_avg, arr[i].exp_avg_sq = (
            p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr())
        arr[i].numel = p.numel()
        slot = _SLOTS.take(p.device) if L.fwd_f16x3() else None
        arr[i].absmax = slot.data_ptr() if slot is not None else None
        slots.append(slot)
    L.check(_lib().fg_adam_step(arr, len(entries), float(lr), float(beta1), float(beta2), float(eps), int(step),
                                L.stream_handle()), "adam_step")
    for (p, _, _, _), slot in zip(entries, slots):
        # the kernel wrote p through a raw pointer: torch's version counter did not move, so a
        # later in-place torch write (another optimizer, load_state_dict) still invalidates this
        p._fg_amax, p._fg_amax_ver = slot, p._version
    if slots and slots[0] is not None and PACK_CACHE:
        _repack([e[0] for e in entries])
