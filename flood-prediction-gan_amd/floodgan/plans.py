"""Convolution plans: how each conv of the hot path maps onto the implicit-GEMM engine.

Pure host logic (no device calls), so it is unit-tested on the CPU against torch's own
conv2d / conv_transpose2d through a numpy emulation of the engine's addressing
(tests/test_plans_cpu.py).  A plan is a dict whose keys are the fields of
fg_conv_problem / fg_wgrad_problem / fg_weight_map (include/floodgan.h); tensor operands
are (Buf-or-tensor, element offset) pairs that floodgan.ops turns into device pointers.

Reference geometry (models/model_architectures.py):
  conv    k7 s1 reflect-p3   conv1 (:312), deconv3_content (:328)
  conv    k3 s2 zero-p1      conv2, conv3 (:314-316)
  conv    k3 s1 reflect-p1   PairedAttentionBlock.conv1/conv2 (:407-409, pads :413-415)
  convT   k3 s2 p1 op1       deconv1_*, deconv2_* (:324-333)
  conv    k1                 deconv3_attention (:334)
  conv    k4 s2 zero-p1      discriminator model.0/2/5 (:424-433)
  conv    k4 s1 zero-p1      discriminator model.8/11 (:435-437)
"""
import torch

JQ = 16  # the engine's k-tile; packed kernel rows are padded to a multiple of it


def rup(v, q=JQ):
    return (v + q - 1) // q * q


class Buf:
    """NHWC fp32 activation buffer: interior h x w, `pad`-wide border, c channels/pixel,
    backed by one flat tensor.  Element (n, y, x, ch) sits at
    ((n*(h+2p) + y+p)*(w+2p) + x+p)*c + ch  (y, x may reach into the border)."""

    __slots__ = ("t", "n", "h", "w", "c", "pad")

    def __init__(self, t, n, h, w, c, pad=0):
        assert t.numel() >= n * (h + 2 * pad) * (w + 2 * pad) * c
        self.t, self.n, self.h, self.w, self.c, self.pad = t, n, h, w, c, pad

    @classmethod
    def empty(cls, n, h, w, c, pad=0, device="cuda"):
        return cls(torch.empty(n * (h + 2 * pad) * (w + 2 * pad) * c, dtype=torch.float32, device=device),
                   n, h, w, c, pad)

    @classmethod
    def zeros(cls, n, h, w, c, pad=0, device="cuda"):
        return cls(torch.zeros(n * (h + 2 * pad) * (w + 2 * pad) * c, dtype=torch.float32, device=device),
                   n, h, w, c, pad)

    @property
    def hp(self):
        return self.h + 2 * self.pad

    @property
    def wp(self):
        return self.w + 2 * self.pad

    @property
    def s_img(self):
        return self.hp * self.wp * self.c

    @property
    def s_row(self):
        return self.wp * self.c

    def off(self, y, x):
        """element offset of image 0, interior pixel (y, x)"""
        return ((y + self.pad) * self.wp + (x + self.pad)) * self.c

    def padded(self):
        """the same storage seen as an unpadded buffer of the full padded extent"""
        return Buf(self.t, self.n, self.hp, self.wp, self.c, 0)

    def nhwc(self):
        """4-D [n, hp, wp, c] tensor view of the storage (padded extent)"""
        return self.t[: self.n * self.s_img].view(self.n, self.hp, self.wp, self.c)

    def interior(self):
        """[n, h, w, c] view of the interior"""
        p = self.pad
        return self.nhwc()[:, p:p + self.h, p:p + self.w, :]

    def __repr__(self):
        return f"Buf(n={self.n}, h={self.h}, w={self.w}, c={self.c}, pad={self.pad})"


class Slice:
    """Channels [c0, c0 + c) of a Buf: the U-Net's torch.cat([skip, up], 1) halves are slices of one
    buffer (models/model_architectures.py:62).  A kernel given a slice view walks the channel count of
    its source operand with the wider buffer's pixel stride."""

    __slots__ = ("buf", "c0", "c")

    def __init__(self, buf, c0, c):
        assert 0 <= c0 and c0 + c <= buf.c and c0 % 4 == 0
        self.buf, self.c0, self.c = buf, c0, c

    @property
    def t(self):
        return self.buf.t

    n = property(lambda self: self.buf.n)
    h = property(lambda self: self.buf.h)
    w = property(lambda self: self.buf.w)

    def interior(self):
        return self.buf.interior()[..., self.c0:self.c0 + self.c]


def _ydesc(Y):
    """(storage object, element offset of image 0 pixel (py, px) fn, s_img, s_row, pixel stride) of a conv
    output Buf or Slice (a slice is written with its buffer's strides, channels shifted by c0)"""
    if isinstance(Y, Slice):
        b = Y.buf
        return b, (lambda y, x: b.off(y, x) + Y.c0), b.s_img, b.s_row, b.c, Y.c
    return Y, Y.off, Y.s_img, Y.s_row, Y.c, Y.c


def out_size(h, k, s, p):
    return (h + 2 * p - k) // s + 1


# ------------------------------------------------------------------------------------------
# weight maps (fg_weight_map)
# ------------------------------------------------------------------------------------------


def _wmap(n_out, kh, kw, c, c_valid, dim0_is_n, shape, rtab, stab, n_base=0):
    assert len(rtab) == kh and len(stab) == kw and kh <= 8 and kw <= 8
    return dict(n_out=n_out, kh=kh, kw=kw, c=c, c_valid=c_valid, jp=rup(kw * c), dim0_is_n=dim0_is_n,
                d0=shape[0], d1=shape[1], KH=shape[2], KW=shape[3], n_base=n_base,
                rtab=list(rtab), stab=list(stab))


def wmap_conv_fwd(shape, c_alloc):
    """forward conv, weight (O, I, k, k): packed row n = o, column (r, s, ch = i)"""
    O, I, kh, kw = shape
    return _wmap(O, kh, kw, c_alloc, I, 1, shape, range(kh), range(kw))


def wmap_conv_dgrad_s1(shape, c_alloc_gy):
    """stride-1 input gradient = correlation of gy with the flipped, transposed kernel"""
    O, I, kh, kw = shape
    return _wmap(I, kh, kw, c_alloc_gy, O, 0, shape, [kh - 1 - r for r in range(kh)],
                 [kw - 1 - s for s in range(kw)])


def phase_taps(k, p, ph):
    """Stride-2 sub-pixel decomposition.  Output index 2a+ph of  y[o] = sum_{2i-p+r=o} x[i] w[r]
    reads x[a + d] for taps r = ph + p - 2d, d = dmin .. dmin+len-1.  Returns (dmin, [r...])."""
    pairs = sorted(((ph + p - r) // 2, r) for r in range(k) if (r - ph - p) % 2 == 0)
    dmin = pairs[0][0]
    assert [d for d, _ in pairs] == list(range(dmin, dmin + len(pairs)))
    return dmin, [r for _, r in pairs]


def wmap_phase(shape, gathered_is_dim0, k, p, py, px, c_alloc, n_base=0, n_out=None):
    """Phase (py, px) of a stride-2 transposed op.  The gathered operand's channels index
    weight dim 0 (conv-transpose weight (I, O, k, k) in its forward; conv weight (O, I, k, k)
    in a strided conv's input gradient); packed rows index dim 1."""
    assert gathered_is_dim0
    dy, ry = phase_taps(k, p, py)
    dx, rx = phase_taps(k, p, px)
    n_out = shape[1] if n_out is None else n_out
    return _wmap(n_out, len(ry), len(rx), c_alloc, shape[0], 0, shape, ry, rx, n_base), dy, dx


def wmap_convT_dgrad(shape, c_alloc_gy):
    """input gradient of a stride-2 conv-transpose (weight (I, O, k, k)) = stride-2 conv of gy"""
    I, O, kh, kw = shape
    return _wmap(I, kh, kw, c_alloc_gy, O, 1, shape, range(kh), range(kw))


def wmap_wgrad(shape, a_is_dim0, c_alloc_x, k):
    """slab [a][r, s, ch] -> PyTorch weight gradient; a indexes dim 0, ch indexes dim 1"""
    assert a_is_dim0
    return _wmap(shape[0], k, k, c_alloc_x, shape[1], 1, shape, range(k), range(k))


def packed_numel(m):
    return m["n_out"] * m["kh"] * m["jp"]


# ------------------------------------------------------------------------------------------
# forward-kernel problems (fg_conv_problem)
# ------------------------------------------------------------------------------------------


def conv_problem(X, pad_used, k, stride, wp, wmap, Y, bias=None, act=0, accumulate=0, y_nchw=None):
    """Dense conv over X's interior with `pad_used` taken from X's (pre-filled) border.
    Output rows (n, Ho, Wo) land in Y's interior (NHWC) or, when y_nchw=(tensor, C, H, W) is
    given, in a contiguous NCHW tensor."""
    assert X.pad >= pad_used
    Ho, Wo = out_size(X.h, k, stride, pad_used), out_size(X.w, k, stride, pad_used)
    assert wmap["kh"] == k and wmap["kw"] == k and wmap["c"] == X.c
    prob = dict(x=(X, X.off(-pad_used, -pad_used)), w=(wp, 0), bias=bias,
                sxn=X.s_img, sxa=stride * X.s_row, sxb=stride * X.c, sxr=X.s_row,
                m_img=X.n, m_a=Ho, m_b=Wo, kh=k, j_valid=k * X.c, jp=wmap["jp"],
                n_out=wmap["n_out"], ldw=k * wmap["jp"], act=act, accumulate=accumulate)
    if y_nchw is None:
        obj, off, s_img, s_row, pix, cw = _ydesc(Y)
        assert (Y.h, Y.w, Y.n) == (Ho, Wo, X.n) and cw >= wmap["n_out"], (Y, Ho, Wo)
        prob.update(y=(obj, off(0, 0)), syn=s_img, sya=s_row, syb=pix, syc=1)
    else:
        t, Cc, Hh, Ww = y_nchw
        assert (Hh, Ww) == (Ho, Wo)
        prob.update(y=(t, 0), syn=Cc * Hh * Ww, sya=Ww, syb=1, syc=Hh * Ww)
    return prob


def window_problem(X, y0, x0, rows, cols, kh, kw, wp, wmap, Y, oy0, ox0, w_row0=0):
    """Stride-1 conv over a rectangular window of output positions: output (oy0 + i, ox0 + j) of Y
    (coordinates relative to Y's interior origin, the border included) = sum over taps (r < kh, s < kw)
    of X(y0 + i + r, x0 + j + s) (relative to X's interior origin; inside X's padded extent) with the
    packed weights of wmap (its rtab / stab say which kernel rows / columns the taps are).  w_row0 > 0:
    the taps are rows w_row0 .. w_row0 + kh - 1 of a pack with wmap["kh"] rows (a sub-range of a full
    kernel's pack, no pack of its own)"""
    assert -X.pad <= y0 and y0 + rows - 1 + kh - 1 <= X.h - 1 + X.pad
    assert -X.pad <= x0 and x0 + cols - 1 + kw - 1 <= X.w - 1 + X.pad
    assert -Y.pad <= oy0 and oy0 + rows <= Y.h + Y.pad and -Y.pad <= ox0 and ox0 + cols <= Y.w + Y.pad
    assert w_row0 + kh <= wmap["kh"] and wmap["kw"] == kw and wmap["c"] == X.c and Y.c >= wmap["n_out"]
    # weight-row offset in the 4-byte units of the problem's w reference: fp32 packs hold 1 float per k, the
    # f16x3 pre-split packs 2 fp16 (h, l), the bf16x6 packs 3 bf16 (h, m, l)
    units = {torch.float32: 1, torch.float16: 1, torch.bfloat16: 1.5}[wp.dtype] * w_row0 * wmap["jp"]
    assert units == int(units)
    return dict(x=(X, X.off(y0, x0)), w=(wp, int(units)), bias=None, sxn=X.s_img, sxa=X.s_row, sxb=X.c,
                sxr=X.s_row, m_img=X.n, m_a=rows, m_b=cols, kh=kh, j_valid=kw * X.c, jp=wmap["jp"],
                n_out=wmap["n_out"], ldw=wmap["kh"] * wmap["jp"], act=0, accumulate=0, y=(Y, Y.off(oy0, ox0)),
                syn=Y.s_img, sya=Y.s_row, syb=Y.c, syc=1)


def wmap_conv_dgrad_s1_taps(shape, c_alloc_gy, rows, cols):
    """wmap_conv_dgrad_s1 restricted to the gather taps `rows` x `cols` (indices into the full 0..k-1
    correlation): the edge strips of a padded-domain input gradient, where the zero border of the
    output gradient leaves a single kernel row or column"""
    O, I, kh, kw = shape
    return _wmap(I, len(rows), len(cols), c_alloc_gy, O, 0, shape, [kh - 1 - r for r in rows],
                 [kw - 1 - s for s in cols])


def phase_problems(S, shape, k, p, Y, wp_list, maps, bias=None, act=0, accumulate=0, y_nchw=None, n_out=None):
    """The four output phases of a stride-2 transposed op reading S (zero border >= 1):
    a ConvTranspose2d(k, 2, p, output_padding) forward, or a stride-2 conv's input gradient.
    wp_list/maps: per phase (py, px) in order (0,0), (0,1), (1,0), (1,1)."""
    assert S.pad >= 1
    if y_nchw is None:
        Ho, Wo = Y.h, Y.w
    else:
        _, Cc, Ho, Wo = y_nchw
    probs = []
    for i, (py, px) in enumerate(((0, 0), (0, 1), (1, 0), (1, 1))):
        m, dy, dx = maps[i]
        ma, mb = (Ho - py + 1) // 2, (Wo - px + 1) // 2
        assert ma - 1 + dy + m["kh"] - 1 <= S.h - 1 + S.pad and dy >= -S.pad
        assert mb - 1 + dx + m["kw"] - 1 <= S.w - 1 + S.pad and dx >= -S.pad
        prob = dict(x=(S, S.off(dy, dx)), w=(wp_list[i], 0), bias=bias,
                    sxn=S.s_img, sxa=S.s_row, sxb=S.c, sxr=S.s_row,
                    m_img=S.n, m_a=ma, m_b=mb, kh=m["kh"], j_valid=m["kw"] * S.c, jp=m["jp"],
                    n_out=m["n_out"], ldw=m["kh"] * m["jp"], act=act, accumulate=accumulate)
        if y_nchw is None:
            obj, off, s_img, s_row, pix, _ = _ydesc(Y)
            prob.update(y=(obj, off(py, px)), syn=s_img, sya=2 * s_row, syb=2 * pix, syc=1)
        else:
            t = y_nchw[0]
            prob.update(y=(t, py * Wo + px), syn=Cc * Ho * Wo, sya=2 * Wo, syb=2, syc=Ho * Wo)
        probs.append(prob)
    return probs


# column groups of the quad form in the order (py, px) = (0,0), (1,1), (0,1), (1,0): the 64 x 128 waves of its tile
# hold two groups each, and this pairing gives them 5 and 4 of the 9 live (group, segment) products of a 3-tap
# kernel instead of 3 and 6 (conv_f3.hip QUAD)
QUAD_PHASES = ((0, 0), (1, 1), (0, 1), (1, 0))


def quad_map(shape, k, p, c_alloc, n_out=None):
    """The four phases of a stride-2 transposed op with a 3-tap kernel as ONE pack (the quad form,
    fg_weight_map.q_n): packed row q*n_out + o is output channel o of phase QUAD_PHASES[q]; k runs over the
    2 x 2 input neighbourhood (a + R, b + S), R, S in {0, 1}, of the output block (2a.., 2b..).  Returns
    (map, d0, q_mask): d0 the neighbourhood's offset, q_mask bit q*4 + R*2 + S set where phase q has a tap."""
    n_out = shape[1] if n_out is None else n_out
    taps = {ph: phase_taps(k, p, ph) for ph in (0, 1)}
    d0 = min(d for d, _ in taps.values())
    assert all(d - d0 + len(r) <= 2 for d, r in taps.values()), "the quad form needs <= 2 taps per phase"

    def tab(ph):
        d, r = taps[ph]
        return [r[i - (d - d0)] if 0 <= i - (d - d0) < len(r) else -1 for i in range(2)]

    rtab, stab, mask = [], [], 0
    for q, (py, px) in enumerate(QUAD_PHASES):
        rt, st = tab(py), tab(px)
        rtab += rt
        stab += st
        for R in range(2):
            for S in range(2):
                if rt[R] >= 0 and st[S] >= 0:
                    mask |= 1 << (q * 4 + R * 2 + S)
    m = dict(n_out=4 * n_out, kh=2, kw=2, c=c_alloc, c_valid=shape[0], jp=rup(2 * c_alloc), dim0_is_n=0,
             d0=shape[0], d1=shape[1], KH=shape[2], KW=shape[3], n_base=0, rtab=rtab, stab=stab, q_n=n_out)
    return m, d0, mask


def quad_problem(S, m, d0, mask, wp, Y, bias=None):
    """The quad-form problem over S (zero border >= 1) into Y (NHWC Buf, 2x S's extent) -- see quad_map"""
    assert S.pad >= 1 and -S.pad <= d0 and d0 + 1 + S.h - 1 <= S.h - 1 + S.pad and isinstance(Y, Buf)
    assert (Y.h, Y.w, Y.n) == (2 * S.h, 2 * S.w, S.n) and Y.c == m["q_n"]
    prob = dict(x=(S, S.off(d0, d0)), w=(wp, 0), bias=bias, sxn=S.s_img, sxa=S.s_row, sxb=S.c, sxr=S.s_row,
                m_img=S.n, m_a=S.h, m_b=S.w, kh=2, j_valid=2 * S.c, jp=m["jp"], n_out=m["n_out"], ldw=2 * m["jp"],
                act=0, accumulate=0, y=(Y, Y.off(0, 0)), syn=Y.s_img, sya=2 * Y.s_row, syb=2 * Y.c, syc=1,
                q_n=m["q_n"], q_mask=mask,
                q_yoff=[Y.off(py, px) - Y.off(0, 0) for py, px in QUAD_PHASES])
    return prob


def phase_maps(shape, k, p, c_alloc, n_base=0, n_out=None):
    return [wmap_phase(shape, True, k, p, py, px, c_alloc, n_base, n_out)
            for py, px in ((0, 0), (0, 1), (1, 0), (1, 1))]


# ------------------------------------------------------------------------------------------
# weight-gradient problems (fg_wgrad_problem)
# ------------------------------------------------------------------------------------------

WG_BLOCKS = 512    # one wave of resident weight-gradient workgroups (256 CUs x 2): fewer fp32 slabs


def wgrad_tile(n_a):
    """(rows, cols) of the weight-gradient tile the engine picks for n_a result rows"""
    if n_a > 128:
        return (256, 128)
    return (128, 128) if n_a > 64 else ((64, 256) if n_a > 32 else (32, 256))


F3_WG_BLOCKS = 256  # the pipelined f16x3 weight-gradient kernel: 128 KiB LDS, one workgroup per CU


def wgrad_splits(n_a, K, M, f3=False):
    """(splits, pixels per split) of a weight-gradient problem: about one resident wave of
    workgroups.  f3: the pipelined f16x3 kernel's 256 x 256 tiles and 32-pixel stages."""
    if f3:
        ba, bk, blocks, q = (256 if n_a >= 256 else 128 if n_a > 64 else 64), 256, F3_WG_BLOCKS, 32
    else:
        (ba, bk), blocks, q = wgrad_tile(n_a), WG_BLOCKS, 16
    tiles = -(-n_a // ba) * -(-K // bk)
    splits = max(1, min(blocks // max(tiles, 1), -(-M // 256)))
    chunk = rup(-(-M // splits), q)
    splits = -(-M // chunk)
    return splits, chunk


STEM_PX = 64        # conv_stem.hip: output pixels per strip
STEM_SPLITS = 256   # about one workgroup per CU


def stem_wgrad_layout(prob):
    """(splits, m_chunk) for the stem weight-gradient kernel (conv_stem.hip: the 7x7 conv over the 9-channel input
    with 64 outputs) -- one workgroup per 64-px column strip of `rows` output rows, m_chunk = 64 * rows -- or None
    when the kernel does not take the problem (fgc::stem_wgrad_rows, the same conditions)"""
    if not (prob["n_a"] == 64 and prob["kh"] == 7 and prob["j_valid"] == 63 and prob["sxb"] == 9
            and prob["sxr"] == prob["sxa"] and prob["m_b"] % STEM_PX == 0 and prob["spb"] >= 64
            and (prob["spn"] | prob["spa"] | prob["spb"]) % 4 == 0):
        return None
    strips = prob["m_img"] * (prob["m_b"] // STEM_PX)
    m_a = prob["m_a"]
    # the most rows per split that still gives about STEM_SPLITS workgroups (a divisor of m_a)
    want = max(1, -(-strips * m_a // STEM_SPLITS))
    rows = next((r for r in range(want, m_a + 1) if m_a % r == 0), m_a)
    return strips * (m_a // rows), STEM_PX * rows


def f3_wgrad_eligible(prob):
    """the shapes the pipelined f16x3 weight-gradient kernel takes (conv_wgrad_f3.hip)"""
    return prob["n_a"] >= 64 and prob["kh"] * prob["j_valid"] >= 256 and prob["n_a"] % 4 == 0 \
        and prob["j_valid"] % 4 == 0


def wgrad_problem(P, n_a, X, x_off_yx, sxa, sxb, k, slab=None):
    """out[split][a][r, s, ch] = sum over P's interior rows of P[m][a] * X-gather.
    P: Buf whose interior rows are the reduction index; X gathered as in the forward."""
    M = P.n * P.h * P.w
    K = k * k * X.c
    splits, chunk = wgrad_splits(n_a, K, M)
    return dict(p=(P, P.off(0, 0)), x=(X, X.off(*x_off_yx)), out=slab,
                spn=P.s_img, spa=P.s_row, spb=P.c,
                sxn=X.s_img, sxa=sxa, sxb=sxb, sxr=X.s_row,
                m_img=P.n, m_a=P.h, m_b=P.w, n_a=n_a, kh=k, j_valid=k * X.c,
                splits=splits, m_chunk=chunk)


def wgrad_conv(gy, X, pad_used, k, stride, O):
    """conv weight gradient: P = gy (rows = output pixels), X gathered like the forward"""
    return wgrad_problem(gy, O, X, (-pad_used, -pad_used), stride * X.s_row, stride * X.c, k)


def wgrad_convT(x, gyp, k, p, I):
    """ConvTranspose2d(k, s=2, p) weight gradient: P = x (rows = input pixels), gathered gy
    (zero border >= p) at 2i - p + r."""
    assert gyp.pad >= p
    return wgrad_problem(x, I, gyp, (-p, -p), 2 * gyp.s_row, 2 * gyp.c, k)


def slab_numel(prob):
    return prob["splits"] * prob["n_a"] * prob["kh"] * prob["j_valid"]
