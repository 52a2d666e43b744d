"""CPU check of the convolution plans (floodgan/plans.py): a numpy emulation of exactly the
addressing the HIP engine performs (fg_conv_problem / fg_wgrad_problem / fg_weight_map,
include/floodgan.h) must reproduce torch's conv2d / conv_transpose2d forward, input and weight
gradients for every geometry of the PairedAttention path."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from floodgan import plans as PL
from floodgan.plans import Buf


# ---------------- emulator ----------------

def _arr(ref):
    obj, off = ref
    t = obj.t if isinstance(obj, Buf) else obj
    return t.view(-1).numpy(), off


def emu_pack(w, m):
    w = w.contiguous().view(-1).numpy()
    K = m["kh"] * m["jp"]
    out = np.zeros((m["n_out"], K), np.float64)
    for n in range(m["n_out"]):
        for kr in range(m["kh"]):
            for j in range(m["kw"] * m["c"]):
                ks, ch = divmod(j, m["c"])
                if ch >= m["c_valid"]:
                    continue
                r, s, nn = m["rtab"][kr], m["stab"][ks], n + m["n_base"]
                if m["dim0_is_n"]:
                    src = ((nn * m["d1"] + ch) * m["KH"] + r) * m["KW"] + s
                else:
                    src = ((ch * m["d1"] + nn) * m["KH"] + r) * m["KW"] + s
                out[n, kr * m["jp"] + j] = w[src]
    return torch.from_numpy(out.astype(np.float32)).view(-1)


def _rows(p, prefix):
    M = p["m_img"] * p["m_a"] * p["m_b"]
    m = np.arange(M)
    img, rem = np.divmod(m, p["m_a"] * p["m_b"])
    a, b = np.divmod(rem, p["m_b"])
    return img * p[f"{prefix}n"] + a * p[f"{prefix}a"] + b * p[f"{prefix}b"]


def emu_conv(p):
    x, xo = _arr(p["x"])
    wp = p["w"][0].view(-1).numpy().reshape(p["n_out"], -1)
    y, yo = _arr(p["y"])
    rows = _rows(p, "sx") + xo
    k = np.arange(p["kh"] * p["jp"])
    r, j = np.divmod(k, p["jp"])
    valid = j < p["j_valid"]
    idx = rows[:, None] + r[None, :] * p["sxr"] + np.where(valid, j, 0)[None, :]
    assert idx.min() >= 0 and idx[:, valid].max() < x.size, "out-of-bounds gather"
    A = np.where(valid[None, :], x[idx], 0.0).astype(np.float64)
    out = A @ wp[:, : p["kh"] * p["jp"]].T.astype(np.float64)
    if p["bias"] is not None:
        out += p["bias"].numpy()[None, :]
    if p["act"] == 1:
        out = np.maximum(out, 0)
    elif p["act"] == 2:
        out = np.where(out > 0, out, 0.2 * out)
    yrows = _rows(p, "sy") + yo
    yidx = yrows[:, None] + np.arange(p["n_out"])[None, :] * p["syc"]
    assert yidx.min() >= 0 and yidx.max() < y.size, "out-of-bounds store"
    if p["accumulate"]:
        out = out + y[yidx]
    y[yidx] = out.astype(np.float32)


def emu_wgrad(p):
    P, po = _arr(p["p"])
    X, xo = _arr(p["x"])
    rp = _rows(p, "sp") + po
    rx = _rows(p, "sx") + xo
    K = p["kh"] * p["j_valid"]
    k = np.arange(K)
    r, j = np.divmod(k, p["j_valid"])
    ia = rp[:, None] + np.arange(p["n_a"])[None, :]
    ib = rx[:, None] + (r * p["sxr"] + j)[None, :]
    assert ia.min() >= 0 and ia.max() < P.size and ib.min() >= 0 and ib.max() < X.size, "out-of-bounds"
    A = P[ia].astype(np.float64)      # [M, n_a]
    B = X[ib].astype(np.float64)      # [M, K]
    return A.T @ B                                                           # [n_a, K]


def emu_reduce(slab, m, dw):
    dw = dw.view(-1).numpy()
    J = m["kw"] * m["c"]
    for a in range(m["n_out"]):
        for k in range(m["kh"] * J):
            kr, j = divmod(k, J)
            ks, ch = divmod(j, m["c"])
            if ch >= m["c_valid"]:
                continue
            r, s, n = m["rtab"][kr], m["stab"][ks], a + m["n_base"]
            dst = ((n * m["d1"] + ch) * m["KH"] + r) * m["KW"] + s
            dw[dst] = slab[a, k]


def to_buf(x_nchw, pad, mode, c_alloc=None):
    n, c, h, w = x_nchw.shape
    c_alloc = c_alloc or c
    xp = F.pad(x_nchw, (pad,) * 4, mode=mode) if pad else x_nchw
    nhwc = torch.zeros(n, h + 2 * pad, w + 2 * pad, c_alloc)
    nhwc[..., :c] = xp.permute(0, 2, 3, 1)
    return Buf(nhwc.reshape(-1).clone(), n, h, w, c_alloc, pad)


def from_buf(B, c=None):
    c = c or B.c
    return B.interior()[..., :c].permute(0, 3, 1, 2).contiguous()


def close(a, b, tol=2e-5):
    a, b = a.double(), b.double()
    return float((a - b).norm() / max(b.norm(), 1e-12)) < tol


torch.manual_seed(0)

# (cin, cout, k, stride, pad, mode) -- every conv geometry of G and D (reduced channels)
CONV_CASES = [(9, 8, 7, 1, 3, "reflect"), (8, 12, 3, 2, 1, "constant"), (8, 8, 3, 1, 1, "reflect"),
              (8, 27, 7, 1, 3, "reflect"), (8, 10, 1, 1, 0, "constant"), (12, 8, 4, 2, 1, "constant"),
              (8, 16, 4, 1, 1, "constant"), (16, 1, 4, 1, 1, "constant")]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_forward_plan(case):
    cin, cout, k, s, p, mode = case
    x = torch.randn(2, cin, 12, 12)
    w = torch.randn(cout, cin, k, k)
    b = torch.randn(cout)
    ref = F.conv2d(F.pad(x, (p,) * 4, mode=mode) if p else x, w, b, stride=s)
    X = to_buf(x, p, mode)
    m = PL.wmap_conv_fwd(w.shape, X.c)
    wp = emu_pack(w, m)
    Ho = PL.out_size(12, k, s, p)
    Y = Buf(torch.zeros(2 * Ho * Ho * cout), 2, Ho, Ho, cout, 0)
    emu_conv(PL.conv_problem(X, p, k, s, wp, m, Y, bias=b))
    assert close(from_buf(Y), ref)


@pytest.mark.parametrize("case", [c for c in CONV_CASES if c[3] == 1])
def test_conv_dgrad_s1_plan(case):
    cin, cout, k, s, p, mode = case
    x = torch.randn(2, cin, 10, 10)
    w = torch.randn(cout, cin, k, k)
    if mode == "reflect":
        # gradient w.r.t. the PADDED input = full correlation (pad k-1), later folded
        xp = F.pad(x, (p,) * 4, mode="reflect").requires_grad_(True)
        y = F.conv2d(xp, w)
        gy = torch.randn_like(y)
        (ref,) = torch.autograd.grad(y, xp, gy)
        pd, eff = k - 1, 0
    else:
        xr = x.clone().requires_grad_(True)
        y = F.conv2d(xr, w, padding=p)
        gy = torch.randn_like(y)
        (ref,) = torch.autograd.grad(y, xr, gy)
        pd, eff = k - 1 - p, p
    G = to_buf(gy, pd, "constant")
    m = PL.wmap_conv_dgrad_s1(w.shape, G.c)
    wp = emu_pack(w, m)
    Hh = ref.shape[-1]
    Y = Buf(torch.zeros(2 * Hh * Hh * cin), 2, Hh, Hh, cin, 0)
    emu_conv(PL.conv_problem(G, pd, k, 1, wp, m, Y))
    assert close(from_buf(Y), ref)


@pytest.mark.parametrize("k", [3, 4])
@pytest.mark.parametrize("H", [8, 7])
def test_strided_conv_dgrad_phase_plan(k, H):
    cin, cout = 6, 10
    x = torch.randn(2, cin, H, H, requires_grad=True)
    w = torch.randn(cout, cin, k, k)
    y = F.conv2d(x, w, stride=2, padding=1)
    gy = torch.randn_like(y)
    (ref,) = torch.autograd.grad(y, x, gy)
    G = to_buf(gy, 1, "constant")
    maps = PL.phase_maps(w.shape, k, 1, G.c)
    wps = [emu_pack(w, m) for m, _, _ in maps]
    Y = Buf(torch.zeros(2 * H * H * cin), 2, H, H, cin, 0)
    for prob in PL.phase_problems(G, w.shape, k, 1, Y, wps, maps):
        emu_conv(prob)
    assert close(from_buf(Y), ref)


def test_convT_forward_phase_plan():
    cin, cout, H = 8, 6, 5
    x = torch.randn(2, cin, H, H)
    w = torch.randn(cin, cout, 3, 3)
    b = torch.randn(cout)
    ref = F.conv_transpose2d(x, w, b, stride=2, padding=1, output_padding=1)
    X = to_buf(x, 1, "constant")
    maps = PL.phase_maps(w.shape, 3, 1, X.c)
    wps = [emu_pack(w, m) for m, _, _ in maps]
    Y = Buf(torch.zeros(2 * 4 * H * H * cout), 2, 2 * H, 2 * H, cout, 0)
    for prob in PL.phase_problems(X, w.shape, 3, 1, Y, wps, maps, bias=b):
        emu_conv(prob)
    assert close(from_buf(Y), ref)


def test_convT_dgrad_plan():
    cin, cout, H = 8, 6, 5
    x = torch.randn(2, cin, H, H, requires_grad=True)
    w = torch.randn(cin, cout, 3, 3)
    y = F.conv_transpose2d(x, w, stride=2, padding=1, output_padding=1)
    gy = torch.randn_like(y)
    (ref,) = torch.autograd.grad(y, x, gy)
    G = to_buf(gy, 1, "constant")
    m = PL.wmap_convT_dgrad(w.shape, G.c)
    Y = Buf(torch.zeros(2 * H * H * cin), 2, H, H, cin, 0)
    emu_conv(PL.conv_problem(G, 1, 3, 2, emu_pack(w, m), m, Y))
    assert close(from_buf(Y), ref)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_wgrad_plan(case):
    cin, cout, k, s, p, mode = case
    x = torch.randn(2, cin, 12, 12)
    w = torch.randn(cout, cin, k, k, requires_grad=True)
    y = F.conv2d(F.pad(x, (p,) * 4, mode=mode) if p else x, w, stride=s)
    gy = torch.randn_like(y)
    (ref,) = torch.autograd.grad(y, w, gy)
    X = to_buf(x, p, mode)
    GY = to_buf(gy, 0, "constant")
    prob = PL.wgrad_conv(GY, X, p, k, s, cout)
    slab = emu_wgrad(prob)
    dw = torch.zeros_like(w)
    emu_reduce(slab, PL.wmap_wgrad(w.shape, True, X.c, k), dw)
    assert close(dw, ref)


def test_convT_wgrad_plan():
    cin, cout, H = 8, 6, 5
    x = torch.randn(2, cin, H, H)
    w = torch.randn(cin, cout, 3, 3, requires_grad=True)
    y = F.conv_transpose2d(x, w, stride=2, padding=1, output_padding=1)
    gy = torch.randn_like(y)
    (ref,) = torch.autograd.grad(y, w, gy)
    X = to_buf(x, 0, "constant")
    GY = to_buf(gy, 1, "constant")
    prob = PL.wgrad_convT(X, GY, 3, 1, cin)
    slab = emu_wgrad(prob)
    dw = torch.zeros_like(w)
    emu_reduce(slab, PL.wmap_wgrad(w.shape, True, GY.c, 3), dw)
    assert close(dw, ref)


def test_phase_partial_channels():
    """D model.0 input gradient restricted to the 3 generated channels (n_base=9)."""
    x = torch.randn(2, 12, 8, 8, requires_grad=True)
    w = torch.randn(6, 12, 4, 4)
    y = F.conv2d(x, w, stride=2, padding=1)
    gy = torch.randn_like(y)
    (ref,) = torch.autograd.grad(y, x, gy)
    G = to_buf(gy, 1, "constant")
    maps = PL.phase_maps(w.shape, 4, 1, G.c, n_base=9, n_out=3)
    wps = [emu_pack(w, m) for m, _, _ in maps]
    out = torch.zeros(2, 3, 8, 8)
    for prob in PL.phase_problems(G, w.shape, 4, 1, None, wps, maps, y_nchw=(out.view(-1), 3, 8, 8)):
        emu_conv(prob)
    assert close(out, ref[:, 9:12])


def test_quad_map_and_problem():
    """the quad form (plans.quad_map / quad_problem) emulated in fp64 on the CPU: the 4 phases of
    ConvTranspose2d(ci, 64, 3, 2, 1, 1) as one GEMM over the 2 x 2 input neighbourhood, scattered by q_yoff,
    equal torch's conv_transpose2d; the packed weights are zero exactly where q_mask is clear; each wave of the
    64 x 128 tiling (column groups {0, 1} and {2, 3}) has 5 resp. 4 live (group, segment) products"""
    import numpy as np
    from floodgan import plans as PL
    from floodgan.plans import Buf
    torch.manual_seed(0)
    N, H, W, ci = 2, 3, 4, 32
    x = torch.randn(N, ci, H, W, dtype=torch.float64)
    w = torch.randn(ci, 64, 3, 3, dtype=torch.float64)
    ref = torch.nn.functional.conv_transpose2d(x, w, stride=2, padding=1, output_padding=1)
    S = Buf(torch.zeros(N * (H + 2) * (W + 2) * ci, dtype=torch.float64), N, H, W, ci, 1)
    S.interior().copy_(x.permute(0, 2, 3, 1))
    Y = Buf(torch.zeros(N * (2 * H + 2) * (2 * W + 2) * 64, dtype=torch.float64), N, 2 * H, 2 * W, 64, 1)
    m, d0, mask = PL.quad_map(w.shape, 3, 1, ci)
    assert (m["n_out"], m["q_n"], d0) == (256, 64, 0)
    Wp = np.zeros((256, 2 * m["jp"]))
    for n in range(256):
        q, o = divmod(n, 64)
        for kr in range(2):
            for ks in range(2):
                r, s = m["rtab"][q * 2 + kr], m["stab"][q * 2 + ks]
                if r >= 0 and s >= 0:
                    Wp[n, kr * m["jp"] + ks * ci: kr * m["jp"] + (ks + 1) * ci] = w[:, o, r, s].numpy()
    for q in range(4):
        for seg in range(4):
            R, Sg = divmod(seg, 2)
            blk = Wp[q * 64:(q + 1) * 64, R * m["jp"] + Sg * ci: R * m["jp"] + (Sg + 1) * ci]
            assert bool(np.abs(blk).sum() > 0) == bool((mask >> (q * 4 + seg)) & 1)
    live = [sum((mask >> (q * 4 + sg)) & 1 for q in g for sg in range(4)) for g in ((0, 1), (2, 3))]
    assert live == [5, 4]
    p = PL.quad_problem(S, m, d0, mask, None, Y)
    xs, yv = S.t.numpy().ravel(), Y.t.numpy().ravel()
    for img in range(N):
        for a in range(H):
            for b in range(W):
                row = p["x"][1] + img * p["sxn"] + a * p["sxa"] + b * p["sxb"]
                A = np.concatenate([xs[row + r * p["sxr"]: row + r * p["sxr"] + p["jp"]] for r in range(2)])
                out = Wp @ A
                base = p["y"][1] + img * p["syn"] + a * p["sya"] + b * p["syb"]
                for n in range(256):
                    q, o = divmod(n, 64)
                    yv[base + o + p["q_yoff"][q]] = out[n]
    got = Y.interior().permute(0, 3, 1, 2)
    assert float((got - ref).abs().max()) < 1e-10
