"""Run one conv-engine launch shape repeatedly (for rocprofv3 counter passes).
  python scripts/conv_one.py [fwd|fwd_stats|fwd_stats_ps|wgrad|dgrad_ps|wgrad_ps|stem_fwd|stem_wgrad|win_fwd|quad_stats|convT4_stats] [reps]
  -- resblock 3x3 256->256 @128, bs 8 (stem_*: the generator stem 7x7 9->64 @512, bs 8, on its strip kernels)
  (fwd_stats: with the InstanceNorm statistics epilogue, as the step's conv1 runs; fwd_stats_ps: on a FG_PRESPLIT
  operand written by the norm pass, as the step's conv2 runs; dgrad_ps: the input-gradient interior launch of
  executor._dgrad_s1_padded over a pre-split conv-output gradient with its zero border 2; wgrad_ps: the step's
  weight gradient with both operands pre-split, gradient border 2, input reflect border 1)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
import torch  # noqa: E402

from floodgan import _lib as L, ops, plans as PL  # noqa: E402
from floodgan.plans import Buf  # noqa: E402


def stem(kind, dev):
    """the stem launch as the step runs it: the packed input (reflect border 3), forward with the statistics
    epilogue, or the weight gradient against a 64-channel conv-output gradient"""
    from floodgan._lib import FG_PAD_REFLECT
    L.set_conv_math("f16x3")
    N, H = 8, 512
    x = torch.rand(N, 9, H, H, device=dev) * 2 - 1
    X0 = Buf.empty(N, H, H, 9, 3, dev)
    ops.pack_input(x, 9, None, 0, X0, 0, N, FG_PAD_REFLECT)
    if kind == "stem_wgrad":
        gy = Buf.empty(N, H, H, 64, 0, dev)
        gy.t.normal_()
        prob = PL.wgrad_conv(gy, X0, 3, 7, 1, 64)
        dw = torch.empty(64, 9, 7, 7, device=dev)
        wm = PL.wmap_wgrad(dw.shape, True, 9, 7)
        return lambda: ops.wgrad(prob, wm, dw)
    w = torch.randn(64, 9, 7, 7, device=dev) * 0.05
    m = PL.wmap_conv_fwd(w.shape, 9)
    Y = Buf.empty(N, H, H, 64, 0, dev)
    prob = PL.conv_problem(X0, 3, 7, 1, ops.pack_weight(w, m), m, Y, bias=torch.zeros(64, device=dev))
    return lambda: ops.conv([prob], in_stats=True)


def win_fwd(dev):
    """the content head's 7x7 64 -> 27 forward on the row-strip window kernel (bs 8, 512^2), as bench_win.py"""
    L.set_conv_math("f16x3")
    N = 8
    ad2 = Buf.empty(N, 512, 512, 64, 3, dev)
    ad2.t.uniform_(-1, 1)
    w = torch.randn(27, 64, 7, 7, device=dev) * 0.02
    m = PL.wmap_conv_fwd(w.shape, 64)
    cl = Buf.empty(N, 512, 512, 32, 0, dev)
    prob = PL.conv_problem(ad2, 3, 7, 1, ops.pack_weight(w, m), m, cl)
    return lambda: ops.conv_win(prob)


def deconv2(kind, dev):
    """deconv2 (ConvTranspose2d(128, 64, 3, 2, 1, 1), bs 8, 256^2 -> 512^2) on a pre-split relu(IN(.)) operand with
    the statistics epilogue: quad_stats = the quad form, convT4_stats = the four phase problems"""
    from floodgan import executor as X
    L.set_conv_math("f16x3")
    N, H = 8, 256
    c = Buf.empty(N, H, H, 128, 0, dev)
    c.t.normal_()
    mean, rstd = ops.in_stats(c)
    S = Buf.empty(N, H, H, 128, 1, dev)
    ops.in_apply(c, mean, rstd, 1, None, S, 0, presplit=True)
    P = {"t.weight": torch.randn(128, 64, 3, 3, device=dev) * 0.05, "t.bias": torch.zeros(64, device=dev)}
    Y = Buf.empty(N, 2 * H, 2 * H, 64, 0, dev)
    if kind == "quad_stats":
        return lambda: X._convT_fwd(P, "t", S, Y)
    from floodgan import plans as PL
    maps = PL.phase_maps(P["t.weight"].shape, 3, 1, S.c)
    wps = [ops.pack_weight(P["t.weight"], m) for m, _, _ in maps]
    return lambda: ops.conv(PL.phase_problems(S, P["t.weight"].shape, 3, 1, Y, wps, maps, bias=P["t.bias"]),
                            in_stats=True)


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "fwd"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    L.load()
    dev = "cuda"
    if kind.startswith("stem_") or kind in ("win_fwd", "quad_stats", "convT4_stats"):
        fn = (stem(kind, dev) if kind.startswith("stem_") else win_fwd(dev) if kind == "win_fwd" else
              deconv2(kind, dev))
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        print("done", kind, reps)
        return
    N, H, C, k = 8, 128, 256, 3
    X = Buf.empty(N, H, H, C, 1, dev)
    X.t.uniform_(-1, 1)
    w = torch.randn(C, C, k, k, device=dev) * 0.02
    m = PL.wmap_conv_fwd(w.shape, C)
    Y = Buf.empty(N, H, H, C, 0, dev)
    Y.t.uniform_(-1, 1)
    if kind == "fwd_stats_ps":
        c = Buf.empty(N, H, H, C, 0, dev)
        c.t.normal_()
        mean, rstd = ops.in_stats(c)
        ops.in_apply(c, mean, rstd, 1, None, X, 1, presplit=True)      # relu(IN(c)) with the reflect border
    if kind in ("dgrad_ps", "wgrad_ps"):
        c = Buf.empty(N, H, H, C, 0, dev)
        c.t.normal_()
        mean, rstd = ops.in_stats(c)
        G = Buf.empty(N, H, H, C, 2, dev)
        ops.in_apply(c, mean, rstd, 0, None, G, 0, presplit=True)      # a pre-split gradient, zero border 2
        if kind == "dgrad_ps":
            md = PL.wmap_conv_dgrad_s1(w.shape, C)
            out = Buf.empty(N, H, H, C, 1, dev)
            prob = PL.conv_problem(G, 1, k, 1, ops.pack_weight(w, md), md, out)
            fn = lambda: ops.conv([prob])  # noqa: E731
        else:
            c2 = Buf.empty(N, H, H, C, 0, dev)
            c2.t.normal_()
            m2, r2 = ops.in_stats(c2)
            ops.in_apply(c2, m2, r2, 1, None, X, 1, presplit=True)     # relu(IN(.)) with the reflect border
            wprob = PL.wgrad_conv(G, X, 1, k, 1, C)
            dw = torch.empty_like(w)
            wm = PL.wmap_wgrad(w.shape, True, X.c, k)
            fn = lambda: ops.wgrad(wprob, wm, dw)  # noqa: E731
    elif kind in ("fwd", "fwd_stats", "fwd_stats_ps"):
        prob = PL.conv_problem(X, 1, k, 1, ops.pack_weight(w, m), m, Y, bias=torch.zeros(C, device=dev))
        fn = lambda: ops.conv([prob], in_stats=kind != "fwd")  # noqa: E731
    else:
        wprob = PL.wgrad_conv(Y, X, 1, k, 1, C)
        dw = torch.empty_like(w)
        wm = PL.wmap_wgrad(w.shape, True, X.c, k)
        fn = lambda: ops.wgrad(wprob, wm, dw)  # noqa: E731
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    print("done", kind, reps)


if __name__ == "__main__":
    main()
