"""Micro-benchmark (GPU): conv engine kernels at the real bs-8 512^2 geometries, both conv
maths, interleaved in one process, plus an accuracy check vs fp64 on a smaller problem."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from floodgan import _lib as L, ops, plans as PL  # noqa: E402
from floodgan.plans import Buf  # noqa: E402


def nrel(a, b):
    a = a.detach().double().cpu(); b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def make(N, H, Cin, Cout, k, s, p, dev="cuda"):
    X = Buf.empty(N, H, H, Cin, p, dev)
    X.t.uniform_(-1, 1)
    w = torch.randn(Cout, Cin, k, k, device=dev) * 0.02
    m = PL.wmap_conv_fwd(w.shape, Cin)
    Ho = PL.out_size(H, k, s, p)
    Y = Buf.empty(N, Ho, Ho, Cout, 0, dev)
    flops = 2.0 * N * Ho * Ho * Cout * Cin * k * k

    def prob(split):
        wp = ops.pack_weight(w, m, split=split)
        return PL.conv_problem(X, p, k, s, wp, m, Y, bias=torch.zeros(Cout, device=dev))
    return prob, flops, (X, w, Y)

def time_it(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def accuracy(mode, xscale=1.0):
    L.set_conv_math(mode)
    torch.manual_seed(0)
    x = torch.randn(2, 256, 24, 24, dtype=torch.float64) * xscale
    w = torch.randn(256, 256, 3, 3, dtype=torch.float64) * 0.02
    ref = F.conv2d(F.pad(x, (1,) * 4, mode="reflect"), w)
    X = Buf(torch.zeros(2, 26, 26, 256).reshape(-1), 2, 24, 24, 256, 1)
    X.nhwc().copy_(F.pad(x, (1,) * 4, mode="reflect").float().permute(0, 2, 3, 1))
    X = Buf(X.t.cuda(), 2, 24, 24, 256, 1)
    wd = w.float().cuda()
    m = PL.wmap_conv_fwd(wd.shape, 256)
    Y = Buf.empty(2, 24, 24, 256, 0, "cuda")
    ops.conv([PL.conv_problem(X, 1, 3, 1, ops.pack_weight(wd, m), m, Y)])
    torch.cuda.synchronize()
    out = Y.interior().permute(0, 3, 1, 2).cpu()
    # weight gradient of the same conv (gy = ref's shape, random) vs fp64
    gy64 = torch.randn(2, 256, 24, 24, dtype=torch.float64) * xscale
    gw_ref = torch.nn.grad.conv2d_weight(F.pad(x, (1,) * 4, mode="reflect"), w.shape, gy64)
    GY = Buf.empty(2, 24, 24, 256, 0, "cuda")
    GY.interior().copy_(gy64.float().permute(0, 2, 3, 1))
    dw = torch.empty_like(wd)
    ops.wgrad(PL.wgrad_conv(GY, X, 1, 3, 1, 256), PL.wmap_wgrad(wd.shape, True, 256, 3), dw)
    torch.cuda.synchronize()
    # fp32 CPU reference of the same conv for scale
    ref32 = F.conv2d(F.pad(x.float(), (1,) * 4, mode="reflect"), w.float())
    return nrel(out, ref), nrel(dw, gw_ref), nrel(ref32, ref)


def main():
    L.load()
    modes = os.environ.get("MODES", "bf16x6,f16x3").split(",")
    for mode in (["fp32"] + modes if os.environ.get("ACCURACY", "1") == "1" else ()):
        for xs in (1.0, 1e-7, 1e5):
            e, ew, e32 = accuracy(mode, xs)
            print(f"accuracy {mode} (x scale {xs:g}): fwd rel err vs fp64 {e:.3e}, wgrad {ew:.3e} "
                  f"(torch CPU fp32 fwd: {e32:.3e})", flush=True)
    cases = {"resblock 3x3 256->256 @128": (8, 128, 256, 256, 3, 1, 1),
             "conv2 3x3s2 64->128 @512": (8, 512, 64, 128, 3, 2, 1),
             "D model.8 4x4 256->512 @64 (2N)": (16, 64, 256, 512, 4, 1, 1),
             "3x3 128->64 @256 (N=64 class)": (8, 256, 128, 64, 3, 1, 1),
             "deconv3_content 7x7 64->27 @512": (8, 512, 64, 27, 7, 1, 3)}
    tiles = [int(t) for t in os.environ.get("TILES", "0,1,2,3,4,5,6,7,8").split(",")]
    for name, c in cases.items():
        mk, flops, keep = make(*c)
        variants = [("fp32", -1, False)] + [(md, t, True) for md in modes for t in tiles]
        res = {}
        for rep in range(2):
            for mode, tile, split in variants:
                L.set_conv_math(mode)
                L.set_fwd_tile(tile)
                prob = mk(split)
                ms = time_it(lambda: ops.conv([prob]))
                res.setdefault((mode, tile, split), []).append(ms)
        L.set_fwd_tile(-1)
        for (mode, tile, split), v in res.items():
            ms = min(v)
            tag = f"{mode} tile {tile:2d} {'presplit' if split else 'onfly'}" if mode != "fp32" else "fp32"
            print(f"{name:36s} {tag:26s} {ms:8.3f} ms  {flops / ms / 1e9:7.1f} TFLOP/s", flush=True)
        # weight gradient of the same conv
        X, w, Y = keep
        Y.t.uniform_(-1, 1)
        N, H, Cin, Cout, k, s_, p_ = c
        wprob = PL.wgrad_conv(Y, X, p_, k, s_, Cout)
        dw = torch.empty_like(w)
        wm = PL.wmap_wgrad(w.shape, True, X.c, k)
        wtiles = [int(t) for t in os.environ.get("WTILES", "-1").split(",")]
        wvariants = [("fp32", -1)] + [(md, t) for md in modes for t in wtiles]
        res = {}
        for rep in range(2):
            for mode, t in wvariants:
                L.set_conv_math(mode)
                L.set_wgrad_tile(t)
                res.setdefault((mode, t), []).append(time_it(lambda: ops.wgrad(wprob, wm, dw)))
        L.set_conv_math("fp32")
        L.set_wgrad_tile(-1)
        ops.wgrad(wprob, wm, dw)
        ref = dw.clone()
        for md in modes:
            L.set_conv_math(md)
            for t in wtiles:
                L.set_wgrad_tile(t)
                ops.wgrad(wprob, wm, dw)
                torch.cuda.synchronize()
                print(f"{name + ' wgrad':36s} {md} tile {t} vs fp32 rel diff {nrel(dw, ref):.2e}")
        L.set_wgrad_tile(-1)
        for (mode, t), v in res.items():
            ms = min(v)
            print(f"{name + ' wgrad':36s} {mode:7s} tile {t:2d} {ms:8.3f} ms  {flops / ms / 1e9:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
