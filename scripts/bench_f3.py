"""Micro-benchmark (GPU) of the LDS-DMA pipelined f16x3 forward kernel (conv_f3.hip) against
the register-staged f16x3 kernel, at the real bs-8 512^2 geometries: per tile config, time and
relative difference to the register-staged result.
  F3_TILES=0,1,2,3 python scripts/bench_f3.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
import torch  # noqa: E402

from floodgan import _lib as L, ops, plans as PL  # noqa: E402
from bench_conv import make, nrel, time_it  # noqa: E402


def main():
    L.load()
    L.set_conv_math("f16x3")
    cases = {"resblock 3x3 256->256 @128": (8, 128, 256, 256, 3, 1, 1),
             "conv3 3x3s2 128->256 @256": (8, 256, 128, 256, 3, 2, 1),
             "conv2 3x3s2 64->128 @512": (8, 512, 64, 128, 3, 2, 1),
             "D model.8 4x4 256->512 @64 (2N)": (16, 64, 256, 512, 4, 1, 1),
             "D model.5 4x4s2 128->256 @128 (2N)": (16, 128, 128, 256, 4, 2, 1),
             "3x3 128->64 @256 (N=64 class)": (8, 256, 128, 64, 3, 1, 1)}
    tiles = [int(t) for t in os.environ.get("F3_TILES", "-1,0,1,2,3,4,5,6").split(",")]
    for name, c in cases.items():
        mk, flops, keep = make(*c)
        X, w, Y = keep
        prob = mk(True)
        L.set_f3_tile(-2)
        ops.conv([prob])
        ref = Y.t.clone()
        res = {}
        for rep in range(2):
            for t in [-2] + tiles:
                L.set_f3_tile(t)
                res.setdefault(t, []).append(time_it(lambda: ops.conv([prob])))
        for pers in (0, 1, 0, 1):
            L.load().fg_set_f3_persistent(pers)
            L.set_f3_tile(-1)
            ms = time_it(lambda: ops.conv([prob]))
            print(f"{name:36s} {'f3 persistent ' + str(pers):16s} {ms:8.3f} ms {flops / ms / 1e9:7.1f} TFLOP/s", flush=True)
        L.load().fg_set_f3_persistent(1)
        for t in [-2] + tiles:
            L.set_f3_tile(t)
            Y.t.zero_()
            ops.conv([prob])
            torch.cuda.synchronize()
            d = nrel(Y.t, ref)
            ms = min(res[t])
            tag = "register-staged" if t == -2 else f"f3 tile {t}"
            print(f"{name:36s} {tag:16s} {ms:8.3f} ms {flops / ms / 1e9:7.1f} TFLOP/s  rel diff {d:.2e}", flush=True)
    L.set_f3_tile(-1)
    # transposed-conv phase batches (deconv1 256->128 @128->256, deconv2 128->64 @256->512)
    from floodgan.plans import Buf
    for name, (cin, cout, Hin) in {"deconv1 ConvT 256->128 @128": (256, 128, 128),
                                   "deconv2 ConvT 128->64 @256": (128, 64, 256)}.items():
        N = 8
        X = Buf.empty(N, Hin, Hin, cin, 1, "cuda")
        X.t.uniform_(-1, 1)
        w = torch.randn(cin, cout, 3, 3, device="cuda") * 0.02
        Y = Buf.empty(N, 2 * Hin, 2 * Hin, cout, 0, "cuda")
        maps = PL.phase_maps(w.shape, 3, 1, X.c)
        probs = PL.phase_problems(X, w.shape, 3, 1, Y, [ops.pack_weight(w, m) for m, _, _ in maps], maps)
        flops = 2.0 * N * (2 * Hin) ** 2 * cout * cin * 9 / 4
        L.set_f3_tile(-2)
        ops.conv(probs)
        ref = Y.t.clone()
        for pers in (-1, 0, 1, -1, 0, 1):
            if pers < 0:
                L.set_f3_tile(-2)
            else:
                L.set_f3_tile(-1)
                L.load().fg_set_f3_persistent(pers)
            ms = time_it(lambda: ops.conv(probs))
            tag = "register-staged" if pers < 0 else f"f3 persistent {pers}"
            print(f"{name:36s} {tag:16s} {ms:8.3f} ms {flops / ms / 1e9:7.1f} TFLOP/s  rel diff {nrel(Y.t, ref):.2e}",
                  flush=True)
        L.set_f3_tile(-1)
        L.load().fg_set_f3_persistent(1)
    # weight gradients: pipelined f16x3 kernel vs the register-staged one
    for name, c in {"resblock wgrad 3x3 256x256 @128": (8, 128, 256, 256, 3, 1, 1),
                    "D model.8 wgrad 4x4 256->512 @64 (2N)": (16, 64, 256, 512, 4, 1, 1),
                    "conv3 wgrad 3x3s2 128->256 @256": (8, 256, 128, 256, 3, 2, 1),
                    "conv2 wgrad 3x3s2 64->128 @512": (8, 512, 64, 128, 3, 2, 1),
                    "D model.2 wgrad 4x4s2 64->128 @256 (2N)": (16, 256, 64, 128, 4, 2, 1)}.items():
        mk, flops, keep = make(*c)
        X, w, Y = keep
        Y.t.uniform_(-1, 1)
        N, H, Cin, Cout, k, s_, p_ = c
        wprob = PL.wgrad_conv(Y, X, p_, k, s_, Cout)
        wm = PL.wmap_wgrad(w.shape, True, X.c, k)
        dw = torch.empty_like(w)
        res = {}
        for rep in range(2):
            for on in (0, 1, 2):
                L.set_wgrad_f3(on)
                res.setdefault(on, []).append(time_it(lambda: ops.wgrad(wprob, wm, dw)))
        outs = {}
        for on in (0, 1, 2):
            L.set_wgrad_f3(on)
            ops.wgrad(wprob, wm, dw)
            torch.cuda.synchronize()
            outs[on] = dw.clone()
        for on in (0, 1, 2):
            ms = min(res[on])
            print(f"{name:36s} {('f3 sched ' + str(on - 1)) if on else 'register-staged':16s} {ms:8.3f} ms {flops / ms / 1e9:7.1f} TFLOP/s"
                  f"  rel diff {nrel(outs[on], outs[0]):.2e}", flush=True)
        L.set_wgrad_f3(2)
    # the row-strip window kernel on the content head (fwd, and the input gradient's geometry)
    from floodgan.plans import Buf
    dev = "cuda"
    for name, (cin_alloc, nout, pad) in {"content fwd 7x7 64->27 @512": (64, 27, 3),
                                         "content dgrad 7x7 27(32)->64 @518": (32, 64, 6)}.items():
        N, H = 8, 512
        X = Buf.empty(N, H, H, cin_alloc, pad, dev)
        X.t.uniform_(-1, 1)
        if pad == 3:
            w = torch.randn(nout, cin_alloc, 7, 7, device=dev) * 0.02
            m = PL.wmap_conv_fwd(w.shape, cin_alloc)
            Ho = H
        else:
            w = torch.randn(27, nout, 7, 7, device=dev) * 0.02
            m = PL.wmap_conv_dgrad_s1(w.shape, cin_alloc)
            Ho = H + 6
        Y = Buf.empty(N, Ho, Ho, 32 if nout <= 32 else nout, 0, dev)
        prob = PL.conv_problem(X, pad, 7, 1, ops.pack_weight(w, m), m, Y)
        flops = 2.0 * N * Ho * Ho * nout * cin_alloc * 49
        for use in (False, True, False, True):
            ops.USE_WIN = use
            ms = time_it(lambda: ops.conv([prob]))
            print(f"{name:36s} {'window' if use else 'im2col':16s} {ms:8.3f} ms {flops / ms / 1e9:7.1f} TFLOP/s",
                  flush=True)
        ops.USE_WIN = True
    # content-head weight gradient: row-strip kernel vs the generic f16x3 one
    N, H = 8, 512
    X = Buf.empty(N, H, H, 64, 3, dev)
    X.t.uniform_(-1, 1)
    GY = Buf.empty(N, H, H, 32, 6, dev)
    GY.t.uniform_(-1, 1)
    wprob = PL.wgrad_conv(GY, X, 3, 7, 1, 27)
    wm = PL.wmap_wgrad((27, 64, 7, 7), True, 64, 7)
    dw = torch.empty(27, 64, 7, 7, device=dev)
    flops = 2.0 * N * H * H * 27 * 64 * 49
    outs = {}
    for use in (False, True, False, True):
        ops.USE_WIN = use
        ms = time_it(lambda: ops.wgrad(wprob, wm, dw))
        outs[use] = dw.clone()
        print(f"{'content wgrad 7x7 64->27 @512':36s} {'window' if use else 'im2col':16s} {ms:8.3f} ms "
              f"{flops / ms / 1e9:7.1f} TFLOP/s  rel diff {nrel(outs[use], outs[False]):.2e}", flush=True)
    ops.USE_WIN = True


if __name__ == "__main__":
    main()
