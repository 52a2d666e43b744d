"""Tile configs of the pipelined kernel on the step's narrow-N 4-phase transposed convs with FG_PRESPLIT operands and
the statistics epilogue (deconv2 128->64 256^2->512^2, deconv1 256->128 128^2->256^2, bs 8), interleaved repeats:
  python scripts/bench_narrow_cfg.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch  # noqa: E402

from floodgan import _lib as L, ops, plans as PL  # noqa: E402
from floodgan.plans import Buf  # noqa: E402
from bench_conv import time_it  # noqa: E402


def case(N, H, cin, cout):
    c = Buf.empty(N, H, H, cin, 0, "cuda")
    c.t.normal_()
    mean, rstd = ops.in_stats(c)
    X = Buf.empty(N, H, H, cin, 1, "cuda")
    ops.in_apply(c, mean, rstd, 1, None, X, 0, presplit=True)
    w = torch.randn(cin, cout, 3, 3, device="cuda") * 0.02
    Y = Buf.empty(N, 2 * H, 2 * H, cout, 0, "cuda")
    maps = PL.phase_maps(w.shape, 3, 1, X.c)
    wps = [ops.pack_weight(w, m) for m, _, _ in maps]
    probs = PL.phase_problems(X, w.shape, 3, 1, Y, wps, maps, bias=torch.zeros(cout, device="cuda"))
    flops = 2.0 * N * (2 * H) ** 2 * cout * cin * 9 / 4
    return (lambda st=True: ops.conv(probs, in_stats=st)), flops, (X, w, Y, c)


def main():
    lib = L.load()
    cases = {"deconv2 128->64 (N=64)": (case(8, 256, 128, 64), [-1, 7, 10, 9, 6]),
             "deconv1 256->128 (N=128)": (case(8, 128, 256, 128), [-1, 6, 11, 4, 5])}
    for name, ((fn, flops, keep), cfgs) in cases.items():
        res = {}
        for _ in range(3):
            for cfg in cfgs:
                L.set_f3_tile(cfg)
                for st in (True, False):
                    res.setdefault((cfg, st), []).append(time_it(lambda: fn(st), reps=10))
        L.set_f3_tile(-1)
        for cfg in cfgs:
            for st in (True, False):
                ms = min(res[(cfg, st)])
                print(f"{name:28s} cfg {cfg:3d} stats {int(st)}: {ms:.4f} ms  {flops / ms / 1e9:6.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
