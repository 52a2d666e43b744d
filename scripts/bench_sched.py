"""Interleaved A/B (GPU) of a pipelined-forward-kernel switch (fg_set_f3_sched / fg_set_f3_order)
on the bs-8 512^2 forward geometries, with the relative difference between the results.
  python scripts/bench_sched.py [sched|order] [values]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch  # noqa: E402

from floodgan import _lib as L, ops, plans as PL  # noqa: E402
from floodgan.plans import Buf  # noqa: E402
from bench_conv import make, nrel, time_it  # noqa: E402


SW = sys.argv[1] if len(sys.argv) > 1 else "sched"
VALS = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1, 2]
DEFAULT = {"sched": -1, "order": 7}[SW]


def setsw(v):
    getattr(L.load(), "fg_set_f3_" + SW)(v)


def ab(name, run, out, flops, reps=3):
    res, outs = {v: [] for v in VALS}, {}
    for _ in range(reps):
        for v in VALS:
            setsw(v)
            res[v].append(time_it(run))
    for v in VALS:
        setsw(v)
        out.zero_()
        run()
        torch.cuda.synchronize()
        outs[v] = out.clone()
    setsw(DEFAULT)
    for v in VALS:
        ms = min(res[v])
        print(f"{name:36s} {SW} {v} {ms:8.3f} ms {flops / ms / 1e9:7.1f} TFLOP/s"
              f"  rel diff {nrel(outs[v], outs[VALS[0]]):.2e}", flush=True)


def main():
    L.load()
    L.set_conv_math("f16x3")
    cases = {"resblock 3x3 256->256 @128": (8, 128, 256, 256, 3, 1, 1),
             "conv3 3x3s2 128->256 @256": (8, 256, 128, 256, 3, 2, 1),
             "conv2 3x3s2 64->128 @512": (8, 512, 64, 128, 3, 2, 1),
             "D model.8 4x4 256->512 @64 (2N)": (16, 64, 256, 512, 4, 1, 1),
             "D model.5 4x4s2 128->256 @128 (2N)": (16, 128, 128, 256, 4, 2, 1),
             "3x3 128->64 @256 (N=64 class)": (8, 256, 128, 64, 3, 1, 1)}
    for name, c in cases.items():
        mk, flops, keep = make(*c)
        X, w, Y = keep
        prob = mk(True)
        ab(name, lambda: ops.conv([prob]), Y.t, flops)
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
        ab(name, lambda: ops.conv(probs), Y.t, flops)


if __name__ == "__main__":
    main()
