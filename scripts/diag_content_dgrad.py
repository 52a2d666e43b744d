"""A/B (GPU) of the content head's input gradient (7x7, 27(32) -> 64 over the 518^2 padded domain, bs 8):
the pipelined f16x3 kernel (cfg 7, 256x64 tiles: every gy pixel re-gathered once per tap) vs the
row-strip window kernel (conv_win<32, 7, 4>: each kernel row's strip staged once, the 7 taps as shifted
reads), outputs compared.
  python scripts/diag_content_dgrad.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch  # noqa: E402

from bench_conv import time_it  # noqa: E402
from floodgan import _lib as L, ops, plans as PL  # noqa: E402
from floodgan.plans import Buf  # noqa: E402


def main():
    L.load()
    L.set_conv_math("f16x3")
    N = int(os.environ.get("N", "8"))
    torch.manual_seed(0)
    w = torch.randn(27, 64, 7, 7, device="cuda") * 0.02
    gcl = Buf.zeros(N, 512, 512, 32, 6, "cuda")
    gcl.interior()[..., :27].uniform_(-1, 1)
    m = PL.wmap_conv_dgrad_s1(w.shape, 32)
    wp = ops.pack_weight(w, m)
    flops = 2.0 * N * 518 * 518 * 64 * 27 * 49
    outs = {}
    for mode in ("f3", "win"):
        Y = Buf.empty(N, 518, 518, 64, 0, "cuda")
        prob = PL.conv_problem(gcl, 6, 7, 1, wp, m, Y)
        if mode == "f3":
            fn = lambda: ops.conv([prob])  # noqa: E731
        else:
            fn = lambda: ops.conv_win(prob)  # noqa: E731
        fn()
        outs[mode] = Y.t.clone()
        ms = min(time_it(fn) for _ in range(3))
        print(f"content dgrad 7x7 32->64 @518 bs {N} {mode:4s} {ms:8.3f} ms {flops / ms / 1e9:7.1f} TFLOP/s",
              flush=True)
    d = (outs["f3"] - outs["win"]).norm() / outs["f3"].norm()
    print(f"rel diff win vs f3 {float(d):.2e}")


if __name__ == "__main__":
    main()
