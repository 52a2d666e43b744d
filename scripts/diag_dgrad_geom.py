"""Why is the resblock input-gradient conv (3x3 over the border-2 gradient, 130x130 outputs) slower than
the forward conv (128x128 outputs) at the same K and N?  Times the pipelined f16x3 kernel over output
widths 128 / 130 / 132 and buffer borders 1 / 2, and the k-walk orders (fg_set_f3_order).
  python scripts/diag_dgrad_geom.py"""
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


def case(N, H, pad, pad_used, C=256, k=3):
    X = Buf.empty(N, H, H, C, pad, "cuda")
    X.t.uniform_(-1, 1)
    w = torch.randn(C, C, k, k, device="cuda") * 0.02
    m = PL.wmap_conv_fwd(w.shape, C)
    Ho = PL.out_size(H, k, 1, pad_used)
    Y = Buf.empty(N, Ho, Ho, C, 0, "cuda")
    wp = ops.pack_weight(w, m)
    prob = PL.conv_problem(X, pad_used, k, 1, wp, m, Y)
    flops = 2.0 * N * Ho * Ho * C * C * k * k
    return prob, flops, (X, w, Y, wp)


def main():
    L.load()
    L.set_conv_math("f16x3")
    lib = L.load()
    cases = {"fwd: 128 px out, border 1": (8, 128, 1, 1), "dgrad: 130 px out, border 2": (8, 128, 2, 2),
             "130 px out from 130 px in, border 1": (8, 130, 1, 1), "132 px out (in 130, border 2)": (8, 130, 2, 2),
             "128 px out from border-2 buffer": (8, 128, 2, 1), "126 px out (in 128 border 0)": (8, 128, 0, 0)}
    for order in (7, 6, 5, 4, 3):
        lib.fg_set_f3_order(order)
        for name, c in cases.items():
            prob, flops, keep = case(*c)
            ms = min(time_it(lambda: ops.conv([prob])) for _ in range(3))
            print(f"order {order}  {name:40s} {ms:8.3f} ms {flops / ms / 1e9:7.1f} TFLOP/s", flush=True)
    lib.fg_set_f3_order(7)


if __name__ == "__main__":
    main()
