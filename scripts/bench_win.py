"""Timing (GPU) of the row-strip window kernel on the content head's forward (7x7 64 -> 27 at 512^2) and input
gradient (7x7 27(32) -> 64 over 518^2), bs 8 (round 4: its LDS-DMA form, one barrier per tap, was replaced by the
register-staged one, profiles/round4/r4c_ab_win.log; round 5 keeps only the two-workgroup kernels).
  python scripts/bench_win.py"""
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
    N = 8
    torch.manual_seed(0)
    ad2 = Buf.empty(N, 512, 512, 64, 3, "cuda")
    ad2.t.uniform_(-1, 1)
    w = torch.randn(27, 64, 7, 7, device="cuda") * 0.02
    m = PL.wmap_conv_fwd(w.shape, 64)
    cl = Buf.empty(N, 512, 512, 32, 0, "cuda")
    fwd = PL.conv_problem(ad2, 3, 7, 1, ops.pack_weight(w, m), m, cl)
    gcl = Buf.zeros(N, 512, 512, 32, 6, "cuda")
    gcl.interior()[..., :27].uniform_(-1, 1)
    md = PL.wmap_conv_dgrad_s1(w.shape, 32)
    Y = Buf.empty(N, 518, 518, 64, 0, "cuda")
    dgr = PL.conv_problem(gcl, 6, 7, 1, ops.pack_weight(w, md), md, Y)
    for name, prob, out, flops in (("content fwd 7x7 64->27 @512", fwd, cl, 2.0 * N * 512 * 512 * 27 * 64 * 49),
                                   ("content dgrad 7x7 27->64 @518", dgr, Y, 2.0 * N * 518 * 518 * 64 * 27 * 49)):
        out.t.zero_()
        ms = min(time_it(lambda: ops.conv_win(prob)) for _ in range(5))
        print(f"{name:32s} {ms * 1e3:8.1f} us {flops / ms / 1e9:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
