"""A/B (GPU) of the content-head weight gradient's split count (ops.WIN_WGRAD_SPLITS: workgroups = 7 x splits,
multiples of 8 keep a split's 7 kernel rows on one XCD) at bs 8, 512^2; results compared against splits 144.
  python scripts/diag_wgrad_win_splits.py"""
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
    X = Buf.zeros(N, 512, 512, 64, 3, "cuda")
    X.t.uniform_(-1, 1)
    GY = Buf.zeros(N, 512, 512, 32, 6, "cuda")
    GY.interior()[..., :27].uniform_(-1e-3, 1e-3)
    prob = PL.wgrad_conv(GY, X, 3, 7, 1, 27)
    assert ops.wgrad_win_eligible(prob)
    wm = PL.wmap_wgrad((27, 64, 7, 7), True, X.c, 7)
    flops = 2.0 * N * 512 * 512 * 27 * 64 * 49
    ref = None
    for sp in [int(v) for v in os.environ.get("SPLITS", "144,72,288,216").split(",")] * 2:
        ops.WIN_WGRAD_SPLITS = sp
        dw = torch.empty((27, 64, 7, 7), dtype=torch.float32, device="cuda")
        ops.wgrad(prob, wm, dw)
        torch.cuda.synchronize()
        if ref is None:
            ref = dw.clone()
        d = float((dw - ref).norm() / ref.norm())
        ms = min(time_it(lambda: ops.wgrad(prob, wm, dw)) for _ in range(3))
        print(f"content wgrad splits {sp:4d} {ms * 1e3:8.1f} us {flops / ms / 1e9:7.1f} TFLOP/s  rel diff vs 144 {d:.1e}",
              flush=True)
    ops.WIN_WGRAD_SPLITS = 216


if __name__ == "__main__":
    main()
