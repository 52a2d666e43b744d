"""Feasibility timing (GPU) for a phase-merged stride-2 transposed conv: the four sub-pixel phases of
ConvTranspose2d(128, 64, 3, 2, 1, 1) at 256^2 -> 512^2 (bs 8) as ONE 2x2 stride-1 GEMM over the input
(K = 4 taps x 128, N = 4 phases x 64 = 256, zero taps where a phase has fewer) vs the current four-phase
launch (N = 64 per phase).  Timing only: the 2x2 GEMM's output is not scattered to the phases.
  python scripts/diag_phase_merge.py"""
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
    for cin, cout, Hin in ((128, 64, 256), (256, 128, 128)):
        X = Buf.empty(N, Hin, Hin, cin, 1, "cuda")
        X.t.uniform_(-1, 1)
        w = torch.randn(cin, cout, 3, 3, device="cuda") * 0.02
        Y = Buf.empty(N, 2 * Hin, 2 * Hin, cout, 0, "cuda")
        maps = PL.phase_maps(w.shape, 3, 1, X.c)
        probs = PL.phase_problems(X, w.shape, 3, 1, Y, [ops.pack_weight(w, m) for m, _, _ in maps], maps)
        useful = 2.0 * N * (2 * Hin) ** 2 * cout * cin * 9 / 4
        ms = min(time_it(lambda: ops.conv(probs)) for _ in range(3))
        print(f"convT {cin}->{cout} @{Hin} four phases     {ms:8.3f} ms {useful / ms / 1e9:7.1f} useful TFLOP/s", flush=True)
        # merged: 2x2 stride-1 GEMM over X's interior + its bottom/right zero border, N = 4 * cout
        wm = torch.randn(4 * cout, cin, 2, 2, device="cuda") * 0.02
        mm = PL.wmap_conv_fwd(wm.shape, cin)
        Z = Buf.empty(N, Hin, Hin, 4 * cout, 0, "cuda")
        prob = PL.window_problem(X, 0, 0, Hin, Hin, 2, 2, ops.pack_weight(wm, mm), mm, Z, 0, 0)
        ms2 = min(time_it(lambda: ops.conv([prob])) for _ in range(3))
        print(f"convT {cin}->{cout} @{Hin} merged 2x2 GEMM  {ms2:8.3f} ms {useful / ms2 / 1e9:7.1f} useful TFLOP/s "
              f"({2.0 * N * Hin * Hin * 4 * cout * 4 * cin / ms2 / 1e9:.1f} executed)", flush=True)


if __name__ == "__main__":
    main()
