"""Timing (GPU) of the resblock input gradient's pieces at bs 8, 128^2, C 256 (executor._dgrad_s1_padded):
the 128-px interior launch and the four edge strips' launch, the strips on their default route and forced
onto each pipelined tile config; result of every route compared with the default.
  python scripts/diag_strips.py"""
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
    lib = L.load()
    N, H, C = 8, 128, 256
    torch.manual_seed(0)
    gy = Buf.zeros(N, H, H, C, 2, "cuda")
    gy.interior().uniform_(-1, 1)
    w = torch.randn(C, C, 3, 3, device="cuda") * 0.02
    m = PL.wmap_conv_dgrad_s1(w.shape, C)
    wp = ops.pack_weight(w, m)
    out = Buf.zeros(N, H, H, C, 1, "cuda")
    interior = [PL.conv_problem(gy, 1, 3, 1, wp, m, out)]
    strips = [PL.window_problem(gy, 0, -2, 1, H + 2, 1, 3, wp, m, out, -1, -1, w_row0=2),
              PL.window_problem(gy, H - 1, -2, 1, H + 2, 1, 3, wp, m, out, H, -1, w_row0=0)]
    for col, x0, ox in ((2, 0, -1), (0, H - 1, H)):
        ms = PL.wmap_conv_dgrad_s1_taps(w.shape, C, (0, 1, 2), (col,))
        strips.append(PL.window_problem(gy, -1, x0, H, 1, 3, 1, ops.pack_weight(w, ms), ms, out, 0, ox))
    sflops = 2.0 * N * (2 * (H + 2) + 2 * H) * C * 3 * C
    ti = min(time_it(lambda: ops.conv(interior)) for _ in range(3))
    print(f"interior 128x128 (512 tiles)          {ti * 1e3:8.1f} us", flush=True)
    ref = None
    for cfg in (-1, 9, 7, 4, -2):
        lib.fg_set_f3_tile(cfg)
        out.t.zero_()
        ops.conv(strips)
        torch.cuda.synchronize()
        o = out.t.clone()
        ref = o if ref is None else ref
        ts = min(time_it(lambda: ops.conv(strips)) for _ in range(3))
        name = {-1: "default route", -2: "register-staged x6"}.get(cfg, f"pipelined cfg {cfg}")
        print(f"strips ({name:20s})          {ts * 1e3:8.1f} us {sflops / ts / 1e9:7.1f} TFLOP/s  rel diff vs "
              f"default {float((o - ref).norm() / ref.norm()):.2e}", flush=True)
    lib.fg_set_f3_tile(-1)


if __name__ == "__main__":
    main()
