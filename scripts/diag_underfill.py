"""Tile-config timing (GPU) of the step's f3 launches that give fewer than one 256 x 256 tile per CU: the
discriminator's model.8 input gradient and model.5 forward in the G step (batch 8: 128 tiles of 256 x 256),
and the resblock input gradient's edge strips (18 tiles).  fg_set_f3_tile forces each config; -1 is the
automatic choice.
  python scripts/diag_underfill.py"""
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


def conv_case(N, H, cin, cout, k, s, pad_used, border):
    X = Buf.zeros(N, H, H, cin, border, "cuda")
    X.interior().uniform_(-1, 1)
    w = torch.randn(cout, cin, k, k, device="cuda") * 0.02
    m = PL.wmap_conv_fwd(w.shape, cin)
    Ho = PL.out_size(H, k, s, pad_used)
    Y = Buf.empty(N, Ho, Ho, cout, 0, "cuda")
    prob = PL.conv_problem(X, pad_used, k, s, ops.pack_weight(w, m), m, Y)
    return [prob], 2.0 * N * Ho * Ho * cout * cin * k * k, (X, w, Y)


def main():
    L.load()
    L.set_conv_math("f16x3")
    lib = L.load()
    cases = {
        # D model.8 input gradient in the G step: gy [8, 512, 63, 63] with a zero border 2 -> 64^2 x 256
        "D model.8 dgrad 4x4 512->256 @64 (bs 8)": conv_case(8, 63, 512, 256, 4, 1, 2, 2),
        # D model.5 forward in the G step: 4x4 s2 128->256, 128^2 -> 64^2
        "D model.5 fwd 4x4s2 128->256 @64 (bs 8)": conv_case(8, 128, 128, 256, 4, 2, 1, 1),
        # D model.8 forward in the G step: 4x4 s1 256->512, 64^2 -> 63^2 (250 tiles)
        "D model.8 fwd 4x4 256->512 @63 (bs 8)": conv_case(8, 64, 256, 512, 4, 1, 1, 1),
    }
    for name, (probs, flops, keep) in cases.items():
        for cfg in (-1, 4, 0, 6, 3, 9):
            lib.fg_set_f3_tile(cfg)
            ms = min(time_it(lambda: ops.conv(probs)) for _ in range(3))
            print(f"{name:42s} cfg {cfg:3d} {ms * 1e3:8.1f} us {flops / ms / 1e9:7.1f} TFLOP/s", flush=True)
    lib.fg_set_f3_tile(-1)


if __name__ == "__main__":
    main()
