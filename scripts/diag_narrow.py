"""Timing (GPU) of the step's narrow-N convs (N <= 32, which the pipelined kernel does not take by default) on
the register-staged x6 kernel vs the pipelined kernel forced to its 128 x 64 tile (cfg 9), bs 8 512^2:
the attention head's 1x1 conv 64 -> 10 and the discriminator's input gradient restricted to the 3 generated
channels (four stride-2 phases, 2 x 2 taps x 64 channels each, written NCHW and accumulated).
  python scripts/diag_narrow.py"""
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
    N, H = 8, 512
    torch.manual_seed(0)
    # attention head: 1x1 64 -> 10 into the 16-channel logits buffer
    ad2 = Buf.empty(N, H, H, 64, 0, "cuda")
    ad2.t.uniform_(-1, 1)
    w = torch.randn(10, 64, 1, 1, device="cuda") * 0.1
    b = torch.randn(10, device="cuda")
    m = PL.wmap_conv_fwd(w.shape, 64)
    al = Buf.zeros(N, H, H, 16, 0, "cuda")
    att = [PL.conv_problem(ad2, 0, 1, 1, ops.pack_weight(w, m), m, al, bias=b)]
    # D model.0 input gradient, channels 9..11 of 12, into an NCHW [N, 3, H, W] tensor (accumulated)
    w0 = torch.randn(64, 12, 4, 4, device="cuda") * 0.02
    ge0 = Buf.zeros(N, H // 2, H // 2, 64, 1, "cuda")
    ge0.interior().uniform_(-1, 1)
    gout = torch.zeros(N, 3, H, H, device="cuda")
    maps = PL.phase_maps(w0.shape, 4, 1, 64, n_base=9, n_out=3)
    dgr = PL.phase_problems(ge0, w0.shape, 4, 1, None, [ops.pack_weight(w0, mm) for mm, _, _ in maps], maps,
                            y_nchw=(gout.view(-1), 3, H, H), accumulate=1)
    for name, probs, out in (("attention head 1x1 64->10", att, al.t), ("D model.0 input grad, 3 channels", dgr, gout)):
        res = {}
        for cfg in (-1, 9, 7):
            lib.fg_set_f3_tile(cfg)
            out.zero_()
            ops.conv(probs)
            torch.cuda.synchronize()
            res[cfg] = out.clone()
            ms = min(time_it(lambda: ops.conv(probs)) for _ in range(3))
            d = float((res[cfg] - res[-1]).norm() / res[-1].norm())
            print(f"{name:34s} {'x6 (default)' if cfg < 0 else f'pipelined cfg {cfg}':18s} {ms * 1e3:8.1f} us  "
                  f"rel diff vs x6 {d:.2e}", flush=True)
        lib.fg_set_f3_tile(-1)


if __name__ == "__main__":
    main()
