"""The stem's weight gradient (7x7 over the packed 9-channel input -> 64, bs 8, 512^2): the register-staged kernel on
the 9-channel rows vs the pipelined kernel's 64-row tile on a 12-channel (zero-padded) copy:
  python scripts/bench_stem_wgrad.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch  # noqa: E402

from floodgan import _lib as L, ops, plans as PL  # noqa: E402
from floodgan._lib import FG_PAD_REFLECT  # noqa: E402
from floodgan.plans import Buf  # noqa: E402
from bench_conv import time_it  # noqa: E402


def main():
    L.load()
    N, H = 8, 512
    x = torch.rand(N, 9, H, H, device="cuda") * 2 - 1
    gc1 = Buf.empty(N, H, H, 64, 0, "cuda")
    gc1.t.normal_()
    res = {}
    for C in (9, 12):
        X0 = Buf.empty(N, H, H, C, 3, "cuda")
        ops.pack_input(x, 9, None, 0, X0, 0, N, FG_PAD_REFLECT)
        prob = PL.wgrad_conv(gc1, X0, 3, 7, 1, 64)
        dw = torch.empty(64, 9, 7, 7, device="cuda")
        wm = PL.wmap_wgrad(dw.shape, True, C, 7)
        res[C] = (time_it(lambda: ops.wgrad(prob, wm, dw), reps=5), dw.clone())
        res[(C, "pack")] = time_it(lambda: ops.pack_input(x, 9, None, 0, X0, 0, N, FG_PAD_REFLECT), reps=5)
    err = float((res[12][1] - res[9][1]).norm() / res[9][1].norm())
    print(f"stem wgrad 9 ch (register-staged): {res[9][0]:.3f} ms; 12 ch (pipelined 64-row tile): {res[12][0]:.3f} ms; "
          f"pack 9 ch {res[(9, 'pack')]:.3f} ms, 12 ch {res[(12, 'pack')]:.3f} ms; rel diff {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
