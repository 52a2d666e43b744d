"""The stem's weight gradient (7x7 over the packed 9-channel input -> 64, bs 8, 512^2), interleaved A/B: the strip
kernel (conv_stem.hip, its own 256 splits) against the register-staged x6 kernel (forced with fg_set_wgrad_tile 2 and
the generic split layout); outputs compared, and both against an fp64 reference of one image's weight gradient.
  python scripts/bench_stem_wgrad.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from floodgan import _lib as L, ops, plans as PL  # noqa: E402
from floodgan._lib import FG_PAD_REFLECT  # noqa: E402
from floodgan.plans import Buf  # noqa: E402
from bench_conv import time_it  # noqa: E402


def main():
    L.load()
    L.set_conv_math("f16x3")
    N, H = 8, 512
    torch.manual_seed(0)
    x = torch.rand(N, 9, H, H, device="cuda") * 2 - 1
    gc1 = Buf.empty(N, H, H, 64, 0, "cuda")
    gc1.t.normal_()
    X0 = Buf.empty(N, H, H, 9, 3, "cuda")
    ops.pack_input(x, 9, None, 0, X0, 0, N, FG_PAD_REFLECT)
    prob = PL.wgrad_conv(gc1, X0, 3, 7, 1, 64)
    dw = torch.empty(64, 9, 7, 7, device="cuda")
    wm = PL.wmap_wgrad(dw.shape, True, 9, 7)
    out = {}
    for rep in range(2):
        for kind in ("stem", "x6"):
            L.load().fg_set_wgrad_tile(-1 if kind == "stem" else 2)
            ms = time_it(lambda: ops.wgrad(prob, wm, dw), reps=5)
            out[kind] = dw.clone()
            print(f"stem wgrad {kind:4s} ({ops.LAST_WGRAD_KERNEL}): {ms * 1e3:8.1f} us per wgrad + reduce, "
                  f"{2 * N * H * H * 64 * 441 / ms / 1e9:7.1f} TFLOP/s", flush=True)
    L.load().fg_set_wgrad_tile(-1)
    # fp64 reference over the whole batch
    gy = gc1.interior().permute(0, 3, 1, 2).double().cpu()
    ref = torch.nn.grad.conv2d_weight(F.pad(x.double().cpu(), (3,) * 4, mode="reflect"), dw.shape, gy)
    for kind, v in out.items():
        print(f"{kind}: rel err vs fp64 {float((v.double().cpu() - ref).norm() / ref.norm()):.2e}")
    print(f"stem vs x6 rel diff {float((out['stem'] - out['x6']).norm() / out['x6'].norm()):.2e}", flush=True)


if __name__ == "__main__":
    main()
