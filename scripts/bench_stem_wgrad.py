"""The stem (7x7 over the packed 9-channel input -> 64, bs 8, 512^2), interleaved A/B of the strip kernels
(conv_stem.hip) against the register-staged x6 kernels: the weight gradient (the strip kernel's own 256 splits vs the x6
kernel forced with fg_set_wgrad_tile 2 on the generic split layout) and the forward with the statistics epilogue
(FLOODGAN_STEM_FWD 1 / 0); outputs compared, and the weight gradients against fp64.
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
    # forward (+ statistics epilogue; the x6 path computes the statistics in a separate pass)
    w = torch.randn(64, 9, 7, 7, device="cuda") * 0.05
    m = PL.wmap_conv_fwd(w.shape, 9)
    Y = Buf.empty(N, H, H, 64, 0, "cuda")
    fprob = PL.conv_problem(X0, 3, 7, 1, ops.pack_weight(w, m), m, Y, bias=torch.zeros(64, device="cuda"))
    fout = {}
    for rep in range(2):
        for on in ("1", "0"):
            os.environ["FLOODGAN_STEM_FWD"] = on
            def run():
                st = ops.conv([fprob], in_stats=True)
                return st if st is not None else ops.in_stats(Y)
            ms = time_it(run, reps=5)
            fout[on] = Y.t.clone()
            print(f"stem fwd + stats, strip kernel {on} ({ops.LAST_CONV_KERNEL}): {ms * 1e3:8.1f} us, "
                  f"{2 * N * H * H * 64 * 441 / ms / 1e9:7.1f} TFLOP/s", flush=True)
    os.environ.pop("FLOODGAN_STEM_FWD")
    print(f"stem fwd strip vs x6 rel diff {float((fout['1'] - fout['0']).norm() / fout['0'].norm()):.2e}", flush=True)
    # fp64 reference over the whole batch
    gy = gc1.interior().permute(0, 3, 1, 2).double().cpu()
    ref = torch.nn.grad.conv2d_weight(F.pad(x.double().cpu(), (3,) * 4, mode="reflect"), dw.shape, gy)
    for kind, v in out.items():
        print(f"{kind}: rel err vs fp64 {float((v.double().cpu() - ref).norm() / ref.norm()):.2e}")
    print(f"stem vs x6 rel diff {float((out['stem'] - out['x6']).norm() / out['x6'].norm()):.2e}", flush=True)


if __name__ == "__main__":
    main()
