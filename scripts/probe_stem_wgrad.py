"""Which kernel the stem's weight gradient (7x7, 12 -> 64 channels, n_a = 64) takes: run it once (bs 2, 128^2) under
rocprofv3 --kernel-trace and print the problem as the library sees it."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
import torch  # noqa: E402

from floodgan import _lib as L, ops, plans as PL  # noqa: E402
from floodgan.plans import Buf  # noqa: E402

lib = L.load()
N, H = 2, 128
gc1 = Buf.empty(N, H, H, 64, 0, "cuda")
gc1.t.normal_()
X0 = Buf.empty(N, H, H, 12, 3, "cuda")
X0.t.normal_()
prob = PL.wgrad_conv(gc1, X0, 3, 7, 1, 64)
print("eligible", PL.f3_wgrad_eligible(prob), "wgrad_f16x3", L.wgrad_f16x3(), "f3_on", L.wgrad_f3_on(),
      {k: prob[k] for k in ("n_a", "kh", "j_valid", "sxn", "sxa", "sxb", "sxr")})
dw = torch.empty(64, 12, 7, 7, device="cuda")
ops.wgrad(prob, PL.wmap_wgrad(dw.shape, True, 12, 7), dw)
torch.cuda.synchronize()
print("done")
