"""The resblock 3x3 256->256 conv (bs 8, 128^2) on the pipelined kernel, fp32 vs FG_PRESPLIT operand, per tile
config (cfg 4 = 256x256 with 8 waves of 32x256; cfg 5 = 256x256 with 8 waves of 64x128: a third fewer LDS fragment
bytes per MFMA, which the pre-split operand allows without splitting A twice), interleaved repeats.
  python scripts/bench_f3_presplit.py [cfgs, default 4,5]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch  # noqa: E402

from floodgan import _lib as L, ops, plans as PL  # noqa: E402
from floodgan.plans import Buf  # noqa: E402
from bench_conv import time_it  # noqa: E402


def main():
    cfgs = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [4, 5]
    lib = L.load()
    N, H, C = 8, 128, 256
    c = Buf.empty(N, H, H, C, 0, "cuda")
    c.t.normal_()
    mean, rstd = ops.in_stats(c)
    xs = {}
    for ps in (False, True):
        xb = Buf.empty(N, H, H, C, 1, "cuda")
        ops.in_apply(c, mean, rstd, 1, None, xb, 1, presplit=ps)
        xs[ps] = xb
    w = torch.randn(C, C, 3, 3, device="cuda") * 0.02
    m = PL.wmap_conv_fwd(w.shape, C)
    wp = ops.pack_weight(w, m)
    Y = Buf.empty(N, H, H, C, 0, "cuda")
    flops = 2.0 * N * H * H * C * C * 9
    res = {}
    outs = {}
    for _ in range(4):
        for cfg in cfgs:
            for ps in (False, True):
                if cfg != 4 and not ps:
                    continue
                lib.fg_set_f3_tile(cfg)
                prob = PL.conv_problem(xs[ps], 1, 3, 1, wp, m, Y)
                res.setdefault((cfg, ps), []).append(time_it(lambda: ops.conv([prob]), reps=20))
                outs[(cfg, ps)] = Y.t.clone()
    lib.fg_set_f3_tile(-1)
    ref = outs[(4, False)]
    for k, v in res.items():
        ms = min(v)
        err = float((outs[k] - ref).norm() / ref.norm())
        print(f"cfg {k[0]} presplit {int(k[1])}: {ms:.4f} ms  {flops / ms / 1e9:6.1f} TFLOP/s  rel diff vs cfg 4 fp32 {err:.1e}",
              flush=True)


if __name__ == "__main__":
    main()
