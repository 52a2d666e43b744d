"""Micro-benchmark (GPU) of the instance-norm kernels at the bs-8 512^2 step's shapes: time per call
and the HBM bytes each call must move (achieved GB/s against the ~6.3 TB/s a stream reaches).
  python scripts/bench_in.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch  # noqa: E402

from floodgan import _lib as L, ops  # noqa: E402
from floodgan.plans import Buf  # noqa: E402
from bench_conv import time_it  # noqa: E402


def main():
    L.load()
    dev = "cuda"
    for name, (N, H, C, fold, gadd) in {"resblock 256 @128 (fold 1, residual grad)": (8, 128, 256, 1, True),
                                        "conv2 out 128 @256 (fold 0)": (8, 256, 128, 0, False),
                                        "deconv2 out 64 @512 (fold 0)": (8, 512, 64, 0, False)}.items():
        src = Buf.empty(N, H, H, C, 0, dev)
        src.t.uniform_(-1, 1)
        dst = Buf.empty(N, H, H, C, 1, dev)
        mean, rstd = ops.in_stats(src)
        g = Buf.empty(N, H + 2 * fold, H + 2 * fold, C, 0, dev)
        g.t.uniform_(-1, 1)
        ga = Buf.empty(N, H, H, C, 0, dev) if gadd else None
        if ga is not None:
            ga.t.uniform_(-1, 1)
        gd = Buf.empty(N, H, H, C, 1, dev)
        plane = N * H * H * C * 4
        t_stats = time_it(lambda: ops.in_stats(src))
        t_apply = time_it(lambda: ops.in_apply(src, mean, rstd, 1, None, dst, 1))
        t_bwd = time_it(lambda: ops.in_bwd(g, fold, ga, src, mean, rstd, 1, gd, None))
        nb_bwd = plane * (2 + 2 + (2 if gadd else 0) + 1)     # stats: src, g (+gadd); apply: src, g (+gadd), dst
        lib = L.load()
        lib.fg_set_in_rows(0)
        t_apply0 = time_it(lambda: ops.in_apply(src, mean, rstd, 1, None, dst, 1))
        t_bwd0 = time_it(lambda: ops.in_bwd(g, fold, ga, src, mean, rstd, 1, gd, None))
        lib.fg_set_in_rows(1)
        t_apply_ps = time_it(lambda: ops.in_apply(src, mean, rstd, 1, None, dst, 1, presplit=True))
        t_bwd_ps = time_it(lambda: ops.in_bwd(g, fold, ga, src, mean, rstd, 1, gd, None, presplit=True))
        # what torch's own streaming kernels reach on the same bytes
        a, b = src.t, g.t[:src.t.numel()]
        c = torch.empty_like(a)
        t_copy = time_it(lambda: c.copy_(a))
        t_add = time_it(lambda: torch.add(a, b, out=c))
        for tag, t, nb in (("in_stats", t_stats, plane), ("in_apply", t_apply, 2 * plane),
                           ("in_apply grid-stride", t_apply0, 2 * plane), ("in_apply presplit", t_apply_ps, 2 * plane),
                           ("in_bwd (stats+apply)", t_bwd, nb_bwd), ("in_bwd grid-stride", t_bwd0, nb_bwd),
                           ("in_bwd presplit", t_bwd_ps, nb_bwd),
                           ("torch copy_", t_copy, 2 * plane), ("torch add", t_add, 3 * plane)):
            print(f"{name:44s} {tag:22s} {t * 1e3:8.1f} us  {nb / t / 1e6:7.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
