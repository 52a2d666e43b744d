"""Tile-config sweep of the pipelined f16x3 kernel on the step's N=64 convolutions at bs 8, 512^2 (the
conv_fwd_f3_kernel<128,64> class: the content head's input gradient, the deconv2 phases, conv2's input
gradient).  fg_set_f3_tile forces each config (0..9) in turn; -2 = the register-staged x6 kernel.
  python scripts/diag_n64.py"""
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


def buf(n, h, c, pad):
    b = Buf.empty(n, h, h, c, pad, "cuda")
    b.t.uniform_(-1, 1)
    return b


def main():
    L.load()
    L.set_conv_math("f16x3")
    lib = L.load()
    N = 8
    cases = {}
    # content-head input gradient: 7x7 over the 32-channel (27 valid) gradient, border 6 -> 518^2 x 64
    w = torch.randn(27, 64, 7, 7, device="cuda") * 0.02
    gcl = buf(N, 512, 32, 6)
    Y = Buf.empty(N, 518, 518, 64, 0, "cuda")
    m = PL.wmap_conv_dgrad_s1(w.shape, 32)
    wp = ops.pack_weight(w, m)
    cases["content dgrad 7x7 32->64 @518"] = ([PL.conv_problem(gcl, 6, 7, 1, wp, m, Y)],
                                               2.0 * N * 518 * 518 * 64 * 27 * 49, (w, gcl, Y, wp))
    # deconv2 forward: ConvTranspose2d(128, 64, 3, 2, 1, output_padding=1), 256^2 -> 512^2
    w2 = torch.randn(128, 64, 3, 3, device="cuda") * 0.02
    ad1 = buf(N, 256, 128, 1)
    Y2 = Buf.empty(N, 512, 512, 64, 0, "cuda")
    maps = PL.phase_maps(w2.shape, 3, 1, 128)
    wps = [ops.pack_weight(w2, mm) for mm, _, _ in maps]
    cases["deconv2 convT 128->64 @512 (4 phases)"] = (PL.phase_problems(ad1, w2.shape, 3, 1, Y2, wps, maps),
                                                      2.0 * N * 512 * 512 * 64 * 128 * 9 / 4, (w2, ad1, Y2, wps))
    # conv2 input gradient: Conv2d(64, 128, 3, 2, 1) -> dgrad phases from the 128-ch 256^2 gradient
    w3 = torch.randn(128, 64, 3, 3, device="cuda") * 0.02
    gc2 = buf(N, 256, 128, 1)
    Y3 = Buf.empty(N, 512, 512, 64, 0, "cuda")
    maps3 = PL.phase_maps(w3.shape, 3, 1, 128)
    wps3 = [ops.pack_weight(w3, mm) for mm, _, _ in maps3]
    cases["conv2 dgrad 128->64 @512 (4 phases)"] = (PL.phase_problems(gc2, w3.shape, 3, 1, Y3, wps3, maps3),
                                                    2.0 * N * 512 * 512 * 64 * 128 * 9 / 4, (w3, gc2, Y3, wps3))
    # N=128 class: conv2 forward (3x3 s2 64->128, 512^2 -> 256^2), deconv1 forward (convT 256->128 phases)
    w4 = torch.randn(128, 64, 3, 3, device="cuda") * 0.02
    a1 = buf(N, 512, 64, 1)
    Y4 = Buf.empty(N, 256, 256, 128, 0, "cuda")
    m4 = PL.wmap_conv_fwd(w4.shape, 64)
    wp4 = ops.pack_weight(w4, m4)
    n128 = {"conv2 fwd 3x3s2 64->128 @256": ([PL.conv_problem(a1, 1, 3, 2, wp4, m4, Y4)],
                                             2.0 * N * 256 * 256 * 128 * 64 * 9, (w4, a1, Y4, wp4))}
    w5 = torch.randn(256, 128, 3, 3, device="cuda") * 0.02
    h = buf(N, 128, 256, 1)
    Y5 = Buf.empty(N, 256, 256, 128, 0, "cuda")
    maps5 = PL.phase_maps(w5.shape, 3, 1, 256)
    wps5 = [ops.pack_weight(w5, mm) for mm, _, _ in maps5]
    n128["deconv1 convT 256->128 @256 (4 phases)"] = (PL.phase_problems(h, w5.shape, 3, 1, Y5, wps5, maps5),
                                                      2.0 * N * 256 * 256 * 128 * 256 * 9 / 4, (w5, h, Y5, wps5))
    for name, (probs, flops, keep) in n128.items():
        for cfg in (-1, 6, 1, 3, 0, 2, 5, 4):
            lib.fg_set_f3_tile(cfg)
            ms = min(time_it(lambda: ops.conv(probs)) for _ in range(3))
            print(f"{name:40s} cfg {cfg:3d} {ms:8.3f} ms {flops / ms / 1e9:7.1f} TFLOP/s", flush=True)
    for name, (probs, flops, keep) in cases.items():
        for cfg in (-1, 9, 7, 8, 6, 3, -2):
            lib.fg_set_f3_tile(cfg)
            try:
                ms = min(time_it(lambda: ops.conv(probs)) for _ in range(3))
                print(f"{name:40s} cfg {cfg:3d} {ms:8.3f} ms {flops / ms / 1e9:7.1f} TFLOP/s", flush=True)
            except RuntimeError as e:
                print(f"{name:40s} cfg {cfg:3d} failed: {e}", flush=True)
    lib.fg_set_f3_tile(-1)


if __name__ == "__main__":
    main()
