"""Where the narrow-N pipelined launches spend their time (needs the -DFG_F3_DIAG library, scripts/gpu_diag.sh
build): the deconv2 4-phase ConvTranspose2d 128->64 (bs 8, 256^2 -> 512^2, with the statistics epilogue, as the
step runs it), the deconv1 phases 256->128 (128^2 -> 256^2) and a 3x3 128->64 @256, in the diag modes
0 full, 1 compute only, 2 data movement only, 16 no epilogue, 17 compute only + no epilogue, 18 DMA only + no
epilogue (timing only: the outputs of modes != 0 are garbage).
  FLOODGAN_LIB=<diag lib> python scripts/diag_f3_narrow.py [modes]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch  # noqa: E402

from floodgan import _lib as L, ops, plans as PL  # noqa: E402
from floodgan.plans import Buf  # noqa: E402
from bench_conv import make, time_it  # noqa: E402

MODES = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 4, 1, 2, 16, 17, 18]
TAGS = {0: "full", 4: "no A split", 1: "compute only", 2: "data movement only", 16: "no epilogue", 17: "compute only, no epi",
        18: "DMA only, no epi"}


def convT_case(N, H, cin, cout):
    X = Buf.empty(N, H, H, cin, 1, "cuda")
    X.t.uniform_(-1, 1)
    w = torch.randn(cin, cout, 3, 3, device="cuda") * 0.02
    Y = Buf.empty(N, 2 * H, 2 * H, cout, 0, "cuda")
    maps = PL.phase_maps(w.shape, 3, 1, X.c)
    wps = [ops.pack_weight(w, m) for m, _, _ in maps]
    probs = PL.phase_problems(X, w.shape, 3, 1, Y, wps, maps, bias=torch.zeros(cout, device="cuda"))
    flops = 2.0 * N * (2 * H) ** 2 * cout * cin * 9 / 4
    return (lambda: ops.conv(probs, in_stats=True)), flops, (X, w, Y)


def main():
    L.load()
    L.set_conv_math("f16x3")
    cases = {"deconv2 convT 128->64 256->512 (stats)": convT_case(8, 256, 128, 64),
             "deconv1 convT 256->128 128->256 (stats)": convT_case(8, 128, 256, 128)}
    mk, flops, keep = make(8, 256, 128, 64, 3, 1, 1)
    prob = mk(True)
    cases["3x3 128->64 @256"] = ((lambda: ops.conv([prob])), flops, keep)
    for name, (fn, flops, keep) in cases.items():
        res = {}
        for _ in range(3):
            for mode in MODES:
                os.environ["FG_F3_DIAG"] = str(mode)
                res.setdefault(mode, []).append(time_it(fn))
        os.environ["FG_F3_DIAG"] = "0"
        for mode in MODES:
            ms = min(res[mode])
            print(f"{name:42s} {TAGS.get(mode, mode)!s:24s} {ms:8.3f} ms {flops / ms / 1e9:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
