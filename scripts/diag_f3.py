"""Timing diagnosis of the pipelined forward kernel (needs a library built with -DFG_F3_DIAG, see
scripts/gpu_diag.sh; the outputs of modes 1/2 are garbage): per geometry, the time of the full
kernel (mode 0), of its compute alone (mode 1: no data movement after the first stages) and of
its data movement alone (mode 2: DMA + barriers, no MFMA work); 4/5 without the A split, 9/13 as 1/5
without the per-stage barrier; 32 with every A piece read from a fixed L2-resident window.
  python scripts/diag_f3.py [modes, default 0,1,2,4,5]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

from floodgan import _lib as L, ops  # noqa: E402
from bench_conv import make, time_it  # noqa: E402


TAGS = {0: "full", 1: "compute only", 2: "data movement only", 4: "no A split", 5: "compute only, no A split",
        9: "compute only, no barrier", 13: "compute, no split, no barrier", 32: "A from a fixed L2 window"}
MODES = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 1, 2, 4, 5]


def main():
    L.load()
    L.set_conv_math("f16x3")
    cases = {"resblock 3x3 256->256 @128": (8, 128, 256, 256, 3, 1, 1),
             "conv2 3x3s2 64->128 @512": (8, 512, 64, 128, 3, 2, 1),
             "D model.8 4x4 256->512 @64 (2N)": (16, 64, 256, 512, 4, 1, 1),
             "3x3 128->64 @256 (N=64 class)": (8, 256, 128, 64, 3, 1, 1)}
    for name, c in cases.items():
        mk, flops, keep = make(*c)
        prob = mk(True)
        res = {}
        for _ in range(3):
            for mode in MODES:
                os.environ["FG_F3_DIAG"] = str(mode)
                res.setdefault(mode, []).append(time_it(lambda: ops.conv([prob])))
        os.environ["FG_F3_DIAG"] = "0"
        for mode, tag in TAGS.items():
            if mode not in MODES:
                continue
            ms = min(res[mode])
            print(f"{name:36s} {tag:20s} {ms:8.3f} ms {flops / ms / 1e9:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
