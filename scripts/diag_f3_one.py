"""One diagnostic geometry of the pipelined forward kernel, for counter passes on the -DFG_F3_DIAG
library (scripts/gpu_pmc_step.sh with DIAG=1): the resblock 3x3 256->256 conv at 128^2, bs 8, `reps`
launches in the mode FG_F3_DIAG selects (0 full, 1 compute only, 2 data movement only, 4 no A split,
5 compute only without the split; outputs of modes != 0 are garbage).
  FG_F3_DIAG=5 python scripts/diag_f3_one.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch  # noqa: E402

from floodgan import _lib as L, ops  # noqa: E402
from bench_conv import make  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    L.load()
    L.set_conv_math("f16x3")
    mk, flops, keep = make(8, 128, 256, 256, 3, 1, 1)
    prob = mk(True)
    for _ in range(reps):
        ops.conv([prob])
    torch.cuda.synchronize()
    print("done mode", os.environ.get("FG_F3_DIAG", "0"), reps, flush=True)


if __name__ == "__main__":
    main()
