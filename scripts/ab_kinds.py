"""Per-kind launch times of the resblock convs (HIP events on the launch stream, bench.py's KernelTimer tags)
under an engine switch, interleaved in ONE process on the bs-8 512^2 step:
  python scripts/ab_kinds.py f3_sched [rounds] [steps] [values, default 0,1]     (switches: scripts/ab_step.py)"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch  # noqa: E402

from ab_step import switch  # noqa: E402
from floodgan import ops  # noqa: E402
from floodgan.model import Model  # noqa: E402

TAGS = ["resblock_conv_fwd", "resblock_conv_dgrad", "resblock_conv_wgrad"]


def main():
    name = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    vals = [int(v) for v in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0, 1]
    dev = torch.device("cuda")
    m = Model(model="PairedAttention", num_epochs=2, topography="all", device=dev)
    g = torch.Generator().manual_seed(1234)
    x = (torch.rand((8, 9, 512, 512), generator=g) * 2 - 1).to(dev)
    y = (torch.rand((8, 3, 512, 512), generator=g) * 2 - 1).to(dev)
    for v in vals:
        switch(name, v)
        m.step_fn(x, y).cpu()
    res = {v: {t: [] for t in TAGS + ["step"]} for v in vals}
    for _ in range(rounds):
        for v in vals:
            switch(name, v)
            timer = ops.KernelTimer(TAGS)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with timer:
                for _ in range(steps):
                    m.step_fn(x, y).cpu()
            torch.cuda.synchronize()
            res[v]["step"].append((time.perf_counter() - t0) / steps * 1e3)
            for t, d in timer.durations_ms().items():
                res[v][t] += d
    for v in vals:
        print(f"{name}={v}: " + "  ".join(f"{t.replace('resblock_conv_', '')} {statistics.median(d) * (1 if t == 'step' else 1e3):.1f}"
                                         for t, d in res[v].items()) + "  (step ms, kinds us; medians)", flush=True)


if __name__ == "__main__":
    main()
