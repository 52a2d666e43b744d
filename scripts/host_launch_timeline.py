"""Host-side timeline of one paired step: when (after the step's call) the host issues each C-ABI entry point.

The GPU idles at the start of every step until the host has issued the first kernels (the previous step ended
with the losses' copy to the host).  This prints the host time of the first launches of a step and the total
host time per step, with the GPU otherwise idle (synchronised before the step) and busy (steady state).
  python scripts/host_launch_timeline.py [first_n]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
import torch  # noqa: E402

from floodgan import _lib as L  # noqa: E402
from floodgan.model import Model  # noqa: E402


class _Proxy:
    def __init__(self, lib, log):
        self._lib, self._log = lib, log

    def __getattr__(self, name):
        fn = getattr(self._lib, name)
        if not name.startswith("fg_") or name in ("fg_last_error", "fg_last_launch", "fg_get_conv_math"):
            return fn
        log = self._log

        def call(*a):
            log.append((time.perf_counter(), name))
            return fn(*a)
        return call


def main():
    first = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    dev = torch.device("cuda")
    m = Model(model="PairedAttention", num_epochs=2, topography="all", device=dev)
    g = torch.Generator().manual_seed(1234)
    x = (torch.rand((8, 9, 512, 512), generator=g) * 2 - 1).to(dev)
    y = (torch.rand((8, 3, 512, 512), generator=g) * 2 - 1).to(dev)
    for _ in range(2):
        m.step_fn(x, y).cpu()
    lib = L.load()
    log = []
    L._lib = _Proxy(lib, log)
    try:
        for rep in range(3):
            torch.cuda.synchronize()
            log.clear()
            t0 = time.perf_counter()
            out = m.step_fn(x, y)
            t1 = time.perf_counter()
            out.cpu()
            t2 = time.perf_counter()
            print(f"step {rep}: host issue {1e3 * (t1 - t0):.2f} ms, until losses {1e3 * (t2 - t0):.2f} ms, "
                  f"{len(log)} C-ABI calls")
            print("   " + "  ".join(f"{1e6 * (t - t0):.0f}us:{n[3:]}" for t, n in log[:first]))
    finally:
        L._lib = lib


if __name__ == "__main__":
    main()
