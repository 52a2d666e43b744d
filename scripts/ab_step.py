"""A/B of engine switches on the full bs-8 512^2 training step, interleaved in ONE process (device
clocks and boxes differ by several percent, so separate bench runs cannot resolve small gains).
  python scripts/ab_step.py f3_persistent [rounds] [steps] [values, default 0,1]
Switches: timer (values 0 = no KernelTimer, 1/2/3 = bench's KernelTimer with marker events of system / device / no
release, 4 = events on the dispatch packet),
f3_persistent, f3_sched, f3_order, f3_fill, f3_interleave, wgrad_f3, use_win, in_rows, presplit, ps_wide (values 4,5), ps_tall, ps_resid, stem_fwd, d0_dgrad, fused_head, n1_rows (values: rows per block)."""
import contextlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
import torch  # noqa: E402

from floodgan import _lib as L, ops  # noqa: E402
from floodgan.model import Model  # noqa: E402


def switch(name, on):
    lib = L.load()
    if name == "f3_persistent":
        lib.fg_set_f3_persistent(int(on))
    elif name == "f3_sched":
        lib.fg_set_f3_sched(int(on))
    elif name == "f3_order":
        lib.fg_set_f3_order(int(on))
    elif name == "wgrad_f3":
        L.set_wgrad_f3(on)
    elif name == "f3_fill":
        lib.fg_set_f3_fill(int(on))
    elif name == "presplit":
        ops.PRESPLIT = bool(on)
    elif name == "ps_resid":
        ops.PRESPLIT_RESID = bool(on)
    elif name == "ps_wide":
        lib.fg_set_f3_ps_wide(int(on))
    elif name == "ps_tall":
        lib.fg_set_f3_ps_tall(int(on))
    elif name == "in_rows":
        lib.fg_set_in_rows(int(on))
    elif name == "f3_interleave":
        lib.fg_set_f3_interleave(int(on))
    elif name == "use_win":
        ops.USE_WIN = bool(on)
    elif name == "stem_fwd":
        os.environ["FLOODGAN_STEM_FWD"] = str(int(on))
    elif name == "d0_dgrad":
        from floodgan import executor
        executor.D0_DGRAD = bool(on)
    elif name == "fused_head":
        from floodgan import executor
        executor.FUSED_HEAD = bool(on)
    elif name == "timer":
        pass                                      # applied around the timed loop (main)
    elif name == "n1_rows":
        ops.N1_ROWS = int(on)
    else:
        raise SystemExit(f"unknown switch {name}")


def main():
    name = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    vals = [int(v) for v in sys.argv[4].split(",")] if len(sys.argv) > 4 else [0, 1]
    dev = torch.device("cuda")
    m = Model(model="PairedAttention", num_epochs=2, topography="all", device=dev)
    g = torch.Generator().manual_seed(1234)
    x = (torch.rand((8, 9, 512, 512), generator=g) * 2 - 1).to(dev)
    y = (torch.rand((8, 3, 512, 512), generator=g) * 2 - 1).to(dev)
    for on in vals:
        switch(name, on)
        m.step_fn(x, y).cpu()
    res = {v: [] for v in vals}
    kinds = {v: {} for v in vals}
    tags = ["resblock_conv_fwd", "resblock_conv_dgrad", "resblock_conv_wgrad"]
    for _ in range(rounds):
        for on in vals:
            switch(name, on)
            timer = (ops.KernelTimer(tags, events=["system", "device", "none", "dispatch"][on - 1])
                     if name == "timer" and on > 0 else
                     ops.KernelTimer(tags + ["resblock_dgrad_strips"]) if name != "timer" else contextlib.nullcontext())
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with timer:
                for _ in range(steps):
                    m.step_fn(x, y).cpu()
            torch.cuda.synchronize()
            res[on].append((time.perf_counter() - t0) / steps * 1e3)
            if name != "timer" or on > 0:
                for t, d in timer.durations_ms().items():
                    kinds[on].setdefault(t, []).extend(d)
    for on in vals:
        v = sorted(res[on])
        k = "  ".join(f"{t.split('_')[-1]} {sum(d) / len(d) * 1e3:.1f} us" for t, d in sorted(kinds[on].items()) if d)
        print(f"{name}={on}: ms/step min {v[0]:.2f} median {v[len(v) // 2]:.2f}  ({8e3 / v[0]:.1f} img/s best)  {k}")


if __name__ == "__main__":
    main()
