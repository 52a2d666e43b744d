"""Where the step's ATen launches come from: one bs-8 512^2 training step under torch.profiler with
Python stacks, every aten op that launched a device kernel listed with its call count and the innermost
floodgan frame that issued it (ATen fills in the latency tail).
  python scripts/fill_sites.py"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from floodgan.model import Model  # noqa: E402


def main():
    dev = torch.device("cuda")
    m = Model(model="PairedAttention", num_epochs=2, topography="all", device=dev)
    g = torch.Generator().manual_seed(1234)
    x = (torch.rand((8, 9, 512, 512), generator=g) * 2 - 1).to(dev)
    y = (torch.rand((8, 3, 512, 512), generator=g) * 2 - 1).to(dev)
    for _ in range(2):
        m.step_fn(x, y).cpu()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        m.step_fn(x, y).cpu()
        torch.cuda.synchronize()
    sites = collections.Counter()
    for ev in prof.events():
        if not ev.name.startswith("aten::") or ev.device_type != torch.autograd.DeviceType.CPU:
            continue
        frames = [f for f in (ev.stack or []) if "floodgan" in f or "bench" in f]
        sites[(ev.name, bool(ev.kernels), frames[0] if frames else "?")] += 1
    print("count  op  launched-a-kernel  innermost floodgan frame")
    for (name, k, frame), c in sites.most_common(80):
        print(f"{c:5d}  {name:28s} {'K' if k else '-'} {frame}")


if __name__ == "__main__":
    main()
