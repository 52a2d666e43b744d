"""Which f16x3 weight packs a steady-state training step still launches one by one (fg_pack_weight_f16 outside the
post-Adam batched re-pack): wraps ops.pack_weight's library call and prints the call sites of the third step."""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
import torch  # noqa: E402

from floodgan import _lib as L, ops  # noqa: E402
from floodgan.model import Model  # noqa: E402


def main():
    dev = torch.device("cuda")
    m = Model(model="PairedAttention", num_epochs=2, topography="all", device=dev)
    g = torch.Generator().manual_seed(1)
    x = (torch.rand((8, 9, 512, 512), generator=g) * 2 - 1).to(dev)
    y = (torch.rand((8, 3, 512, 512), generator=g) * 2 - 1).to(dev)
    lib = L.load()
    real = lib.fg_pack_weight_f16
    sites = collections.Counter()

    class Wrap:
        def __call__(self, *a):
            st = traceback.extract_stack()[-4:-1]
            sites[" <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in reversed(st))] += 1
            return real(*a)
    for it in range(3):
        if it == 2:
            lib.fg_pack_weight_f16 = Wrap()
        m.step_fn(x, y).cpu()
    lib.fg_pack_weight_f16 = real
    print(sum(sites.values()), "single packs in one step")
    for k, v in sites.most_common():
        print(f"{v:4d}  {k}")


if __name__ == "__main__":
    main()
