"""Measurement probe (not the product path): what capturing the whole paired step in a HIP graph would save.

Captures one PairedStep (bs 8, 512^2) with torch.cuda.graph after eager warm-up, then times K replays against K
eager steps, each followed by the losses' copy to the host as in bench.py.  The replays repeat the captured
launches verbatim -- Adam's step count and every host-side decision frozen at capture -- so their numbers are
timing only, not training.
  python scripts/graph_probe.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
import torch  # noqa: E402

from floodgan.model import Model  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda")
    m = Model(model="PairedAttention", num_epochs=2, topography="all", device=dev)
    g = torch.Generator().manual_seed(1234)
    x = (torch.rand((8, 9, 512, 512), generator=g) * 2 - 1).to(dev)
    y = (torch.rand((8, 3, 512, 512), generator=g) * 2 - 1).to(dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            m.step_fn(x, y).cpu()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()

    def eager(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            m.step_fn(x, y).cpu()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    res = {"eager": [eager(steps) for _ in range(3)], "graph": []}
    # (no eager step after the capture: a pre-capture buffer the captured step frees could be handed to eager
    # work and then written by a replay)
    graph = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(graph, capture_error_mode="relaxed"):
            out = m.step_fn(x, y)
    except Exception as e:                      # noqa: BLE001
        print(f"capture failed: {type(e).__name__}: {e}")
        return 1

    def replay(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            graph.replay()
            out.cpu()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    for _ in range(3):
        res["graph"].append(replay(steps))
    for k, v in res.items():
        v = sorted(v)
        print(f"{k}: ms/step min {v[0]:.3f} median {v[1]:.3f}")
    print("losses after replays (frozen-step timing only):", out.cpu().tolist())
    return 0


if __name__ == "__main__":
    sys.exit(main())
