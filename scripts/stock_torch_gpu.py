"""Out-of-the-box GPU reference point: the reference algorithm (the CPU
oracle's functional restatement, oracle/paired_attention.py) run on stock PyTorch-ROCm
(MIOpen convolutions, ATen elementwise/norm/Adam) on one MI355X, bs 8, 512x512.  Test/
measurement infrastructure only -- not the product path.
  python scripts/stock_torch_gpu.py [--batch 8] [--res 512] [--steps 5] [--warmup 2]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from oracle import paired_attention as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda")
    G, D = O.init_params(47, 9)
    st = O.PairedStepOracle(G={k: v.to(dev) for k, v in G.items()}, D={k: v.to(dev) for k, v in D.items()})
    g = torch.Generator().manual_seed(1234)
    x = (torch.rand((a.batch, 9, a.res, a.res), generator=g) * 2 - 1).to(dev)
    y = (torch.rand((a.batch, 3, a.res, a.res), generator=g) * 2 - 1).to(dev)
    for _ in range(a.warmup):
        st.step(x, y)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        losses = st.step(x, y)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"what": "stock PyTorch-ROCm (MIOpen) run of the reference algorithm",
                      "img_per_s": round(a.batch * a.steps / dt, 3), "ms_per_step": round(1e3 * dt / a.steps, 2),
                      "batch": a.batch, "res": a.res, "steps": a.steps, "torch": torch.__version__,
                      "losses_last_step": [round(v, 5) for v in losses]}), flush=True)


if __name__ == "__main__":
    main()
