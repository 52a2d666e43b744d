"""bench.py's multi-rank path end to end on the one-GPU test box.

`bench.py --gpus 2 --dist-backend gloo` starts two ranks itself (the launcher the driver's N-GPU runs use when
WORLD_SIZE is unset), both on the box's one GPU: process group, parameter broadcast, the bucketed all-reduces
during the backward, the barrier + max-over-ranks timing and rank 0's single JSON line with the whole-job rate.
The same code runs one rank per GPU over RCCL on a multi-GPU node (the RCCL collectives themselves:
tests/test_gpu_rccl.py; the two-rank arithmetic: tests/test_gpu_dp.py)."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("launcher", ["bench", "torchrun"])
def test_bench_two_ranks_one_line(launcher):
    """launcher "bench": bench.py starts its ranks itself; "torchrun": the driver's N-GPU command line
    (torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1)"""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    args = ["--gpus", "2", "--dist-backend", "gloo", "--res", "128", "--batch", "2", "--steps", "3", "--warmup", "1",
            "--no-cpu-baseline", "--no-fp32-math"]
    pre = ([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
            "127.0.0.1", "--master-port", str(29500 + os.getpid() % 1000)] if launcher == "torchrun" else [sys.executable])
    r = subprocess.run(pre + [os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True, text=True,
                       timeout=600)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, f"rc {r.returncode}:\n{r.stdout[-2000:]}\n{r.stderr[-4000:]}"
    assert len(lines) == 1, r.stdout[-2000:]          # rank 0 only
    rec = json.loads(lines[0])
    print({k: rec[k] for k in ("value", "ms_per_step", "n_gpus", "config")})
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 4 and rec["config"]["parallelism"] == "dp2"
    assert rec["value"] > 0 and abs(rec["value"] - 4 * 1e3 / rec["ms_per_step"]) < 1e-2 * rec["value"]
    assert rec["roofline"]["launches"] == 3 * 18 and rec["roofline"]["avg_launch_ms"] > 0
    assert all(v == v for v in rec["losses_last_step"])       # finite, not NaN
