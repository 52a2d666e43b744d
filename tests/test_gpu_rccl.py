"""The RCCL path executed on the one-GPU test box.

`bench.py --rccl-world1` initialises a ONE-rank ProcessGroupNCCL ("nccl" = RCCL on ROCm) and forces the
paired step's bucketed asynchronous SUM all-reduces through it (floodgan.parallel.set_force_collectives):
D's buckets before Adam(D) and G's overlapping the generator backward, exactly as a multi-rank run issues
them (/root/reference models/model.py:632-633, :645-646 are the exchange points).  At world 1 a SUM
all-reduce is the identity, so the step must be bit-identical to the same step without collectives: this
pins that ProcessGroupNCCL's stream, the bucket hand-offs from the backward's current stream and the waits
before Adam neither race nor corrupt the gradients.  The multi-rank arithmetic (1/world pre-scaling, the
all-reduced gradient = the whole-batch gradient) is pinned by tests/test_gpu_dp.py and the gloo tests."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_world1_bucketed_allreduce_bit_identical():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--rccl-world1", "--res", "64", "--batch",
                        "2", "--steps", "3", "--warmup", "1"], env=env, capture_output=True, text=True, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, f"no JSON line (rc {r.returncode}):\n{r.stdout[-2000:]}\n{r.stderr[-4000:]}"
    rec = json.loads(lines[-1])
    print(rec)
    assert rec["backend"] == "nccl" and rec["world_size"] == 1
    # every bucket of both networks went through ProcessGroupNCCL on every step (warm-up included)
    assert rec["buckets_per_step"] >= 10 and rec["collectives_per_step"] == rec["buckets_per_step"]
    assert rec["bytes_per_step"] == 4 * (11841765 + 2773953)
    assert rec["losses_bit_identical"] and rec["params_bit_identical"]
    assert r.returncode == 0
