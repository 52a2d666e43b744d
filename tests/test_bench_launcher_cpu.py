"""bench.py's own N-rank launcher: `python bench.py --gpus N` with WORLD_SIZE unset
starts N rank processes with torch.distributed.run's environment, relays rank 0's stdout, and fails
when any rank fails; a WORLD_SIZE that disagrees with --gpus is refused.  CPU only: the children here
are a stand-in script, not the GPU step."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

CHILD = r"""
import json, os, sys
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
        "FLOODGAN_DIST_BACKEND", "HSA_ENABLE_IPC_MODE_LEGACY")
print(json.dumps({"argv": sys.argv[1:], **{k: os.environ.get(k) for k in keys}}), flush=True)
if os.environ["RANK"] == os.environ.get("FAIL_RANK"):
    sys.exit(3)
if os.environ.get("FAIL_RANK") is not None:
    import time; time.sleep(60)          # a healthy rank blocked in a collective
"""


def test_rank_envs_match_torchrun():
    envs = bench.rank_envs(4, 29511, base={"PATH": "/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, backend="gloo")
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    for e in envs:
        assert e["WORLD_SIZE"] == "4" and e["LOCAL_WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29511"
        assert e["FLOODGAN_DIST_BACKEND"] == "gloo" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
        assert e["PATH"] == "/bin"
    assert "HSA_ENABLE_IPC_MODE_LEGACY" in bench.rank_envs(1, 1, base={})[0]


def test_launch_ranks_relays_rank0(tmp_path, capfd):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    os.environ.pop("FAIL_RANK", None)
    rc = bench.launch_ranks(3, ["--gpus", "3", "--steps", "2"], backend="gloo", script=str(script), timeout=120)
    assert rc == 0
    out, err = capfd.readouterr()
    lines = [json.loads(x) for x in out.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and lines[0]["RANK"] == "0"                 # only rank 0 on stdout
    assert lines[0]["argv"] == ["--gpus", "3", "--steps", "2"] and lines[0]["WORLD_SIZE"] == "3"
    others = sorted(json.loads(x)["RANK"] for x in err.splitlines() if x.startswith("{"))
    assert others == ["1", "2"]


def test_launch_ranks_fails_and_stops_the_rest(tmp_path):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    os.environ["FAIL_RANK"] = "1"
    try:
        rc = bench.launch_ranks(2, [], script=str(script), timeout=120)
    finally:
        os.environ.pop("FAIL_RANK")
    assert rc == 3


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "refusing" in r.stderr
