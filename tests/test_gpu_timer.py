"""bench.py's live per-kernel timing (ops.KernelTimer): events on the timed kernel's own dispatch packet.

The roofline figure of the bench line divides the resblock conv's FLOPs by its average launch time measured with
HIP events inside the timed steps.  Marker events around the launch (torch.cuda.Event) put a packet with a
system-scope release -- an L2 writeback and invalidate -- into the stream at every timed launch, which the timed
step then carries (~6 us per event, profiles/round6/r6k_*).  The default mode attaches the events to the conv's own
dispatch (fg_timing_arm -> hipExtLaunchKernel).  These tests pin that the tagged calls are the ones that consume the
arm (one timed launch per tagged call, positive durations), that a tagged call launching no timed kernel fails
loudly instead of timing nothing, and that bench.py reports the launches it timed."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))

TAGS = ["resblock_conv_fwd", "resblock_conv_dgrad", "resblock_conv_wgrad"]


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.mark.parametrize("events", ["dispatch", "none", "system"])
def test_kernel_timer_counts_and_durations(events):
    _need_gpu()
    from floodgan import ops
    from floodgan.model import Model
    dev = torch.device("cuda")
    m = Model(model="PairedAttention", num_epochs=2, topography="all", device=dev)
    g = torch.Generator().manual_seed(5)
    x = (torch.rand((2, 9, 128, 128), generator=g) * 2 - 1).to(dev)
    y = (torch.rand((2, 3, 128, 128), generator=g) * 2 - 1).to(dev)
    m.step_fn(x, y).cpu()
    timer = ops.KernelTimer(TAGS, events=events)
    with timer:
        for _ in range(2):
            m.step_fn(x, y).cpu()
    d = timer.durations_ms()
    print(events, {t: (len(v), sum(v) / max(len(v), 1)) for t, v in d.items()})
    # 9 resblocks x 2 convs per step: the forward launches once per conv; the backward once per conv for the
    # input gradient's interior and once for the weight gradient (the G step; the D step does not reach G)
    for t in TAGS:
        assert len(d[t]) == 2 * 18, (t, len(d[t]))
        assert all(0.0 < v < 100.0 for v in d[t]), (t, d[t][:4])
    assert timer.durations_ms() == {t: [] for t in TAGS}   # events released


def test_dispatch_arm_not_consumed_raises():
    _need_gpu()
    from floodgan import _lib as L, ops
    t = torch.randn(4096, device="cuda")
    out = torch.zeros(64, device="cuda")
    with ops.KernelTimer(["absmax"]):
        with pytest.raises(RuntimeError, match="launched no timed kernel"):
            ops._timed("absmax", lambda: L.check(L.load().fg_absmax(L.ptr(t), t.numel(), L.ptr(out),
                                                                      L.stream_handle()), "absmax"))
    assert L.load().fg_timing_disarm() == 0      # the failed call left no arm behind
    torch.cuda.synchronize()


def test_bench_reports_dispatch_timed_launches():
    _need_gpu()
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--res", "128", "--batch", "2", "--steps",
                        "2", "--warmup", "1", "--no-cpu-baseline", "--no-fp32-math"], env=env, capture_output=True,
                       text=True, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, f"no JSON line (rc {r.returncode}):\n{r.stdout[-2000:]}\n{r.stderr[-4000:]}"
    rec = json.loads(lines[-1])
    rl = rec["roofline"]
    print(rl)
    assert r.returncode == 0
    assert rl["launches"] == 2 * 18 and rl["avg_launch_ms"] > 0
    assert "dispatch packet" in rl["timing"]
