"""Run-to-run determinism of the fused training step: the same state (parameters + both Adam states) and the same
batch, stepped `reps` times; every G / D gradient and the losses are compared bit for bit with the first repeat.
Every kernel of the step is deterministic by construction (fixed-order reductions), so any difference is a race.
  python scripts/diag_determinism.py [reps] [res] [bs] [switch=value ...]
switches (in-process): head_1x1, use_win, splitpix, presplit, ps_resid, f3_persistent, fused_in_stats;
process-level ones (FLOODGAN_F3_NARROW, FLOODGAN_STEM_FWD) through the environment."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
import torch  # noqa: E402

from floodgan import _lib as L, executor, ops  # noqa: E402
from floodgan.model import Model  # noqa: E402


def apply(sw):
    name, v = sw.split("=")
    v = int(v)
    lib = L.load()
    if name == "head_1x1":
        executor.HEAD_1X1 = bool(v)
    elif name == "use_win":
        ops.USE_WIN = bool(v)
    elif name == "splitpix":
        executor.SPLITPIX = bool(v)
    elif name == "presplit":
        ops.PRESPLIT = bool(v)
    elif name == "ps_resid":
        ops.PRESPLIT_RESID = bool(v)
    elif name == "fused_in_stats":
        ops.FUSED_IN_STATS = bool(v)
    elif name == "f3_persistent":
        lib.fg_set_f3_persistent(v)
    else:
        raise SystemExit(f"unknown switch {name}")


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    res = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    bs = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    for sw in sys.argv[4:]:
        apply(sw)
    dev = torch.device("cuda")
    m = Model(model="PairedAttention", num_epochs=2, topography="all", device=dev)
    g = torch.Generator().manual_seed(77)
    x = (torch.rand((bs, 9, res, res), generator=g) * 2 - 1).to(dev)
    y = (torch.rand((bs, 3, res, res), generator=g) * 2 - 1).to(dev)
    nets = {"G": m.generator, "D": m.discriminator}
    opts = {"G": m.optimizer_generator, "D": m.optimizer_discriminator}
    m.step_fn(x, y).cpu()                       # Adam states exist from here on
    p0 = {n: {k: p.detach().clone() for k, p in net.named_parameters()} for n, net in nets.items()}
    s0 = {n: copy.deepcopy(o.state_dict()) for n, o in opts.items()}
    first, bad = None, 0
    for r in range(reps):
        with torch.no_grad():
            for n, net in nets.items():
                for k, p in net.named_parameters():
                    p.copy_(p0[n][k])
        for n, o in opts.items():
            o.load_state_dict(copy.deepcopy(s0[n]))
        loss = m.step_fn(x, y).cpu()
        cur = {"loss": loss}
        for n, net in nets.items():
            for k, p in net.named_parameters():
                cur[f"{n}.{k}"] = p.grad.detach().clone()
        if first is None:
            first = cur
            continue
        diff = [(k, float((v.double() - first[k].double()).abs().max()),
                 float((v.double() - first[k].double()).norm() / max(float(first[k].double().norm()), 1e-30)))
                for k, v in cur.items() if not torch.equal(v, first[k])]
        if diff:
            bad += 1
            diff.sort(key=lambda t: -t[2])
            print(f"rep {r}: {len(diff)} tensors differ; worst {diff[:4]}", flush=True)
    print(f"switches {sys.argv[4:]} narrow={os.environ.get('FLOODGAN_F3_NARROW', '1')} "
          f"stem_fwd={os.environ.get('FLOODGAN_STEM_FWD', '1')}: {bad} of {reps - 1} repeats differ", flush=True)


if __name__ == "__main__":
    main()
