"""Diagnostic: HIP smooth-loss gradients vs the fp64 oracle with and without teacher-forced
activation decisions, and forced vs unforced oracle, at several sizes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flood-prediction-gan_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from oracle import paired_attention as O  # noqa: E402
from test_gpu_northstar import _inputs, _model, hip_smooth_grads, oracle_smooth_grads  # noqa: E402

torch.set_num_threads(16)


def nrel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


skip = O.cancelled_biases()[0] | O.cancelled_biases()[1]
for R in [int(r) for r in sys.argv[1:]]:
    x, y = _inputs(1, res=R, seed=99)
    m = _model()
    gG, gD, masks = hip_smooth_grads(m, x.cuda(), y.cuda())
    Gp, Dp = O.init_params()
    dec = O.ActDecisions(masks)
    fG, fD = oracle_smooth_grads(Gp, Dp, x, y, dec)
    uG, uD = oracle_smooth_grads(Gp, Dp, x, y, None)
    hip = {**gG, **{"D." + k: v for k, v in gD.items()}}
    forced = {**fG, **{"D." + k: v for k, v in fD.items()}}
    free = {**uG, **{"D." + k: v for k, v in uD.items()}}

    def worst(a, b):
        return max(((k, nrel(a[k], b[k])) for k in a if k.split("D.")[-1] not in skip), key=lambda t: t[1])
    print(f"R={R}: flips {sum(n for _, _, n, _ in dec.log)} kink {dec.worst():.2e}; hip-vs-forced {worst(hip, forced)}; "
          f"hip-vs-free {worst(hip, free)}; forced-vs-free {worst(forced, free)}", flush=True)
    print("   per-layer flips:", [(n, l, c) for n, l, c, _ in dec.log if c], flush=True)
