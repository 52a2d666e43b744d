"""Diagnostic: the smooth-loss G/D gradients through the drop-in modules (autograd) vs through the
executor-level helper of tests/test_gpu_northstar.py, both on the HIP path, at several sizes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flood-prediction-gan_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from test_gpu_northstar import _inputs, _model, hip_smooth_grads  # noqa: E402


def nrel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


for R in [int(r) for r in sys.argv[1:]] or [64, 256, 512]:
    x, y = _inputs(1, res=R, seed=99)
    m = _model()
    xd, yd = x.cuda(), y.cuda()
    fake = m.generator(xd)
    pred = m.discriminator(torch.cat((xd, fake), 1))
    (F.mse_loss(pred, torch.ones_like(pred)) + 100 * F.mse_loss(fake, yd)).backward()
    gm = {k: p.grad.clone() for k, p in m.generator.named_parameters()}
    dm = {k: p.grad.clone() for k, p in m.discriminator.named_parameters()}
    gG, gD, _ = hip_smooth_grads(m, xd, yd)
    eg = max(((k, nrel(gG[k], gm[k])) for k in gG), key=lambda t: t[1])
    ed = max(((k, nrel(gD[k], dm[k])) for k in gD), key=lambda t: t[1])
    # twice through the executor: determinism
    gG2, gD2, _ = hip_smooth_grads(m, xd, yd)
    e2 = max(((k, nrel(gG2[k], gG[k])) for k in gG), key=lambda t: t[1])
    print(f"R={R}: executor vs module G {eg} D {ed}; executor run-to-run {e2}", flush=True)
