"""Diagnostic (GPU): D-step gradients of the fused PairedStep vs fp64 on the same fake."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from floodgan.model import Model  # noqa: E402
from oracle import paired_attention as O  # noqa: E402


def nrel(a, b):
    a = a.detach().double().cpu(); b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


for R in (32, 64):
    z = np.load(os.path.join(ROOT, f"tests/golden/paired_step_{R}.npz"))
    g = {k.replace("__", "."): z[k] for k in z.files}
    x = torch.from_numpy(g["x0"]); y = torch.from_numpy(g["y0"])
    m = Model(model="PairedAttention", num_epochs=2)
    D0 = {k: v.detach().clone().cpu() for k, v in m.discriminator.named_parameters()}
    # capture D grads right after the D backward by hooking the D optimizer
    cap = {}
    orig = m.optimizer_discriminator.step

    def hooked(*a, **k):
        for n, p in m.discriminator.named_parameters():
            cap[n] = p.grad.detach().clone().cpu()
        return orig(*a, **k)
    m.optimizer_discriminator.step = hooked
    losses = m.step_fn(x.cuda(), y.cuda()).cpu()
    fake = m.step_fn.last_output.detach().cpu().double()
    D = {k: v.double().requires_grad_(True) for k, v in D0.items()}
    xd, yd = x.double(), y.double()
    pf = O.discriminator_forward(D, torch.cat((xd, fake), 1)); pr = O.discriminator_forward(D, torch.cat((xd, yd), 1))
    ((F.mse_loss(pf, torch.zeros_like(pf)) + F.mse_loss(pr, torch.ones_like(pr))) * 0.5).backward()
    _, sd = O.cancelled_biases()
    for k in D0:
        if k not in sd:
            print(R, "Dstep grad", k, nrel(cap[k], D[k].grad))
    print(R, "losses", losses.tolist(), float(F.mse_loss(pr, torch.ones_like(pr))), float(F.mse_loss(pf, torch.zeros_like(pf))))
