"""Diagnostic (GPU): per-layer forward intermediates and per-parameter gradients of the HIP
generator/discriminator executors vs an fp64 CPU recomputation.  Prints a table."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from floodgan import executor as X  # noqa: E402
from oracle import paired_attention as O  # noqa: E402


def nrel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def nchw(B, c=None):
    c = c or B.c
    return B.interior()[..., :c].permute(0, 3, 1, 2).cpu()


def main(R=64, N=2):
    torch.manual_seed(11)
    x = torch.rand(N, 9, R, R) * 2 - 1
    Gp, Dp = O.init_params()
    P = {k: v.cuda() for k, v in Gp.items()}
    Pd = {k: v.double().requires_grad_(True) for k, v in Gp.items()}
    out, mask, S = X.gen_forward(P, x.cuda(), save=True)
    # fp64 recomputation of the intermediates
    xd = x.double()
    IN = lambda t: F.instance_norm(t, eps=1e-5)  # noqa: E731
    c1 = F.conv2d(F.pad(xd, (3,) * 4, mode="reflect"), Pd["conv1.weight"], Pd["conv1.bias"])
    print("c1", nrel(nchw(S["c1"]), c1))
    a1 = F.relu(IN(c1))
    print("a1", nrel(nchw(S["a1"]), a1))
    c2 = F.conv2d(a1, Pd["conv2.weight"], Pd["conv2.bias"], stride=2, padding=1)
    print("c2", nrel(nchw(S["c2"]), c2))
    a2 = F.relu(IN(c2))
    c3 = F.conv2d(a2, Pd["conv3.weight"], Pd["conv3.bias"], stride=2, padding=1)
    print("c3", nrel(nchw(S["c3"]), c3))
    h = F.relu(IN(c3))
    for i in range(9):
        b = S["blocks"][i]
        print(f"block{i} in", nrel(nchw(b["h"]), h))
        h = O.resnet_block(Pd, i, h)
    print("h9", nrel(nchw(S["h"]), h))
    ref_out, ref_mask = O.generator_forward(Pd, xd)
    print("out", nrel(out, ref_out), "mask", nrel(mask, ref_mask))
    g = torch.randn_like(ref_out)
    ref_out.backward(g)
    grads = X.gen_backward(P, S, g.float().cuda())
    torch.cuda.synchronize()
    skip, _ = O.cancelled_biases()
    rows = sorted(((nrel(grads[k], Pd[k].grad), k) for k in Gp if k not in skip), reverse=True)
    for e, k in rows[:12]:
        print(f"grad {k:40s} {e:.3e}")
    print("best", rows[-3:])

    # discriminator, batch 2N
    Dq = {k: v.cuda() for k, v in Dp.items()}
    Ddd = {k: v.double().requires_grad_(True) for k, v in Dp.items()}
    y = torch.rand(2 * N, 3, R, R) * 2 - 1
    xx = torch.cat((x, x), 0)
    buf = X.disc_pack([(xx.cuda(), y.cuda())], 12)
    pred, DS = X.disc_forward(Dq, buf, save=True)
    ref = O.discriminator_forward(Ddd, torch.cat((xx, y), 1).double())
    print("D pred", nrel(pred, ref))
    gp = torch.randn_like(ref)
    ref.backward(gp)
    dg = X.disc_backward(Dq, DS, gp.float().cuda(), param_grads=True)
    torch.cuda.synchronize()
    for k in Dp:
        print(f"Dgrad {k:20s} {nrel(dg[k], Ddd[k].grad):.3e}")


if __name__ == "__main__":
    for R in (32, 64):
        print("==== R", R)
        main(R)
