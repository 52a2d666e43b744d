"""Diagnostic (GPU): instance-norm backward precision on real generator activations."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from floodgan import executor as X, ops  # noqa: E402
from floodgan.plans import Buf  # noqa: E402
from oracle import paired_attention as O  # noqa: E402


def nrel(a, b):
    a = a.detach().double().cpu(); b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


for R in (32, 64):
    torch.manual_seed(11)
    x = torch.rand(2, 9, R, R) * 2 - 1
    Gp, _ = O.init_params()
    P = {k: v.cuda() for k, v in Gp.items()}
    out, mask, S = X.gen_forward(P, x.cuda(), save=True)
    hc = S["heads"]["content"]
    d2 = hc["d2"].interior().permute(0, 3, 1, 2).cpu()          # fp32 values as stored
    mean = d2.double().mean((2, 3)); std = d2.double().std((2, 3), unbiased=False)
    print(R, "mean/std max", float((mean.abs() / std).max()), "median", float((mean.abs() / std).median()))
    gm = hc["md2"].view(2, 64).cpu().double(); gr = hc["rd2"].view(2, 64).cpu().double()
    print(R, "mean err", float(((gm - mean) / std).abs().max()), "rstd rel err", float((gr * torch.sqrt(std**2 + 1e-5) - 1).abs().max()))
    g = torch.randn(2, 64, R, R, dtype=torch.float64)
    c64 = d2.double().requires_grad_(True)
    (ref,) = torch.autograd.grad(F.relu(F.instance_norm(c64, eps=1e-5)), c64, g)
    c32 = d2.clone().requires_grad_(True)
    (ref32,) = torch.autograd.grad(F.relu(F.instance_norm(c32, eps=1e-5)), c32, g.float())
    gb = Buf.empty(2, R, R, 64, 0, "cuda"); gb.t.copy_(g.float().permute(0, 2, 3, 1).reshape(-1).cuda())
    dst = Buf.empty(2, R, R, 64, 0, "cuda")
    ops.in_bwd(gb, 0, None, hc["d2"], hc["md2"], hc["rd2"], 1, dst, None)
    torch.cuda.synchronize()
    ours = dst.interior().permute(0, 3, 1, 2).cpu()
    print(R, "in_bwd ours vs fp64", nrel(ours, ref), " cpu fp32 vs fp64", nrel(ref32, ref))
    xh64 = (d2.double() - mean[..., None, None]) / torch.sqrt(std[..., None, None] ** 2 + 1e-5)
    xh32 = (d2 - hc["md2"].view(2, 64, 1, 1).cpu()) * hc["rd2"].view(2, 64, 1, 1).cpu()
    print(R, "mask flips", int(((xh64 > 0) != (xh32 > 0)).sum()), "of", xh64.numel(), "xhat err", nrel(xh32, xh64))
    err = (ours.double() - ref).abs()
    idx = torch.nonzero(err > 1e3 * float(err.median()))
    print(R, "n big-err elems", idx.shape[0], idx[:10].tolist())
