"""Diagnostic (GPU): isolate the generator head's backward kernels at a given resolution."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from floodgan import ops, plans as PL  # noqa: E402
from floodgan.plans import Buf  # noqa: E402

DEV = "cuda"


def nrel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def buf_from(x, pad, mode, c_alloc=None):
    n, c, h, w = x.shape
    c_alloc = c_alloc or c
    xp = F.pad(x, (pad,) * 4, mode=mode) if pad else x
    t = torch.zeros(n, h + 2 * pad, w + 2 * pad, c_alloc)
    t[..., :c] = xp.float().permute(0, 2, 3, 1)
    return Buf(t.reshape(-1).to(DEV), n, h, w, c_alloc, pad)


def nchw(B, c=None):
    c = c or B.c
    return B.interior()[..., :c].permute(0, 3, 1, 2).cpu()


def run(H, N=2):
    torch.manual_seed(0)
    # (a) 7x7 dgrad 27(->32 alloc) -> 64, full correlation
    w = torch.randn(27, 64, 7, 7, dtype=torch.float64) * 0.02
    gy = torch.randn(N, 27, H, H, dtype=torch.float64)
    xp = torch.zeros(N, 64, H + 6, H + 6, dtype=torch.float64, requires_grad=True)
    (ref,) = torch.autograd.grad(F.conv2d(xp, w), xp, gy)
    G = buf_from(gy, 6, "constant", 32)
    out = Buf.empty(N, H + 6, H + 6, 64, 0, DEV)
    wd = w.float().to(DEV)
    m = PL.wmap_conv_dgrad_s1(wd.shape, 32)
    ops.conv([PL.conv_problem(G, 6, 7, 1, ops.pack_weight(wd, m), m, out)])
    torch.cuda.synchronize()
    print(H, "dgrad7x7", nrel(nchw(out), ref))
    # (b) IN+relu backward with fold 3 from that padded gradient
    c = torch.randn(N, 64, H, H, dtype=torch.float64, requires_grad=True)
    y = F.pad(F.relu(F.instance_norm(c, eps=1e-5)), (3,) * 4, mode="reflect")
    g = torch.randn_like(y)
    (gc,) = torch.autograd.grad(y, c, g)
    cb = buf_from(c.detach(), 0, "constant")
    mean, rstd = ops.in_stats(cb)
    gs = buf_from(g, 0, "constant")
    gs = Buf(gs.t, N, H + 6, H + 6, 64, 0)
    dst = Buf.empty(N, H, H, 64, 1, DEV)
    ops.in_bwd(gs, 3, None, cb, mean, rstd, 1, dst, None)
    torch.cuda.synchronize()
    print(H, "in_bwd fold3", nrel(nchw(dst), gc))
    dst2 = Buf.empty(N, H, H, 64, 0, DEV)
    ops.fold_add(gs, 3, None, dst2)
    x0 = torch.zeros(N, 64, H, H, dtype=torch.float64, requires_grad=True)
    (gf,) = torch.autograd.grad(F.pad(x0, (3,) * 4, mode="reflect"), x0, g)
    torch.cuda.synchronize()
    print(H, "fold_add 3", nrel(nchw(dst2), gf))
    # (c) no fold, same IN
    g2 = torch.randn(N, 64, H, H, dtype=torch.float64)
    (gc2,) = torch.autograd.grad(F.relu(F.instance_norm(c, eps=1e-5)), c, g2)
    dst3 = Buf.empty(N, H, H, 64, 1, DEV)
    ops.in_bwd(buf_from(g2, 0, "constant"), 0, None, cb, mean, rstd, 1, dst3, None)
    torch.cuda.synchronize()
    print(H, "in_bwd plain", nrel(nchw(dst3), gc2))
    # (d) convT dgrad (stride-2 conv over gy) 128<-64 and wgrad convT
    wt = torch.randn(128, 64, 3, 3, dtype=torch.float64) * 0.05
    xin = torch.randn(N, 128, H // 2, H // 2, dtype=torch.float64, requires_grad=True)
    wq = wt.clone().requires_grad_(True)
    yt = F.conv_transpose2d(xin, wq, stride=2, padding=1, output_padding=1)
    gyt = torch.randn_like(yt)
    gx_ref, gw_ref = torch.autograd.grad(yt, (xin, wq), gyt)
    GY = buf_from(gyt, 1, "constant")
    wtd = wt.float().to(DEV)
    gx = Buf.empty(N, H // 2, H // 2, 128, 0, DEV)
    m2 = PL.wmap_convT_dgrad(wtd.shape, 64)
    ops.conv([PL.conv_problem(GY, 1, 3, 2, ops.pack_weight(wtd, m2), m2, gx)])
    dw = torch.empty_like(wtd)
    XB = buf_from(xin.detach(), 1, "constant")
    ops.wgrad(PL.wgrad_convT(XB, GY, 3, 1, 128), PL.wmap_wgrad(wtd.shape, True, 64, 3), dw)
    torch.cuda.synchronize()
    print(H, "convT dgrad", nrel(nchw(gx), gx_ref), "convT wgrad", nrel(dw, gw_ref))


if __name__ == "__main__":
    for H in (32, 64, 128):
        run(H)
