"""Diagnostic (GPU): step through the generator backward and compare every intermediate
gradient with an fp64 autograd recomputation (retain_grad on the matching tensors)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from floodgan import executor as X, ops, plans as PL  # noqa: E402
from floodgan._lib import FG_ACT_RELU  # noqa: E402
from floodgan.plans import Buf  # noqa: E402
from oracle import paired_attention as O  # noqa: E402


def nrel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def nchw(B, c=None):
    c = c or B.c
    return B.interior()[..., :c].permute(0, 3, 1, 2).cpu()


def main(R, N=2):
    torch.manual_seed(11)
    x = torch.rand(N, 9, R, R) * 2 - 1
    Gp, _ = O.init_params()
    P = {k: v.cuda() for k, v in Gp.items()}
    Pd = {k: v.double() for k, v in Gp.items()}
    out, mask, S = X.gen_forward(P, x.cuda(), save=True)
    IN = lambda t: F.instance_norm(t, eps=1e-5)  # noqa: E731
    # fp64 forward of the content head from the (fp64-recomputed) trunk
    xd = x.double()
    h = F.relu(IN(F.conv2d(F.pad(xd, (3,) * 4, mode="reflect"), Pd["conv1.weight"], Pd["conv1.bias"])))
    h = F.relu(IN(F.conv2d(h, Pd["conv2.weight"], Pd["conv2.bias"], stride=2, padding=1)))
    h = F.relu(IN(F.conv2d(h, Pd["conv3.weight"], Pd["conv3.bias"], stride=2, padding=1)))
    for i in range(9):
        h = O.resnet_block(Pd, i, h)
    h = h.detach().requires_grad_(True)
    d1 = F.conv_transpose2d(h, Pd["deconv1_content.weight"], Pd["deconv1_content.bias"], stride=2, padding=1,
                            output_padding=1)
    d1.retain_grad()
    a1 = F.relu(IN(d1))
    a1.retain_grad()
    d2 = F.conv_transpose2d(a1, Pd["deconv2_content.weight"], Pd["deconv2_content.bias"], stride=2, padding=1,
                            output_padding=1)
    d2.retain_grad()
    a2 = F.relu(IN(d2))
    a2p = F.pad(a2, (3,) * 4, mode="reflect")
    a2p.retain_grad()
    cl = F.conv2d(a2p, Pd["deconv3_content.weight"], Pd["deconv3_content.bias"])
    cl.retain_grad()
    gcl_ref = torch.randn_like(cl)
    cl.backward(gcl_ref)
    # GPU: start the content-head backward from the same gcl
    gcl = Buf.empty(N, R, R, 32, 6, "cuda")
    t = torch.zeros(N, R + 12, R + 12, 32)
    t[:, 6:-6, 6:-6, :27] = gcl_ref.float().permute(0, 2, 3, 1)
    gcl.t.copy_(t.reshape(-1).cuda())
    hc = S["heads"]["content"]
    g_ad2c = Buf.empty(N, R + 6, R + 6, 64, 0, "cuda")
    X._dgrad_s1(P, "deconv3_content", gcl, 6, 7, g_ad2c)
    torch.cuda.synchronize()
    print(R, "g_a2p", nrel(g_ad2c.interior().permute(0, 3, 1, 2).cpu(), a2p.grad))
    g_d2 = Buf.empty(N, R, R, 64, 1, "cuda")
    ops.in_bwd(g_ad2c, 3, None, hc["d2"], hc["md2"], hc["rd2"], FG_ACT_RELU, g_d2, None)
    torch.cuda.synchronize()
    print(R, "g_d2", nrel(nchw(g_d2), d2.grad))
    # compare saved forward tensors too
    print(R, "saved d2", nrel(nchw(hc["d2"]), d2), "saved ad2", nrel(nchw(hc["ad2"]), a2))
    w = P["deconv2_content.weight"]
    g_ad1 = Buf.empty(N, R // 2, R // 2, 128, 0, "cuda")
    m = PL.wmap_convT_dgrad(w.shape, 64)
    ops.conv([PL.conv_problem(g_d2, 1, 3, 2, ops.pack_weight(w, m), m, g_ad1)])
    torch.cuda.synchronize()
    print(R, "g_a1", nrel(nchw(g_ad1), a1.grad))


if __name__ == "__main__":
    for R in (32, 64):
        main(R)
