"""Diagnostic (GPU): ReLU-mask agreement between the HIP forward and an fp64 forward."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "flood-prediction-gan_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from floodgan import executor as X  # noqa: E402
from oracle import paired_attention as O  # noqa: E402


def xhat(B, mean, rstd):
    t = B.interior().permute(0, 3, 1, 2).cpu().double()
    n, c = t.shape[:2]
    return (t - mean.view(n, c, 1, 1).cpu().double()) * rstd.view(n, c, 1, 1).cpu().double()


def ref_xhat(t):
    return F.instance_norm(t, eps=1e-5)


for R in (32, 64):
    torch.manual_seed(11)
    x = torch.rand(2, 9, R, R) * 2 - 1
    Gp, _ = O.init_params()
    P = {k: v.cuda() for k, v in Gp.items()}
    out, mask, S = X.gen_forward(P, x.cuda(), save=True)
    for dt in (torch.float64, torch.float32):
        Pd = {k: v.to(dt) for k, v in Gp.items()}
        layers = []
        c = F.conv2d(F.pad(x.to(dt), (3,) * 4, mode="reflect"), Pd["conv1.weight"], Pd["conv1.bias"])
        layers.append(("c1", c, S["c1"], S["m1"], S["r1"])); h = F.relu(ref_xhat(c))
        c = F.conv2d(h, Pd["conv2.weight"], Pd["conv2.bias"], stride=2, padding=1)
        layers.append(("c2", c, S["c2"], S["m2"], S["r2"])); h = F.relu(ref_xhat(c))
        c = F.conv2d(h, Pd["conv3.weight"], Pd["conv3.bias"], stride=2, padding=1)
        layers.append(("c3", c, S["c3"], S["m3"], S["r3"])); h = F.relu(ref_xhat(c))
        for i in range(9):
            b = S["blocks"][i]
            pre = f"resnet_blocks.{i}."
            c = F.conv2d(F.pad(h, (1,) * 4, mode="reflect"), Pd[pre + "conv1.weight"], Pd[pre + "conv1.bias"])
            layers.append((f"b{i}", c, b["cb1"], b["mb1"], b["rb1"]))
            h = O.resnet_block(Pd, i, h)
        for tag in ("content", "attention"):
            hd = S["heads"][tag]
            d1 = F.conv_transpose2d(h, Pd[f"deconv1_{tag}.weight"], Pd[f"deconv1_{tag}.bias"], stride=2, padding=1,
                                    output_padding=1)
            layers.append((f"{tag}_d1", d1, hd["d1"], hd["md1"], hd["rd1"]))
            a1 = F.relu(ref_xhat(d1))
            d2 = F.conv_transpose2d(a1, Pd[f"deconv2_{tag}.weight"], Pd[f"deconv2_{tag}.bias"], stride=2, padding=1,
                                    output_padding=1)
            layers.append((f"{tag}_d2", d2, hd["d2"], hd["md2"], hd["rd2"]))
        tot = 0
        rep = []
        for name, cref, cb, m, r in layers:
            xr = ref_xhat(cref.double())
            xo = xhat(cb, m, r)
            flips = int(((xr > 0) != (xo > 0)).sum())
            tot += flips
            if flips:
                rep.append((name, flips, float(xr[(xr > 0) != (xo > 0)].abs().max())))
        print(R, "HIP vs", str(dt), "relu-mask flips", tot, rep)
    # CPU fp32 vs fp64 flips
    fl = 0
    for dt in (torch.float32,):
        pass
