"""CPU ORACLE for the evaluation path -- TEST INFRASTRUCTURE ONLY (only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import it).

  unet_forward    models/model_architectures.py:508-587 (UNet(3, 1, bilinear=False)), BatchNorm in training
                  mode as the reference evaluates it (models/model.py:380-400 never calls .eval());
                  pinned by tests/golden/segmentation_unet_64.npz (make_golden_segmentation.py runs the
                  reference's own UNet class)
  psnr / ssim / ms_ssim / binary metrics
                  torchmetrics 1.2.0 (requirements.txt:7) as models/model.py:367-378 configures it:
                  PeakSignalNoiseRatio(data_range=(0, 1)), StructuralSimilarityIndexMeasure(data_range=(0, 1)),
                  MultiScaleStructuralSimilarityIndexMeasure(data_range=(0, 1)), MeanSquaredError, Binary*.
                  torchmetrics is not installed in this image: these restate its published algorithm
                  (gaussian 11x11 sigma 1.5 window over reflect-padded inputs, cropped back; five MS-SSIM
                  scales with betas (0.0448, 0.2856, 0.3001, 0.2363, 0.1333), normalize="relu") -- PARITY
                  UNPINNED for the metric formulas.
"""
import torch
import torch.nn.functional as F

ENC = [64, 128, 256, 512, 1024]
BETAS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)


def _dc(P, B, prefix, x, training=True):
    for i, j in ((0, 1), (3, 4)):
        x = F.conv2d(x, P[f"{prefix}.double_conv.{i}.weight"], None, padding=1)
        n = f"{prefix}.double_conv.{j}"
        x = F.relu(F.batch_norm(x, B[n + ".running_mean"], B[n + ".running_var"], P[n + ".weight"], P[n + ".bias"],
                                training=training, momentum=0.1, eps=1e-5))
    return x


def unet_forward(P, B, x, training=True):
    """logits [N, 1, H, W] of the reference UNet (forward :527-538; Up :573-580 incl. its size padding)"""
    xs = [_dc(P, B, "inc", x, training)]
    for k in range(1, 5):
        xs.append(_dc(P, B, f"down{k}.maxpool_conv.1", F.max_pool2d(xs[-1], 2), training))
    h = xs[4]
    for k in range(1, 5):
        skip = xs[4 - k]
        u = F.conv_transpose2d(h, P[f"up{k}.up.weight"], P[f"up{k}.up.bias"], stride=2)
        dy, dx = skip.shape[2] - u.shape[2], skip.shape[3] - u.shape[3]
        u = F.pad(u, [dx // 2, dx - dx // 2, dy // 2, dy - dy // 2])
        h = _dc(P, B, f"up{k}.conv", torch.cat([skip, u], 1), training)
    return F.conv2d(h, P["outc.conv.weight"], P["outc.conv.bias"])


def unit_image(x):
    """models/model.py:397-398"""
    return torch.clamp((x + 1) * 0.5, min=0, max=1)


def flood_mask(logits):
    """models/model.py:399-400"""
    return (torch.sigmoid(logits) > 0.5).float()


def psnr(a, b, data_range=1.0):
    a, b = a.clamp(0, 1).double(), b.clamp(0, 1).double()
    mse = ((a - b) ** 2).sum() / a.numel()
    return float(10 * torch.log10(data_range ** 2 / mse))


def _gaussian(size=11, sigma=1.5, dtype=torch.float64):
    d = torch.arange((1 - size) / 2, (1 + size) / 2, 1, dtype=dtype)
    g = torch.exp(-torch.pow(d / sigma, 2) / 2)
    return (g / g.sum()).unsqueeze(0)


def _ssim_and_cs(a, b, data_range=1.0, k1=0.01, k2=0.03):
    """per-image (ssim, cs) of torchmetrics 1.2.0 _ssim_update"""
    a, b = a.clamp(0, 1).double(), b.clamp(0, 1).double()
    C = a.shape[1]
    c1, c2 = (k1 * data_range) ** 2, (k2 * data_range) ** 2
    g = _gaussian()
    kernel = torch.matmul(g.t(), g).expand(C, 1, 11, 11)
    pad = 5
    a, b = F.pad(a, (pad,) * 4, mode="reflect"), F.pad(b, (pad,) * 4, mode="reflect")
    outs = F.conv2d(torch.cat((a, b, a * a, b * b, a * b)), kernel, groups=C)
    mu_a, mu_b, e_aa, e_bb, e_ab = outs.split(a.shape[0])
    mu_a2, mu_b2, mu_ab = mu_a ** 2, mu_b ** 2, mu_a * mu_b
    upper = 2 * (e_ab - mu_ab) + c2
    lower = (e_aa - mu_a2) + (e_bb - mu_b2) + c2
    ssim_map = ((2 * mu_ab + c1) * upper) / ((mu_a2 + mu_b2 + c1) * lower)
    cs_map = upper / lower
    crop = (Ellipsis, slice(pad, -pad), slice(pad, -pad))
    n = ssim_map.shape[0]
    return ssim_map[crop].reshape(n, -1).mean(-1), cs_map[crop].reshape(n, -1).mean(-1)


def ssim(a, b):
    return float(_ssim_and_cs(a, b)[0].mean())


def ms_ssim(a, b):
    cs_list = []
    for _ in range(len(BETAS)):
        sim, cs = _ssim_and_cs(a, b)
        cs_list.append(torch.relu(cs))
        a, b = F.avg_pool2d(a, 2), F.avg_pool2d(b, 2)
    cs_list[-1] = torch.relu(sim)
    stack = torch.stack(cs_list)
    betas = torch.tensor(BETAS, dtype=torch.float64).view(-1, 1)
    return float(torch.prod(stack ** betas, 0).mean())


def binary_metrics(pred, true):
    """MeanSquaredError / Binary{Accuracy, F1Score, Precision, Recall} of flat 0/1 masks, and of their
    inversions (models/model.py:412-418)"""
    pred, true = pred.flatten().double(), true.flatten().double()

    def div(a, b):
        return float(a / b) if b else 0.0

    def stats(p, t):
        tp = float(((p == 1) & (t == 1)).sum())
        fp = float(((p == 1) & (t == 0)).sum())
        fn = float(((p == 0) & (t == 1)).sum())
        return tp, fp, fn

    out = {"MSE": float(((pred - true) ** 2).mean()), "Accuracy": float((pred == true).double().mean())}
    for tag, p, t in (("Flood", pred, true), ("No_Flood", 1 - pred, 1 - true)):
        tp, fp, fn = stats(p, t)
        out[f"F1_{tag}"] = div(2 * tp, 2 * tp + fp + fn)
        out[f"Precision_{tag}"] = div(tp, tp + fp)
        out[f"Recall_{tag}"] = div(tp, tp + fn)
    return out
