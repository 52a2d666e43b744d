"""Evaluation inference on the HIP path: the segmentation U-Net vs the
reference's own UNet (golden) and the fp64 oracle, the metric kernels vs the oracle's torchmetrics-1.2.0
restatement (formula parity unpinned: torchmetrics is absent), and calculate_metrics end to end."""
import os

import numpy as np
import pytest
import torch

from oracle import evaluation as OE
from test_gpu_parity import DEV, nrel

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "segmentation_unet_64.npz")


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _unet():
    from floodgan.segmentation import UNet, initialise_weights
    torch.manual_seed(5)
    return UNet().apply(initialise_weights)


def test_unet_vs_reference_golden(report):
    gold = {k.replace("__", "."): v for k, v in np.load(GOLD).items()}
    net = _unet().to(DEV)
    g = torch.Generator().manual_seed(77)
    x1 = torch.rand((2, 3, 64, 64), generator=g)
    with torch.no_grad():
        logits = net(x1.to(DEV))
    ref = torch.from_numpy(gold["logits_64"])
    e = nrel(logits, ref)
    agree = float(((logits.cpu() > 0) == (ref > 0)).double().mean())
    report("segmentation_unet_vs_golden", logits_rel=e, mask_agreement=agree)
    assert e < 1e-4 and agree > 0.999
    # training-mode BatchNorm: the running statistics moved exactly as the reference's first call
    net_c = _unet()
    P = dict(net_c.named_parameters())
    B = {k: v.clone() for k, v in net_c.named_buffers()}
    with torch.no_grad():
        OE.unet_forward(P, B, x1)
    worst = max(nrel(v, B[k]) for k, v in net.named_buffers() if v.is_floating_point())
    assert worst < 1e-5, worst


@pytest.mark.parametrize("n,res", [(1, 256), (3, 192), (2, 512)])
def test_metric_kernels_vs_oracle(n, res, report):
    from floodgan.evaluate import ImageMetrics
    g = torch.Generator().manual_seed(res + n)
    a = torch.rand((n, 3, res, res), generator=g)
    b = (a + 0.15 * torch.randn(a.shape, generator=g)).clamp(0, 1)
    im = ImageMetrics(DEV)
    ad, bd = a.to(DEV), b.to(DEV)
    got = dict(psnr=im.psnr(ad, bd), ssim=im.ssim(ad, bd), ms_ssim=im.ms_ssim(ad, bd))
    ref = dict(psnr=OE.psnr(a, b), ssim=OE.ssim(a, b), ms_ssim=OE.ms_ssim(a, b))
    report("metric_kernels_vs_oracle", n=n, res=res, got=got, ref=ref)
    assert abs(got["psnr"] - ref["psnr"]) < 1e-6 * abs(ref["psnr"])
    assert abs(got["ssim"] - ref["ssim"]) < 2e-6
    assert abs(got["ms_ssim"] - ref["ms_ssim"]) < 2e-6
    assert im.ssim(ad, ad) == pytest.approx(1.0, abs=1e-6)


def test_mask_confusion_vs_oracle():
    from floodgan.evaluate import MaskConfusion
    from floodgan.plans import Buf
    g = torch.Generator().manual_seed(9)
    lp, lt = torch.randn(2, 1, 40, 48, generator=g), torch.randn(2, 1, 40, 48, generator=g)
    bufs = []
    for t in (lp, lt):
        b = Buf.zeros(2, 40, 48, 4, 0, DEV)
        b.interior()[..., 0] = t[:, 0].to(DEV)
        bufs.append(b)
    mc = MaskConfusion(DEV)
    mc.update(*bufs)
    mc.update(*bufs)                                   # accumulates like the reference's torch.cat
    got = mc.compute()
    ref = OE.binary_metrics(torch.cat([OE.flood_mask(lp)] * 2), torch.cat([OE.flood_mask(lt)] * 2))
    assert all(got[k] == pytest.approx(ref[k], abs=1e-12) for k in ref), (got, ref)


def test_calculate_metrics_end_to_end(report):
    """Model.calculate_metrics on a synthetic two-batch loader at 256x256 (PairedAttention, seed-47
    weights) vs the same pipeline with the oracle's metrics and UNet (fp64) on the HIP generator outputs"""
    from floodgan.model import Model
    from floodgan.segmentation import UNet, initialise_weights
    g = torch.Generator().manual_seed(21)
    batches = [(torch.rand((2, 9, 256, 256), generator=g) * 2 - 1, torch.rand((2, 3, 256, 256), generator=g) * 2 - 1,
                ["hurricane-harvey_0", "hurricane-harvey_1"]) for _ in range(2)]
    m = Model(model="PairedAttention", training_model=False, val_loader=batches, device=DEV)
    torch.manual_seed(5)
    seg = UNet().apply(initialise_weights)
    seg_ref = {k: v.detach().double().clone() for k, v in seg.state_dict().items()}
    df = m.calculate_metrics(seg_model=seg.to(DEV))
    got = df.iloc[0].to_dict()
    # oracle pipeline on the same generator outputs
    P = {k: v for k, v in seg_ref.items() if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))}
    B = {k: v for k, v in seg_ref.items() if k.endswith(("running_mean", "running_var", "num_batches_tracked"))}
    per = {"PSNR": [], "SSIM": [], "MS-SSIM": []}
    pm, tm = [], []
    for x, y, _ in batches:
        torch.manual_seed(47)
        with torch.no_grad():
            out = m.generator(x.to(DEV)).cpu().double()
        go, gt = OE.unit_image(out), OE.unit_image(y.double())
        per["PSNR"].append(OE.psnr(go, gt))
        per["SSIM"].append(OE.ssim(go, gt))
        per["MS-SSIM"].append(OE.ms_ssim(go, gt))
        with torch.no_grad():
            pm.append(OE.flood_mask(OE.unet_forward(P, B, go)))
            tm.append(OE.flood_mask(OE.unet_forward(P, B, gt)))
    ref = {k: float(np.mean(v)) for k, v in per.items()}
    ref.update(OE.binary_metrics(torch.cat(pm), torch.cat(tm)))
    report("calculate_metrics_end_to_end", got={k: float(v) for k, v in got.items()}, ref=ref)
    for k in ("PSNR", "SSIM", "MS-SSIM"):
        assert abs(got[k] - ref[k]) < 1e-5 * max(1.0, abs(ref[k])), (k, got[k], ref[k])
    # masks: a logit within rounding of 0 may land on either side -> 1e-3 of the pixels
    for k in ("MSE", "Accuracy", "F1_Flood", "Precision_Flood", "Recall_Flood", "F1_No_Flood", "Precision_No_Flood",
              "Recall_No_Flood"):
        assert abs(got[k] - ref[k]) < 1e-3, (k, got[k], ref[k])
    assert np.isnan(got["LPIPS"]) and got["Inference"] > 0
