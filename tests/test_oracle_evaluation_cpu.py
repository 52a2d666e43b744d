"""The evaluation oracle (oracle/evaluation.py) and the segmentation drop-in modules on the CPU: the
reference UNet's golden (tests/golden/make_golden_segmentation.py), and the metric restatements'
known-answer properties (torchmetrics is absent: formula parity unpinned)."""
import os

import numpy as np
import pytest
import torch

from oracle import evaluation as OE

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "segmentation_unet_64.npz")


@pytest.fixture(scope="module")
def gold():
    z = np.load(GOLD)
    return {k.replace("__", "."): z[k] for k in z.files}


def _ours():
    from floodgan.segmentation import UNet, initialise_weights
    torch.manual_seed(5)
    return UNet().apply(initialise_weights)


def test_unet_modules_match_reference_init(gold):
    net = _ours()
    keys = [k[len("init/"):] for k in gold if k.startswith("init/")]
    assert list(net.state_dict()) == keys
    for name, t in net.state_dict().items():
        ref = gold["init/" + name]
        t = t.double().flatten()
        n8 = min(8, t.numel())
        assert np.array_equal(t[:n8].numpy(), ref[2:2 + n8]), name
        assert abs(t.sum().item() - ref[0]) <= 1e-9 * max(1.0, abs(ref[1])), name


def test_oracle_unet_matches_reference_golden(gold):
    net = _ours()
    P = dict(net.named_parameters())
    B = {k: v.clone() for k, v in net.named_buffers()}
    g = torch.Generator().manual_seed(77)
    x1 = torch.rand((2, 3, 64, 64), generator=g)
    x2 = torch.rand((1, 3, 48, 48), generator=g)
    with torch.no_grad():
        l1 = OE.unet_forward(P, B, x1)
        l2 = OE.unet_forward(P, B, x2)
    for out, ref in ((l1, gold["logits_64"]), (l2, gold["logits_48"])):
        assert np.linalg.norm(out.numpy() - ref) / np.linalg.norm(ref) < 1e-5
    for k, v in B.items():
        if not v.is_floating_point():
            continue
        ref = gold["after/" + k]
        assert abs(v.double().sum().item() - ref[0]) <= 1e-4 * max(1.0, abs(ref[1])), k


def test_metric_restatements_known_answers():
    g = torch.Generator().manual_seed(3)
    a = torch.rand((2, 3, 192, 192), generator=g, dtype=torch.float64)
    assert OE.ssim(a, a) == pytest.approx(1.0, abs=1e-12)
    assert OE.ms_ssim(a, a) == pytest.approx(1.0, abs=1e-12)
    b = (a + 0.1).clamp(0, 1)
    mse = float(((a - b) ** 2).mean())
    assert OE.psnr(a, b) == pytest.approx(10 * np.log10(1 / mse), rel=1e-12)
    # SSIM on a constant shift: luminance term only changes; structure intact -> close to but below 1
    s = OE.ssim(a, b)
    assert 0.5 < s < 1.0
    # windows: the cropped map covers exactly the windows inside the image
    s1, cs1 = OE._ssim_and_cs(a[:, :, :64, :64], b[:, :, :64, :64])
    assert s1.shape == (2,) and cs1.shape == (2,)


def test_binary_metrics_restatement():
    p = torch.tensor([1, 1, 0, 0, 1, 0, 1, 0], dtype=torch.float32)
    t = torch.tensor([1, 0, 0, 1, 1, 0, 0, 0], dtype=torch.float32)
    m = OE.binary_metrics(p, t)
    tp, fp, fn, tn = 2, 2, 1, 3
    assert m["MSE"] == pytest.approx((fp + fn) / 8)
    assert m["Accuracy"] == pytest.approx((tp + tn) / 8)
    assert m["Precision_Flood"] == pytest.approx(tp / (tp + fp))
    assert m["Recall_Flood"] == pytest.approx(tp / (tp + fn))
    assert m["F1_Flood"] == pytest.approx(2 * tp / (2 * tp + fp + fn))
    assert m["Precision_No_Flood"] == pytest.approx(tn / (tn + fn))
    assert m["Recall_No_Flood"] == pytest.approx(tn / (tn + fp))
    # zero division -> 0 (torchmetrics' _safe_divide)
    z = OE.binary_metrics(torch.zeros(4), torch.zeros(4))
    assert z["Precision_Flood"] == 0.0 and z["F1_Flood"] == 0.0 and z["Accuracy"] == 1.0


def test_evaluate_host_helpers():
    """the device path's host arithmetic: the gaussian window and the confusion-count metrics"""
    from floodgan.evaluate import MaskConfusion, extract_input_topography, gaussian11
    g = gaussian11()
    assert g.dtype == torch.float32 and abs(float(g.sum()) - 1) < 1e-6 and g.argmax() == 5
    assert torch.allclose(g.double(), OE._gaussian().flatten(), atol=1e-7)
    mc = MaskConfusion(device="cpu")
    mc.counts = torch.tensor([2, 2, 3, 1])            # tp, fp, tn, fn of test_binary_metrics_restatement
    p = torch.tensor([1, 1, 0, 0, 1, 0, 1, 0], dtype=torch.float32)
    t = torch.tensor([1, 0, 0, 1, 1, 0, 0, 0], dtype=torch.float32)
    ref = OE.binary_metrics(p, t)
    got = mc.compute()
    assert all(got[k] == pytest.approx(ref[k]) for k in ref)
    x = torch.arange(9.0).view(1, 9, 1, 1)
    assert extract_input_topography(x, "flow").flatten().tolist() == [0, 1, 2, 4]
    assert extract_input_topography(x, None).flatten().tolist() == [0, 1, 2]
    assert extract_input_topography(x[:, :4], "dem").shape[1] == 4
    with pytest.raises(ValueError):
        extract_input_topography(x[:, :5], "map")
