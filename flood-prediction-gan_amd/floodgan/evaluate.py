"""Evaluation inference: the reference's Model.calculate_metrics
(models/model.py:363-422) and ModelsGroup.compare_metrics (models/group.py:114-221) on the device.

Per batch of the loader: the generator's forward (torch.manual_seed(47) first, as the reference), the
[0, 1] images clamp((x + 1) * 0.5, 0, 1) of output and target, PSNR / SSIM / MS-SSIM of the pair
(torchmetrics 1.2.0 semantics, requirements.txt:7: data_range=(0, 1), per call = per batch, then
averaged over batches), and the segmentation U-Net's flood masks of both images accumulated into
confusion counts; at the end MSE / accuracy / F1 / precision / recall of the flood and no-flood masks
over every pixel seen (the reference concatenates the flattened masks, which is the same counts).

LPIPS (torchmetrics' LearnedPerceptualImagePatchSimilarity) needs pretrained VGG/AlexNet weights that
no offline image can supply: it is reported as NaN.  torchmetrics itself is not installed here, so the
metric formulas follow its published 1.2.0 algorithm and their parity is unpinned (the oracle restates
the same algorithm: oracle/evaluation.py)."""
import math
import time

import numpy as np
import torch

from . import _lib as L
from . import ops
from .segmentation import SegmentationModel, unit_image

MS_SSIM_BETAS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)
K1, K2 = 0.01, 0.03
DATA_RANGE = 1.0
METRIC_NAMES = ["PSNR", "SSIM", "MS-SSIM", "LPIPS", "MSE", "Accuracy", "F1_Flood", "Precision_Flood", "Recall_Flood",
                "F1_No_Flood", "Precision_No_Flood", "Recall_No_Flood"]


def gaussian11(sigma=1.5, size=11):
    """torchmetrics _gaussian in float32: exp(-(d / sigma)^2 / 2) over d = -5..5, normalised"""
    d = torch.arange((1 - size) / 2, (1 + size) / 2, 1, dtype=torch.float32)
    g = torch.exp(-torch.pow(d / sigma, 2) / 2)
    return g / g.sum()


class ImageMetrics:
    """Device PSNR / SSIM / MS-SSIM of [N, C, H, W] images already in [0, 1] (contiguous NCHW)."""

    def __init__(self, device="cuda"):
        self.device = torch.device(device)
        self.g = gaussian11().to(self.device)
        self.betas = torch.tensor(MS_SSIM_BETAS, dtype=torch.float64, device=self.device)
        self.c1, self.c2 = (K1 * DATA_RANGE) ** 2, (K2 * DATA_RANGE) ** 2

    def psnr(self, a, b):
        """10 log10(range^2 / mean squared error over the whole batch) -- one torchmetrics update+compute"""
        out = torch.empty(1, dtype=torch.float64, device=self.device)
        work = torch.empty(int(L.load().fg_sq_err_workspace_doubles()), dtype=torch.float64, device=self.device)
        L.check(L.load().fg_sq_err_sum(L.ptr(a), L.ptr(b), a.numel(), L.ptr(out), L.ptr(work), L.stream_handle()),
                "sq_err_sum")
        mse = float(out) / a.numel()
        return 10.0 * math.log10(DATA_RANGE ** 2 / mse) if mse > 0 else float("inf")

    def _ssim_cs(self, a, b, want_cs=False):
        N, C, H, W = a.shape
        lib = L.load()
        ssim = torch.empty(N, dtype=torch.float64, device=self.device)
        cs = torch.empty(N, dtype=torch.float64, device=self.device) if want_cs else None
        work = torch.empty(int(lib.fg_ssim_workspace_doubles(N, C, H, W)), dtype=torch.float64, device=self.device)
        L.check(lib.fg_ssim(L.ptr(a), L.ptr(b), N, C, H, W, L.ptr(self.g), ops.C.c_float(self.c1),
                            ops.C.c_float(self.c2), L.ptr(ssim), L.ptr(cs), L.ptr(work), L.stream_handle()), "ssim")
        return ssim, cs

    def ssim(self, a, b):
        """mean over the batch of the per-image SSIM"""
        return float(self._ssim_cs(a, b)[0].mean())

    def ms_ssim(self, a, b):
        """torchmetrics MultiScaleStructuralSimilarityIndexMeasure (normalize="relu"): five scales, the
        contrast sensitivity of the first four and the SSIM of the last, F.avg_pool2d(2) in between"""
        N, C, H, W = a.shape
        S = len(MS_SSIM_BETAS)
        if H < 2 ** S or W < 2 ** S or H // (S - 1) ** 2 <= 10:
            raise ValueError(f"MS-SSIM needs images larger than {(S - 1) ** 2 * 10}px (got {H}x{W})")
        cs_all = torch.empty(S - 1, N, dtype=torch.float64, device=self.device)
        lib = L.load()
        for s in range(S):
            ssim, cs = self._ssim_cs(a, b, want_cs=True)
            if s < S - 1:
                cs_all[s] = cs
                h2, w2 = a.shape[2] // 2, a.shape[3] // 2
                pa = torch.empty(N, C, h2, w2, dtype=torch.float32, device=self.device)
                pb = torch.empty_like(pa)
                for src, dst in ((a, pa), (b, pb)):
                    L.check(lib.fg_avg_pool2(L.ptr(src), N * C, src.shape[2], src.shape[3], L.ptr(dst),
                                             L.stream_handle()), "avg_pool2")
                a, b = pa, pb
        out = torch.empty(N, dtype=torch.float64, device=self.device)
        L.check(lib.fg_msssim_combine(N, S, L.ptr(cs_all), L.ptr(ssim), L.ptr(self.betas), L.ptr(out),
                                      L.stream_handle()), "msssim_combine")
        return float(out.mean())


class MaskConfusion:
    """tp / fp / tn / fn of the flood masks over every pixel seen, and the torchmetrics binary metrics
    (zero_division -> 0) of the flood and the inverted no-flood masks"""

    def __init__(self, device="cuda"):
        self.counts = torch.zeros(4, dtype=torch.int64, device=device)

    def update(self, pred_logits, true_logits):
        L.check(L.load().fg_mask_confusion(ops.view(pred_logits), ops.view(true_logits), L.ptr(self.counts),
                                           L.stream_handle()), "mask_confusion")

    def compute(self):
        tp, fp, tn, fn = (int(v) for v in self.counts.cpu())
        n = tp + fp + tn + fn

        def div(a, b):
            return a / b if b else 0.0

        out = {"MSE": div(fp + fn, n), "Accuracy": div(tp + tn, n),
               "F1_Flood": div(2 * tp, 2 * tp + fp + fn), "Precision_Flood": div(tp, tp + fp),
               "Recall_Flood": div(tp, tp + fn)}
        # the no-flood masks are 1 - mask: tp <-> tn, fp <-> fn
        out.update({"F1_No_Flood": div(2 * tn, 2 * tn + fn + fp), "Precision_No_Flood": div(tn, tn + fn),
                    "Recall_No_Flood": div(tn, tn + fp)})
        return out


def extract_input_topography(x, topography):
    """models/utils.py:69-79 on a 9-channel input; inputs the loader already narrowed pass through"""
    from .data import TOPOGRAPHY_SOURCE_CHANNELS
    key = None if topography in (None, "none") else topography
    chans = TOPOGRAPHY_SOURCE_CHANNELS[key]
    if x.shape[1] == len(chans):
        return x
    if x.shape[1] != 9:
        raise ValueError(f"input with {x.shape[1]} channels for topography {topography!r}")
    return x[:, chans]


def score_batch(generator, input_stack, ground_truth, seg, im, confs, sync=True):
    """One batch of models/model.py:388-410 (the segmentation U-Net sees the output, then the target, as
    there): returns (PSNR, SSIM, MS-SSIM, inference seconds); the masks go into every MaskConfusion of
    confs."""
    start = time.time()
    torch.manual_seed(47)
    with torch.no_grad():
        out = generator(input_stack)
    if sync:
        torch.cuda.synchronize()
    t = time.time() - start
    gt, gt_buf = unit_image(ground_truth, buf=True)
    go, go_buf = unit_image(out, buf=True)
    pred_logits = seg.logits_from_buf(go_buf)
    true_logits = seg.logits_from_buf(gt_buf)
    for conf in confs:
        conf.update(pred_logits, true_logits)
    return im.psnr(go, gt), im.ssim(go, gt), im.ms_ssim(go, gt), t


def calculate_metrics(generator, loader, seg_model, topography="all", device="cuda"):
    """The device counterpart of Model.calculate_metrics: {metric: value} averaged as the reference
    does (image metrics over batches, mask metrics over all pixels)."""
    im, conf = ImageMetrics(device), MaskConfusion(device)
    per = {k: [] for k in ("PSNR", "SSIM", "MS-SSIM", "Inference")}
    for input_stack, ground_truth, _ in loader:
        x = extract_input_topography(input_stack, topography).to(device)
        y = ground_truth.to(device)
        p, s, m, t = score_batch(generator, x, y, seg_model, im, [conf])
        for k, v in zip(("PSNR", "SSIM", "MS-SSIM", "Inference"), (p, s, m, t)):
            per[k].append(v)
    res = {k: float(np.mean(v)) for k, v in per.items() if k != "Inference"}
    res["LPIPS"] = float("nan")
    res.update(conf.compute())
    res["Inference"] = float(np.mean(per["Inference"]))
    return {k: res[k] for k in METRIC_NAMES + ["Inference"]}


def compare_metrics(generators, loader, seg_model, compare="model", device="cuda"):
    """ModelsGroup.compare_metrics (models/group.py:114-221): {generator name: {metric: value}} plus the
    per-disaster metrics {generator name: {disaster: {metric: value}}} -- the mask metrics over that
    disaster's pixels and the batch means of PSNR / SSIM / MS-SSIM (LPIPS NaN) over its batches, as the
    reference's grouped table (group.py:211-221).  compare="topography": the
    generators are keyed by topography ("All", "DEM", "Flow accumulation", "Distance to rivers", "Map",
    "None") and see the matching channels of one 9-channel input (models/group.py:83-94)."""
    topo_keys = {"All": "all", "DEM": "dem", "Flow accumulation": "flow", "Distance to rivers": "river", "Map": "map",
                 "None": None}
    im = ImageMetrics(device)
    conf = {g: MaskConfusion(device) for g in generators}
    grouped = {}
    per = {g: {k: [] for k in ("PSNR", "SSIM", "MS-SSIM", "Inference")} for g in generators}
    disasters = []
    for input_stack, ground_truth, names in loader:
        x = input_stack.to(device)
        y = ground_truth.to(device)
        disaster = names[0].split("_")[0]
        disasters.append(disaster)
        for g, gen in generators.items():
            xi = extract_input_topography(x, topo_keys[g]) if compare == "topography" else x
            key = (g, disaster)
            if key not in grouped:
                grouped[key] = MaskConfusion(device)
            im_vals = score_batch(gen, xi, y, seg_model, im, [conf[g], grouped[key]])
            for k, v in zip(("PSNR", "SSIM", "MS-SSIM", "Inference"), im_vals):
                per[g][k].append(v)
    out = {}
    for g in generators:
        res = {k: float(np.mean(v)) for k, v in per[g].items() if k != "Inference"}
        res["LPIPS"] = float("nan")
        res.update(conf[g].compute())
        inf = per[g]["Inference"][5:] if g == next(iter(generators)) else per[g]["Inference"]   # group.py:198-200
        res["Inference"] = float(np.mean(inf)) if inf else float("nan")
        out[g] = {k: res[k] for k in METRIC_NAMES + ["Inference"]}
    by_disaster = {}
    for (g, d), c in grouped.items():
        vals = {k: float(np.mean([v for v, dd in zip(per[g][k], disasters) if dd == d]))
                for k in ("PSNR", "SSIM", "MS-SSIM")}
        vals["LPIPS"] = float("nan")
        vals.update(c.compute())
        by_disaster.setdefault(g, {})[d] = vals
    return out, by_disaster


def segmentation_model(seg_model_path=None, device="cuda"):
    return SegmentationModel(pretrained_model_path=seg_model_path, device=device).model
