"""Golden vectors for the flood-segmentation UNet from the REAL reference class.

Runs only in the build container: imports the reference's models/model_architectures.py (torch only),
builds UNet() under torch.manual_seed(5), applies the reference SegmentationModel's initialise_weights
(models/segmentation_model.py:73-84, restated here: importing segmentation_model would need
torchmetrics) and runs the training-mode forward the evaluation uses (models/model.py:399-400) on
seeded [0, 1] images.  Only numbers are written (tests/golden/segmentation_unet_64.npz): parameter
checksums, the logits of two calls (batch 2 at 64x64, then batch 1 at 48x48 -- 48 exercises Up's size
padding) and the BatchNorm running statistics after them.

Usage:  python tests/golden/make_golden_segmentation.py
"""
import os
import sys

import numpy as np
import torch
from torch import nn

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def initialise_weights(m):
    classname = m.__class__.__name__
    if hasattr(m, "weight") and (classname.find("Conv") != -1 or classname.find("Linear") != -1):
        nn.init.normal_(m.weight.data, 0.0, 0.02)
        if hasattr(m, "bias") and m.bias is not None:
            nn.init.constant_(m.bias.data, 0.0)
    elif classname.find("BatchNorm2d") != -1:
        nn.init.normal_(m.weight.data, 1.0, 0.02)
        nn.init.constant_(m.bias.data, 0.0)


def checksums(sd):
    out = {}
    for name, p in sd.items():
        t = p.detach().double().flatten()
        idx = torch.linspace(0, t.numel() - 1, 16).long()
        out[name] = np.concatenate([[t.sum().item(), t.abs().sum().item()], t[:8].numpy(), t[idx].numpy()])
    return out


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from models import model_architectures as MA  # noqa: E402  (reference, imported read-only)
    torch.set_num_threads(8)
    torch.manual_seed(5)
    net = MA.UNet().apply(initialise_weights)
    rec = {}
    for k, v in checksums(net.state_dict()).items():
        rec["init/" + k] = v
    g = torch.Generator().manual_seed(77)
    x1 = torch.rand((2, 3, 64, 64), generator=g)
    x2 = torch.rand((1, 3, 48, 48), generator=g)
    with torch.no_grad():
        rec["logits_64"] = net(x1).numpy()
        rec["logits_48"] = net(x2).numpy()
    for k, v in checksums(net.state_dict()).items():
        rec["after/" + k] = v
    out = os.path.join(HERE, "segmentation_unet_64.npz")
    np.savez_compressed(out, **{k.replace(".", "__"): v for k, v in rec.items()})
    print("wrote", out)


if __name__ == "__main__":
    main()
