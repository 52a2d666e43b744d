"""The flood-segmentation U-Net the evaluation scores generator outputs with:
drop-in modules and a native forward executor.

Reference: models/model_architectures.py:508-587 (UNet, DoubleConv, Down, Up, OutConv; milesial
style, bilinear=False), models/segmentation_model.py:19-72 (SegmentationModel: construction,
initialise_weights, checkpoint format).  The reference evaluates it without ever calling .eval()
(models/model.py:380-400, models/group.py:136-163): its BatchNorm layers run in training mode --
batch statistics, running statistics updated -- and so does this executor unless the module is put in
eval mode.

Layout.  Encoder level k (x1..x5 = 64..1024 channels at H / 2^(k-1)) is a DoubleConv (3x3 conv, no bias
-> BatchNorm -> ReLU, twice) whose last BatchNorm pass writes the level output twice: as the next
level's max-pool source and, for x1..x4, into the first channel half of the matching decoder level's
cat buffer (torch.cat([x2, x1], 1) of Up.forward, :579).  Each decoder level's ConvTranspose2d(2, 2)
(one tap per output phase: four 1x1 GEMMs, bias fused) writes straight into the second half.  The
1x1 OutConv produces the logits; the flood mask is sigmoid(logits) > 0.5.
"""
import torch
import torch.nn as nn

from . import ops
from . import pix2pix as P2P
from . import plans as PL
from ._lib import FG_ACT_RELU, FG_PAD_ZERO, require_device
from .plans import Buf, Slice

ENC = [64, 128, 256, 512, 1024]


def _dc(prefix):
    """(conv1, bn1, conv2, bn2) parameter prefixes of a DoubleConv at `prefix`"""
    return [f"{prefix}.double_conv.{i}" for i in (0, 1, 3, 4)]


def layer_names():
    """the executor's view of the state_dict: DoubleConvs by level, the up convs, the head"""
    enc = [_dc("inc")] + [_dc(f"down{k}.maxpool_conv.1") for k in range(1, 5)]
    dec = [(f"up{k}.up", _dc(f"up{k}.conv")) for k in range(1, 5)]
    return enc, dec, "outc.conv"


def check_input_size(H, W):
    if H % 16 or W % 16:
        raise RuntimeError(f"segmentation UNet: H, W must be multiples of 16 (got {H}x{W}); the reference pads the "
                           "up path for other sizes (models/model_architectures.py:575-578), which this executor "
                           "does not implement")


def _double_conv(P, B, names, X, mid, out, training, dsts):
    """DoubleConv over X (zero border 1): returns nothing; dsts = (dst0, dst1) of the second ReLU"""
    c1, b1, c2, b2 = names
    N, h, w = X.n, X.h, X.w
    dev = X.t.device
    t = Buf.empty(N, h, w, mid, 0, dev)
    P2P._conv_nb(P, c1, X, 1, 3, 1, t)
    mean, invstd = P2P._stats(B, b1, t, 1, training)
    a = Buf.zeros(N, h, w, mid, 1, dev)
    ops.bn_apply(t, 1, mean, invstd, P[b1 + ".weight"], P[b1 + ".bias"], None, FG_ACT_RELU, a)
    u = Buf.empty(N, h, w, out, 0, dev)
    P2P._conv_nb(P, c2, a, 1, 3, 1, u)
    mean, invstd = P2P._stats(B, b2, u, 1, training)
    ops.bn_apply(u, 1, mean, invstd, P[b2 + ".weight"], P[b2 + ".bias"], None, FG_ACT_RELU, dsts[0],
                 FG_ACT_RELU if dsts[1] is not None else 0, dsts[1])


def _convT2(P, name, X, Y):
    """ConvTranspose2d(k=2, s=2) over X (border >= 1) into Y (Buf or Slice): four single-tap phases"""
    w = P[name + ".weight"]
    maps = PL.phase_maps(w.shape, 2, 0, X.c)
    wps = [ops.pack_weight(w, m) for m, _, _ in maps]
    ops.conv(PL.phase_problems(X, w.shape, 2, 0, Y, wps, maps, bias=P.get(name + ".bias")))


def unet_logits(P, B, X0, training=True):
    """Forward of UNet(3, 1) over X0 (Buf: the [0, 1] image in channels 0..2 of 4, zero border 1).
    Returns the logits Buf [N, H, W, 4] (channel 0)."""
    N, H, W = X0.n, X0.h, X0.w
    check_input_size(H, W)
    dev = X0.t.device
    enc, dec, head = layer_names()
    cats = [Buf.zeros(N, H >> k, W >> k, 2 * ENC[k], 1, dev) for k in range(4)]     # decoder inputs by level
    X = X0
    for k in range(5):
        h, w = H >> k, W >> k
        if k < 4:
            x = Buf.empty(N, h, w, ENC[k], 0, dev)                 # max-pool source
            _double_conv(P, B, enc[k], X, ENC[k], ENC[k], training, (x, Slice(cats[k], 0, ENC[k])))
            X = Buf.zeros(N, h // 2, w // 2, ENC[k], 1, dev)
            ops.maxpool2(x, X)
        else:
            x5 = Buf.zeros(N, h, w, ENC[k], 1, dev)
            _double_conv(P, B, enc[k], X, ENC[k], ENC[k], training, (x5, None))
            X = x5
    for i, (up, names) in enumerate(dec):                            # up1 .. up4
        k = 3 - i                                                    # the encoder level it joins
        c = ENC[k]
        _convT2(P, up, X, Slice(cats[k], c, c))
        last = i == len(dec) - 1
        y = Buf.zeros(N, H >> k, W >> k, c, 0 if last else 1, dev)
        _double_conv(P, B, names, cats[k], c, c, training, (y, None))
        X = y
    logits = Buf.empty(N, H, W, 4, 0, dev)
    P2P._conv_nb(P, head, X, 0, 1, 1, logits)
    return logits


def unit_image(x, buf=None, nchw=True):
    """torch.clamp((x + 1) * 0.5, 0, 1) of an [N, C, H, W] generator output / target: (NCHW tensor or
    None, U-Net input Buf or None)"""
    require_device(x, "image")
    N, C, H, W = x.shape
    out = torch.empty(N, C, H, W, dtype=torch.float32, device=x.device) if nchw else None
    if buf is True:
        buf = Buf.zeros(N, H, W, PL.rup(C, 4), 1, x.device)
    from . import _lib as L
    L.check(L.load().fg_unit_image(ops.sview(x), N, C, H, W, L.ptr(out), ops.view(buf), L.stream_handle()),
            "unit_image")
    ops._wrote(buf)
    return out, buf


# ------------------------------------------------------------------------------------------ modules

def _sd_keys(module):
    return [k for k, _ in module.named_parameters()]


class _UNetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, module, x, *params):
        P = dict(zip(_sd_keys(module), params))
        B = dict(module.named_buffers())
        _, X0 = unit_image_passthrough(x)
        logits = unet_logits(P, B, X0, module.training)
        return logits.interior()[..., :1].permute(0, 3, 1, 2).contiguous()

    @staticmethod
    def backward(ctx, g):
        raise RuntimeError("floodgan: the segmentation UNet is evaluation-only (SURVEY.md §8(f) row 4); training it "
                           "(models/segmentation_model.py:250-277) is out of scope")


def unit_image_passthrough(x):
    """pack an [N, 3, H, W] image as the U-Net's NHWC input (no value change)"""
    require_device(x, "segmentation input")
    N, C, H, W = x.shape
    if C != 3:
        raise RuntimeError(f"segmentation UNet takes 3-channel images (got {C})")
    buf = Buf.zeros(N, H, W, 4, 1, x.device)
    ops.pack_input(x, 3, None, 0, buf, 0, N, FG_PAD_ZERO)
    return None, buf


class DoubleConv(nn.Module):
    """models/model_architectures.py:540-553"""

    def __init__(self, in_channels, out_channels, mid_channels=None):
        super().__init__()
        if not mid_channels:
            mid_channels = out_channels
        self.double_conv = nn.Sequential(
            nn.Conv2d(in_channels, mid_channels, kernel_size=3, padding=1, bias=False), nn.BatchNorm2d(mid_channels),
            nn.ReLU(inplace=True),
            nn.Conv2d(mid_channels, out_channels, kernel_size=3, padding=1, bias=False), nn.BatchNorm2d(out_channels),
            nn.ReLU(inplace=True))

    def forward(self, x):
        raise RuntimeError("floodgan: DoubleConv runs inside its UNet's native forward")


class Down(nn.Module):
    """models/model_architectures.py:555-562"""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.maxpool_conv = nn.Sequential(nn.MaxPool2d(2), DoubleConv(in_channels, out_channels))

    def forward(self, x):
        raise RuntimeError("floodgan: Down runs inside its UNet's native forward")


class Up(nn.Module):
    """models/model_architectures.py:564-580 (bilinear=False: ConvTranspose2d(in, in // 2, 2, 2))"""

    def __init__(self, in_channels, out_channels, bilinear=True):
        super().__init__()
        if bilinear:
            self.up = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)
            self.conv = DoubleConv(in_channels, out_channels, in_channels // 2)
        else:
            self.up = nn.ConvTranspose2d(in_channels, in_channels // 2, kernel_size=2, stride=2)
            self.conv = DoubleConv(in_channels, out_channels)

    def forward(self, x1, x2):
        raise RuntimeError("floodgan: Up runs inside its UNet's native forward")


class OutConv(nn.Module):
    """models/model_architectures.py:582-587"""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size=1)

    def forward(self, x):
        raise RuntimeError("floodgan: OutConv runs inside its UNet's native forward")


class UNet(nn.Module):
    """models/model_architectures.py:508-538 -- same modules, registration order and state_dict keys;
    forward = the native executor (logits [N, 1, H, W]); evaluation-only."""

    def __init__(self, n_channels=3, n_classes=1, bilinear=False):
        super().__init__()
        self.n_channels, self.n_classes, self.bilinear = n_channels, n_classes, bilinear
        self.inc = DoubleConv(n_channels, 64)
        self.down1 = Down(64, 128)
        self.down2 = Down(128, 256)
        self.down3 = Down(256, 512)
        factor = 2 if bilinear else 1
        self.down4 = Down(512, 1024 // factor)
        self.up1 = Up(1024, 512 // factor, bilinear)
        self.up2 = Up(512, 256 // factor, bilinear)
        self.up3 = Up(256, 128 // factor, bilinear)
        self.up4 = Up(128, 64, bilinear)
        self.outc = OutConv(64, n_classes)

    def _check(self):
        if self.bilinear or self.n_channels != 3 or self.n_classes != 1:
            raise NotImplementedError("floodgan's segmentation executor covers the reference's UNet(3, 1, "
                                      "bilinear=False) (models/segmentation_model.py:55)")

    def forward(self, x):
        self._check()
        return _UNetFn.apply(self, x, *[p for _, p in self.named_parameters()])

    def logits_from_buf(self, X0):
        """logits Buf from a prepared input Buf (the evaluation path: unit_image writes it directly)"""
        self._check()
        P = dict(self.named_parameters())
        B = dict(self.named_buffers())
        with torch.no_grad():
            return unet_logits(P, B, X0, self.training)


def initialise_weights(m):
    """models/segmentation_model.py:73-84 (the GAN's initialise_weights)"""
    classname = m.__class__.__name__
    if hasattr(m, "weight") and (classname.find("Conv") != -1 or classname.find("Linear") != -1):
        nn.init.normal_(m.weight.data, 0.0, 0.02)
        if hasattr(m, "bias") and m.bias is not None:
            nn.init.constant_(m.bias.data, 0.0)
    elif classname.find("BatchNorm2d") != -1:
        nn.init.normal_(m.weight.data, 1.0, 0.02)
        nn.init.constant_(m.bias.data, 0.0)


class SegmentationModel:
    """models/segmentation_model.py:19-72, the evaluation side: the UNet, initialised as the reference
    does (no reseeding: it draws from the global generator), optionally loaded from a checkpoint
    ({"model": state_dict, "current_epoch", "num_epochs", "all_losses", "all_accuracies"}, read with
    weights_only=True).  Training the segmentation model (train_model) is out of scope."""

    def __init__(self, data_path=None, pretrained_model_path=None, train=False, device="cuda", seed=47):
        if train:
            raise NotImplementedError("floodgan: segmentation-model training is out of scope (SURVEY.md §8(f) row 4 "
                                      "is evaluation inference)")
        self.data_path, self.pretrained_model_path, self.seed = data_path, pretrained_model_path, seed
        self.current_epoch, self.num_epochs, self.all_losses, self.all_accuracies = 1, 100, [], []
        self.model = UNet().apply(initialise_weights).to(device)
        if pretrained_model_path:
            saved = torch.load(pretrained_model_path, map_location="cpu", weights_only=True)
            self.current_epoch, self.num_epochs = saved["current_epoch"], saved["num_epochs"]
            self.model.load_state_dict(saved["model"])
            self.all_losses, self.all_accuracies = saved["all_losses"], saved["all_accuracies"]

    @staticmethod
    def tensor_to_mask(tensor, predicted=True):
        """models/segmentation_model.py:244-248"""
        return (torch.sigmoid(tensor) > 0.5).float() if predicted else (tensor > 0.5).float()
