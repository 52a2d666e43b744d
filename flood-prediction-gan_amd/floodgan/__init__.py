"""floodgan -- MI355X-native (gfx950) PairedAttention paired-GAN training step and its neighbours.

Drop-in for the reference's hot path (Natasha-R/Flood-Prediction-GAN,
models/model_architectures.py:305-441 + models/model.py:598-658): the module classes and
the Model/train_paired API mirror the reference, the arithmetic runs in hand-written HIP
kernels (libfloodgan.so, C-ABI in include/floodgan.h).  Around it: the cycle models
(train_cycle), the tile data path (floodgan.data), Pix2Pix (U-Net-256 + BatchNorm PatchGAN) and the
evaluation path (segmentation U-Net, device metrics: floodgan.evaluate); torch.library operators in
floodgan.custom_ops.
"""
from ._lib import load as load_library  # noqa: F401
from .model_architectures import (AttentionGANBlock, AttentionGANDiscriminator,  # noqa: F401
                                  AttentionGANGenerator, CycleGANBlock, CycleGANDiscriminator, CycleGANGenerator,
                                  PairedAttentionBlock, PairedAttentionDiscriminator, PairedAttentionGenerator,
                                  Pix2PixBlock, Pix2PixDiscriminator, Pix2PixGenerator)
from .segmentation import UNet  # noqa: F401

__all__ = ["PairedAttentionGenerator", "PairedAttentionBlock", "PairedAttentionDiscriminator",
           "AttentionGANGenerator", "AttentionGANBlock", "AttentionGANDiscriminator",
           "CycleGANGenerator", "CycleGANBlock", "CycleGANDiscriminator",
           "Pix2PixGenerator", "Pix2PixBlock", "Pix2PixDiscriminator", "UNet", "load_library"]
