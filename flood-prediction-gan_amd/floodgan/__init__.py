"""floodgan -- MI355X-native (gfx950) PairedAttention paired-GAN training step.

Drop-in for the reference's hot path (Natasha-R/Flood-Prediction-GAN,
models/model_architectures.py:305-441 + models/model.py:598-658): the module classes and
the Model/train_paired API mirror the reference, the arithmetic runs in hand-written HIP
kernels (libfloodgan.so, C-ABI in include/floodgan.h).
"""
from ._lib import load as load_library  # noqa: F401
from .model_architectures import (AttentionGANBlock, AttentionGANDiscriminator,  # noqa: F401
                                  AttentionGANGenerator, CycleGANBlock, CycleGANDiscriminator, CycleGANGenerator, PairedAttentionBlock, PairedAttentionDiscriminator,
                                  PairedAttentionGenerator)

__all__ = ["PairedAttentionGenerator", "PairedAttentionBlock", "PairedAttentionDiscriminator",
           "AttentionGANGenerator", "AttentionGANBlock", "AttentionGANDiscriminator",
           "CycleGANGenerator", "CycleGANBlock", "CycleGANDiscriminator", "load_library"]
