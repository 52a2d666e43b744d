"""torch.library registrations of the native paths (the "PyTorch-ROCm custom ops" surface of
BASELINE.json north_star): schema'd operators with fake (meta) implementations, so torch.compile /
torch.export / FakeTensor tracing see shapes without running HIP code, and autograd formulas.

  floodgan::paired_attention_generator(x, params) -> (out, mask)
      models/model_architectures.py:339-400 (also AttentionGAN's generator); params in
      model_architectures.GEN_KEYS order.
  floodgan::patchgan_discriminator(x, params) -> pred
      models/model_architectures.py:424-441 (InstanceNorm PatchGAN of PairedAttention / AttentionGAN /
      CycleGAN); params in model_architectures.DISC_KEYS order.
  floodgan::conv2d(x, weight, bias, stride, padding, reflect) -> y
      one forward convolution on the engine (f16x3 by default), NCHW in and out.

The drop-in modules keep their own autograd.Function (it holds the forward's activations for the
explicit backward); these operators are stateless by construction, so their backward -- itself an
opaque operator (floodgan::*_backward), so that tracing the backward sees fake shapes too -- re-runs
the forward with saving on: one extra forward per backward, the price of a traceable op.
"""
from typing import List, Tuple

import torch

from . import executor as X
from . import ops
from . import plans as PL
from ._lib import FG_PAD_REFLECT, FG_PAD_ZERO
from .model_architectures import DISC_KEYS, GEN_KEYS
from .plans import Buf


@torch.library.custom_op("floodgan::paired_attention_generator", mutates_args=(), device_types="cuda")
def paired_attention_generator(x: torch.Tensor, params: List[torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor]:
    out, mask, _ = X.gen_forward(dict(zip(GEN_KEYS, params)), x, save=False)
    return out, mask


@paired_attention_generator.register_fake
def _(x, params):
    N, _, H, W = x.shape
    return x.new_empty(N, 3, H, W), x.new_empty(N, H, W)


def _gen_setup(ctx, inputs, output):
    x, params = inputs
    ctx.save_for_backward(x, *params)


@torch.library.custom_op("floodgan::paired_attention_generator_backward", mutates_args=(), device_types="cuda")
def paired_attention_generator_backward(x: torch.Tensor, params: List[torch.Tensor], g_out: torch.Tensor,
                                        g_mask: torch.Tensor) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    """(dL/dx, [dL/dparam]) of the generator at (x, params) for dL/dout = g_out and dL/dmask = g_mask
    (re-runs the forward)"""
    P = dict(zip(GEN_KEYS, params))
    _, _, S = X.gen_forward(P, x, save=True)
    gx = torch.empty(x.shape, dtype=torch.float32, device=x.device)
    # an empty g_mask: no loss term reads the mask (the caller passes none)
    grads = X.gen_backward(P, S, g_out.contiguous(), input_grad=gx, g_mask=g_mask if g_mask.numel() else None)
    return gx, [grads[k] for k in GEN_KEYS]


@paired_attention_generator_backward.register_fake
def _(x, params, g_out, g_mask):
    return torch.empty_like(x), [torch.empty_like(p) for p in params]


def _gen_backward(ctx, g_out, g_mask):
    x, *params = ctx.saved_tensors
    # autograd materialises the gradient of an unused output as zeros (the mask's term is then a no-op add); with
    # materialize_grads off it arrives as None, passed on as an empty tensor (the operator's schema takes a Tensor)
    if g_mask is None:
        g_mask = g_out.new_empty(0)
    if g_out is None:
        g_out = torch.zeros((x.shape[0], 3) + tuple(x.shape[2:]), dtype=x.dtype, device=x.device)
    return torch.ops.floodgan.paired_attention_generator_backward(x, params, g_out, g_mask)


paired_attention_generator.register_autograd(_gen_backward, setup_context=_gen_setup)


@torch.library.custom_op("floodgan::patchgan_discriminator", mutates_args=(), device_types="cuda")
def patchgan_discriminator(x: torch.Tensor, params: List[torch.Tensor]) -> torch.Tensor:
    pred, _ = X.disc_forward(dict(zip(DISC_KEYS, params)), X.disc_pack([(x, None)], x.shape[1]), save=False)
    return pred


@patchgan_discriminator.register_fake
def _(x, params):
    N, _, H, W = x.shape
    h, W_ = H, W
    for k, s in ((4, 2), (4, 2), (4, 2), (4, 1), (4, 1)):
        h, W_ = PL.out_size(h, k, s, 1), PL.out_size(W_, k, s, 1)
    return x.new_empty(N, 1, h, W_)


def _disc_setup(ctx, inputs, output):
    x, params = inputs
    ctx.save_for_backward(x, *params)


@torch.library.custom_op("floodgan::patchgan_discriminator_backward", mutates_args=(), device_types="cuda")
def patchgan_discriminator_backward(x: torch.Tensor, params: List[torch.Tensor],
                                    g_pred: torch.Tensor) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    P = dict(zip(DISC_KEYS, params))
    _, S = X.disc_forward(P, X.disc_pack([(x, None)], x.shape[1]), save=True)
    gx = torch.empty(x.shape, dtype=torch.float32, device=x.device)
    grads = X.disc_backward(P, S, g_pred.contiguous(), param_grads=True, input_grad=gx,
                            input_grad_channels=(0, x.shape[1]))
    return gx, [grads[k] for k in DISC_KEYS]


@patchgan_discriminator_backward.register_fake
def _(x, params, g_pred):
    return torch.empty_like(x), [torch.empty_like(p) for p in params]


def _disc_backward(ctx, g_pred):
    x, *params = ctx.saved_tensors
    return torch.ops.floodgan.patchgan_discriminator_backward(x, params, g_pred)


patchgan_discriminator.register_autograd(_disc_backward, setup_context=_disc_setup)


@torch.library.custom_op("floodgan::conv2d", mutates_args=(), device_types="cuda")
def conv2d(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, stride: int, padding: int,
           reflect: bool) -> torch.Tensor:
    N, C, H, W = x.shape
    O, _, k, _ = weight.shape
    Xb = Buf.empty(N, H, W, PL.rup(C, 4), padding, x.device)
    ops.pack_input(x, C, None, 0, Xb, 0, N, FG_PAD_REFLECT if reflect else FG_PAD_ZERO)
    Ho, Wo = PL.out_size(H, k, stride, padding), PL.out_size(W, k, stride, padding)
    Y = Buf.empty(N, Ho, Wo, PL.rup(O, 4), 0, x.device)
    m = PL.wmap_conv_fwd(weight.shape, Xb.c)
    ops.conv([PL.conv_problem(Xb, padding, k, stride, ops.pack_weight(weight, m), m, Y, bias=bias)])
    return Y.interior()[..., :O].permute(0, 3, 1, 2).contiguous()


@conv2d.register_fake
def _(x, weight, bias, stride, padding, reflect):
    N, _, H, W = x.shape
    O, _, k, _ = weight.shape
    return x.new_empty(N, O, PL.out_size(H, k, stride, padding), PL.out_size(W, k, stride, padding))
