"""Drop-in replacements for the PairedAttention modules of the reference
(models/model_architectures.py:305-441), running on libfloodgan's HIP kernels.

Same constructors, submodule names, parameter names / shapes / registration order (so
`state_dict()` checkpoints interoperate), same RNG consumption at construction (the layers
ARE nn.Conv2d / nn.ConvTranspose2d, so Model.initialise_weights, models/model.py:162-173,
re-initialises them), same forward signatures and `last_attention_mask`.  Only the arithmetic
differs: forward and backward of the whole network are single autograd nodes whose bodies
are the native executors in floodgan.executor.  There is no CPU path: tensors must live on
a HIP device (the modules raise otherwise).
"""
import torch
import torch.nn as nn

from . import executor as X


def _gen_keys():
    keys = []
    for n in X.generator_param_names():
        keys += [n + ".weight", n + ".bias"]
    return keys


def _disc_keys():
    keys = []
    for n in X.DISC_LAYERS:
        keys += [n + ".weight", n + ".bias"]
    return keys


GEN_KEYS = _gen_keys()
DISC_KEYS = _disc_keys()


class _GeneratorFn(torch.autograd.Function):
    """keys: the executor's names of `params` (GEN_KEYS, or CYCLEGAN_GEN_KEYS for the tanh-head
    generator, which returns an empty mask)."""

    @staticmethod
    def forward(ctx, keys, x, *params):
        P = dict(zip(keys, params))
        save = any(ctx.needs_input_grad)
        out, mask, S = X.gen_forward(P, x, save=save)
        if mask is None:
            mask = out.new_empty(0)
        ctx.keys, ctx.P, ctx.S = keys, P, S
        # the caller-visible tensors the backward reads (input, parameters) go through
        # save_for_backward so an in-place change between forward and backward raises
        ctx.save_for_backward(x, *params)
        if mask.numel() == 0:
            ctx.mark_non_differentiable(mask)
        # the mask stays in the graph as in the reference (attention10, models/model_architectures.py:396):
        # a loss on last_attention_mask back-propagates through the softmax; unused outputs arrive as None
        ctx.set_materialize_grads(False)
        return out, mask

    @staticmethod
    def backward(ctx, g_out, g_mask):
        _ = ctx.saved_tensors          # version check of the input and the parameters
        x = ctx.S["x"]
        if g_out is None:
            g_out = torch.zeros(x.shape[0], 3, x.shape[2], x.shape[3], dtype=torch.float32, device=x.device)
        gx = None
        if ctx.needs_input_grad[1]:   # the cycle path: G(cat(G'(x), conditions)) (models/model.py:677-706)
            gx = torch.empty(x.shape, dtype=torch.float32, device=g_out.device)
        grads = X.gen_backward(ctx.P, ctx.S, g_out, input_grad=gx,
                               g_mask=None if g_mask is None or g_mask.numel() == 0 else g_mask)
        ctx.S = None
        return (None, gx) + tuple(grads[k] if need else None
                                  for k, need in zip(ctx.keys, ctx.needs_input_grad[2:]))


class _DiscriminatorFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, *params):
        P = dict(zip(DISC_KEYS, params))
        buf = X.disc_pack([(x, None)], x.shape[1])
        pred, S = X.disc_forward(P, buf, save=any(ctx.needs_input_grad))
        ctx.P, ctx.S, ctx.xshape = P, S, tuple(x.shape)
        # the input too: an in-place change of D's input between forward and backward raises, as in autograd
        ctx.save_for_backward(x, *params)
        return pred

    @staticmethod
    def backward(ctx, g_pred):
        _ = ctx.saved_tensors          # version check of the input and the parameters
        need_params = any(ctx.needs_input_grad[1:])
        gx = None
        if ctx.needs_input_grad[0]:
            N, C, H, W = ctx.xshape
            gx = torch.empty(N, C, H, W, dtype=torch.float32, device=g_pred.device)
        grads = X.disc_backward(ctx.P, ctx.S, g_pred.contiguous(), param_grads=need_params, input_grad=gx,
                                input_grad_channels=(0, ctx.xshape[1]))
        ctx.S = None
        return (gx,) + tuple(grads.get(k) if need else None for k, need in zip(DISC_KEYS, ctx.needs_input_grad[1:]))


class PairedAttentionGenerator(nn.Module):
    """models/model_architectures.py:305-400 -- ResNet-9 encoder/decoder with a tanh content
    head (27 ch) and a softmax attention head (10 ch) composited with input[:, :3]."""

    _block = None   # the residual block class (set below: PairedAttentionBlock)

    def __init__(self, input_channels):
        super().__init__()
        self.input_channels = input_channels
        self.last_attention_mask = None
        self.conv1 = nn.Conv2d(input_channels, 64, kernel_size=7, stride=1, padding=0)
        self.conv1_norm = nn.InstanceNorm2d(64)
        self.conv2 = nn.Conv2d(64, 128, kernel_size=3, stride=2, padding=1)
        self.conv2_norm = nn.InstanceNorm2d(128)
        self.conv3 = nn.Conv2d(128, 256, kernel_size=3, stride=2, padding=1)
        self.conv3_norm = nn.InstanceNorm2d(256)
        self.resnet_blocks = nn.Sequential(*[self._block(256, 3, 1, 1) for _ in range(9)])
        self.deconv1_content = nn.ConvTranspose2d(256, 128, kernel_size=3, stride=2, padding=1, output_padding=1)
        self.deconv1_norm_content = nn.InstanceNorm2d(128)
        self.deconv2_content = nn.ConvTranspose2d(128, 64, kernel_size=3, stride=2, padding=1, output_padding=1)
        self.deconv2_norm_content = nn.InstanceNorm2d(64)
        self.deconv3_content = nn.Conv2d(64, 27, kernel_size=7, stride=1, padding=0)
        self.deconv1_attention = nn.ConvTranspose2d(256, 128, kernel_size=3, stride=2, padding=1, output_padding=1)
        self.deconv1_norm_attention = nn.InstanceNorm2d(128)
        self.deconv2_attention = nn.ConvTranspose2d(128, 64, kernel_size=3, stride=2, padding=1, output_padding=1)
        self.deconv2_norm_attention = nn.InstanceNorm2d(64)
        self.deconv3_attention = nn.Conv2d(64, 10, kernel_size=1, stride=1, padding=0)
        self.tanh = nn.Tanh()
        self.softmax = nn.Softmax(dim=1)

    def param_dict(self):
        sd = dict(self.named_parameters())
        return {k: sd[k] for k in GEN_KEYS}

    def forward(self, input):
        params = [p for p in self.param_dict().values()]
        out, mask = _GeneratorFn.apply(tuple(GEN_KEYS), input, *params)
        self.last_attention_mask = mask
        return out


class PairedAttentionBlock(nn.Module):
    """models/model_architectures.py:402-418.  Inside the generator the blocks are executed by
    the fused generator node; called on its own a block runs the same kernels through a
    3-module generator-free path (forward only is needed by no caller of the reference)."""

    def __init__(self, channel, kernel, stride, padding):
        super().__init__()
        self.padding = padding
        self.conv1 = nn.Conv2d(channel, channel, kernel, stride, 0)
        self.conv1_norm = nn.InstanceNorm2d(channel)
        self.conv2 = nn.Conv2d(channel, channel, kernel, stride, 0)
        self.conv2_norm = nn.InstanceNorm2d(channel)

    def forward(self, input):
        return _BlockFn.apply(input, self.conv1.weight, self.conv1.bias, self.conv2.weight, self.conv2.bias)


class _BlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        out, S = X.block_forward_nchw(x, {"w1": w1, "b1": b1, "w2": w2, "b2": b2}, save=any(ctx.needs_input_grad))
        ctx.S = S
        ctx.save_for_backward(w1, b1, w2, b2)
        return out

    @staticmethod
    def backward(ctx, g):
        _ = ctx.saved_tensors          # version check of the parameters
        gx, grads = X.block_backward_nchw(ctx.S, g, need_input=ctx.needs_input_grad[0])
        ctx.S = None
        return (gx,) + tuple(grads[k] if need else None
                             for k, need in zip(("w1", "b1", "w2", "b2"), ctx.needs_input_grad[1:]))


class PairedAttentionDiscriminator(nn.Module):
    """models/model_architectures.py:420-441 -- 70x70 PatchGAN over input_channels + 3."""

    _extra_channels = 3   # D sees cat(input, image) in the paired path (models/model.py:616-617)

    def __init__(self, input_channels):
        super().__init__()
        c0 = input_channels + self._extra_channels
        sequence = [nn.Conv2d(c0, 64, kernel_size=4, stride=2, padding=1), nn.LeakyReLU(0.2, True)]
        nf_mult = 1
        for n in range(1, 3):
            nf_prev, nf_mult = nf_mult, min(2 ** n, 8)
            sequence += [nn.Conv2d(64 * nf_prev, 64 * nf_mult, kernel_size=4, stride=2, padding=1, bias=True),
                         nn.InstanceNorm2d(64 * nf_mult), nn.LeakyReLU(0.2, True)]
        sequence += [nn.Conv2d(64 * nf_mult, 512, kernel_size=4, stride=1, padding=1, bias=True),
                     nn.InstanceNorm2d(512), nn.LeakyReLU(0.2, True)]
        sequence += [nn.Conv2d(512, 1, kernel_size=4, stride=1, padding=1)]
        self.model = nn.Sequential(*sequence)

    def param_dict(self):
        sd = dict(self.named_parameters())
        return {k: sd[k] for k in DISC_KEYS}

    def forward(self, x):
        return _DiscriminatorFn.apply(x, *self.param_dict().values())


PairedAttentionGenerator._block = PairedAttentionBlock


# ------------------------------------------------------------------------------------------
# AttentionGAN (cycle path): the same generator graph, a PatchGAN over input_channels
# ------------------------------------------------------------------------------------------

class AttentionGANBlock(PairedAttentionBlock):
    """models/model_architectures.py:260-276 -- identical to PairedAttentionBlock."""


class AttentionGANGenerator(PairedAttentionGenerator):
    """models/model_architectures.py:163-258 -- layer for layer the PairedAttention generator
    (same names, shapes, registration order, forward :197-258 and last_attention_mask), so it
    runs on the same executor; train_cycle additionally needs its input gradient."""

    _block = AttentionGANBlock


class AttentionGANDiscriminator(PairedAttentionDiscriminator):
    """models/model_architectures.py:278-299 -- the PatchGAN over `input_channels` (the cycle
    path feeds it 9-channel images, models/model.py:693-727), not input_channels + 3."""

    _extra_channels = 0


# ------------------------------------------------------------------------------------------
# CycleGAN (cycle path): ResNet-9 generator with a single tanh head, the same PatchGAN
# ------------------------------------------------------------------------------------------

def _cyclegan_names():
    """executor name -> CycleGANGenerator parameter prefix (nn.Sequential indices of
    models/model_architectures.py:95-117: 1, 4, 7 convs; 10-18 blocks with conv_block.1 / .5;
    19, 22 transposed convs; 26 the 7x7 head)"""
    m = {"conv1": "model.1", "conv2": "model.4", "conv3": "model.7"}
    for i in range(9):
        m[f"resnet_blocks.{i}.conv1"] = f"model.{10 + i}.conv_block.1"
        m[f"resnet_blocks.{i}.conv2"] = f"model.{10 + i}.conv_block.5"
    m.update({"deconv1_content": "model.19", "deconv2_content": "model.22", "deconv3_content": "model.26"})
    return m


CYCLEGAN_NAMES = _cyclegan_names()
CYCLEGAN_GEN_KEYS = tuple(f"{n}.{s}" for n in CYCLEGAN_NAMES for s in ("weight", "bias"))


class CycleGANGenerator(nn.Module):
    """models/model_architectures.py:91-120 -- the same encoder / 9 residual blocks / decoder as the
    attention generators, one decoder, reflect-pad 3 + conv 7x7 64->3 + tanh.  Same Sequential
    layout (state_dict keys `model.<i>...`) and construction order (RNG parity); the whole network
    is one autograd node on the native executor (which sees it under its own layer names)."""

    def __init__(self, input_channels):
        super().__init__()
        model = [nn.ReflectionPad2d(3), nn.Conv2d(input_channels, 64, kernel_size=7, padding=0, bias=True),
                 nn.InstanceNorm2d(64), nn.ReLU(True)]
        for i in range(2):
            mult = 2 ** i
            model += [nn.Conv2d(64 * mult, 64 * mult * 2, kernel_size=3, stride=2, padding=1, bias=True),
                      nn.InstanceNorm2d(64 * mult * 2), nn.ReLU(True)]
        model += [CycleGANBlock(dim=256) for _ in range(9)]
        for i in range(2):
            mult = 2 ** (2 - i)
            model += [nn.ConvTranspose2d(64 * mult, int(64 * mult / 2), kernel_size=3, stride=2, padding=1,
                                         output_padding=1, bias=True),
                      nn.InstanceNorm2d(int(64 * mult / 2)), nn.ReLU(True)]
        model += [nn.ReflectionPad2d(3), nn.Conv2d(64, 3, kernel_size=7, padding=0), nn.Tanh()]
        self.model = nn.Sequential(*model)

    def param_dict(self):
        """parameters under the executor's layer names (CYCLEGAN_GEN_KEYS order)"""
        sd = dict(self.named_parameters())
        return {f"{n}.{s}": sd[f"{p}.{s}"] for n, p in CYCLEGAN_NAMES.items() for s in ("weight", "bias")}

    def forward(self, x):
        out, _ = _GeneratorFn.apply(CYCLEGAN_GEN_KEYS, x, *self.param_dict().values())
        return out


class CycleGANBlock(nn.Module):
    """models/model_architectures.py:122-134 -- x + IN(conv(pad(ReLU(IN(conv(pad(x))))))), the
    PairedAttentionBlock computation under Sequential names (conv_block.1 / conv_block.5)."""

    def __init__(self, dim):
        super().__init__()
        self.conv_block = nn.Sequential(nn.ReflectionPad2d(1), nn.Conv2d(dim, dim, kernel_size=3, padding=0, bias=True),
                                        nn.InstanceNorm2d(dim), nn.ReLU(True), nn.ReflectionPad2d(1),
                                        nn.Conv2d(dim, dim, kernel_size=3, padding=0, bias=True),
                                        nn.InstanceNorm2d(dim))

    def forward(self, x):
        c1, c2 = self.conv_block[1], self.conv_block[5]
        return _BlockFn.apply(x, c1.weight, c1.bias, c2.weight, c2.bias)


class CycleGANDiscriminator(AttentionGANDiscriminator):
    """models/model_architectures.py:136-157 -- the same PatchGAN over input_channels."""


# ------------------------------------------------------------------------------------------
# Pix2Pix (paired path): U-Net-256 generator with BatchNorm / Dropout, BatchNorm PatchGAN
# ------------------------------------------------------------------------------------------

from . import pix2pix as P2P  # noqa: E402

PIX2PIX_GEN_KEYS = tuple(P2P.gen_state_keys())
PIX2PIX_DISC_KEYS = tuple(P2P.DISC_KEYS)


class _Pix2PixGeneratorFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, buffers, training, masks, x, *params):
        P = dict(zip(PIX2PIX_GEN_KEYS, params))
        out, S = P2P.gen_forward(P, buffers, x, masks=masks, training=training,
                                 save=any(ctx.needs_input_grad))
        ctx.P, ctx.S, ctx.training = P, S, training
        ctx.save_for_backward(x, *params)
        return out

    @staticmethod
    def backward(ctx, g_out):
        _ = ctx.saved_tensors          # version check of the input and the parameters
        if not ctx.training:
            raise RuntimeError("floodgan: the Pix2Pix generator's backward is implemented for training-mode "
                               "BatchNorm (the reference trains and evaluates in training mode)")
        if ctx.needs_input_grad[3]:
            raise RuntimeError("floodgan: the Pix2Pix generator does not provide an input gradient (no caller of "
                               "the reference needs one)")
        grads = P2P.gen_backward(ctx.P, ctx.S, g_out)
        ctx.S = None
        return (None, None, None, None) + tuple(grads[k] if need else None
                                                for k, need in zip(PIX2PIX_GEN_KEYS, ctx.needs_input_grad[4:]))


class _Pix2PixDiscriminatorFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, buffers, training, x, *params):
        P = dict(zip(PIX2PIX_DISC_KEYS, params))
        buf = X.disc_pack([(x, None)], x.shape[1])
        pred, S = P2P.disc_forward(P, buffers, buf, 1, training, save=any(ctx.needs_input_grad))
        ctx.P, ctx.S, ctx.xshape, ctx.training = P, S, tuple(x.shape), training
        ctx.save_for_backward(*params)
        return pred

    @staticmethod
    def backward(ctx, g_pred):
        _ = ctx.saved_tensors
        if not ctx.training:
            raise RuntimeError("floodgan: the Pix2Pix discriminator's backward is implemented for training-mode "
                               "BatchNorm")
        need_params = any(ctx.needs_input_grad[3:])
        gx = None
        if ctx.needs_input_grad[2]:
            N, C, H, W = ctx.xshape
            gx = torch.empty(N, C, H, W, dtype=torch.float32, device=g_pred.device)
        grads = P2P.disc_backward(ctx.P, ctx.S, g_pred.contiguous(), param_grads=need_params, input_grad=gx,
                                  input_grad_channels=(0, ctx.xshape[1]))
        ctx.S = None
        return (None, None, gx) + tuple(grads.get(k) if need else None
                                        for k, need in zip(PIX2PIX_DISC_KEYS, ctx.needs_input_grad[3:]))


class Pix2PixBlock(nn.Module):
    """models/model_architectures.py:24-62 -- the same modules in the same construction order (RNG
    parity) and nn.Sequential layout (state_dict keys).  Executed by its Pix2PixGenerator's fused node."""

    def __init__(self, outer_nc, inner_nc, input_nc, submodule, outermost, innermost, use_dropout):
        super().__init__()
        self.outermost = outermost
        if input_nc is None:
            input_nc = outer_nc
        downconv = nn.Conv2d(input_nc, inner_nc, kernel_size=4, stride=2, padding=1, bias=False)
        downrelu = nn.LeakyReLU(0.2, True)
        uprelu = nn.ReLU(True)
        downnorm = nn.BatchNorm2d(inner_nc)
        upnorm = nn.BatchNorm2d(outer_nc)
        if outermost:
            upconv = nn.ConvTranspose2d(inner_nc * 2, outer_nc, kernel_size=4, stride=2, padding=1)
            model = [downconv, submodule, uprelu, upconv, nn.Tanh()]
        elif innermost:
            upconv = nn.ConvTranspose2d(inner_nc, outer_nc, kernel_size=4, stride=2, padding=1, bias=False)
            model = [downrelu, downconv, uprelu, upconv, upnorm]
        else:
            upconv = nn.ConvTranspose2d(inner_nc * 2, outer_nc, kernel_size=4, stride=2, padding=1, bias=False)
            model = [downrelu, downconv, downnorm, submodule, uprelu, upconv, upnorm]
            if use_dropout:
                model.append(nn.Dropout(0.5))
        self.model = nn.Sequential(*model)

    def forward(self, x):
        raise RuntimeError("floodgan: a Pix2PixBlock runs inside its Pix2PixGenerator's fused node; call the "
                           "generator")


class Pix2PixGenerator(nn.Module):
    """models/model_architectures.py:9-22 -- U-Net-256: eight Pix2PixBlocks, innermost first.  The
    whole network is one autograd node on floodgan.pix2pix; BatchNorm running statistics are updated
    in place.  dropout_rng: "host" (default since round 5: the masks the reference's CPU path draws from torch's
    generator, bit for bit, regenerated on the device -- floodgan.pix2pix, floodgan.torch_rng) or "device" (hashed
    keep decisions seeded from torch's CPU generator: no RNG parity, ~4 % faster)."""

    dropout_rng = "host"

    def __init__(self, input_channels):
        super().__init__()
        unet_block = Pix2PixBlock(512, 512, None, None, False, True, False)
        for _ in range(3):
            unet_block = Pix2PixBlock(512, 512, None, unet_block, False, False, True)
        unet_block = Pix2PixBlock(256, 512, None, unet_block, False, False, False)
        unet_block = Pix2PixBlock(128, 256, None, unet_block, False, False, False)
        unet_block = Pix2PixBlock(64, 128, None, unet_block, False, False, False)
        self.model = Pix2PixBlock(3, 64, input_channels, unet_block, True, False, False)

    def param_dict(self):
        sd = dict(self.named_parameters())
        return {k: sd[k] for k in PIX2PIX_GEN_KEYS}

    def buffer_dict(self):
        return dict(self.named_buffers())

    def forward(self, input):
        masks = (P2P.draw_dropout(input.shape[0], input.shape[2], input.shape[3], self.dropout_rng, input.device)
                 if self.training else None)
        return _Pix2PixGeneratorFn.apply(self.buffer_dict(), self.training, masks, input,
                                         *self.param_dict().values())


class Pix2PixDiscriminator(nn.Module):
    """models/model_architectures.py:64-85 -- PatchGAN over input_channels + 3 with BatchNorm."""

    def __init__(self, input_channels):
        super().__init__()
        sequence = [nn.Conv2d(input_channels + 3, 64, kernel_size=4, stride=2, padding=1), nn.LeakyReLU(0.2, True)]
        nf_mult = 1
        for n in range(1, 3):
            nf_prev, nf_mult = nf_mult, min(2 ** n, 8)
            sequence += [nn.Conv2d(64 * nf_prev, 64 * nf_mult, kernel_size=4, stride=2, padding=1, bias=False),
                         nn.BatchNorm2d(64 * nf_mult), nn.LeakyReLU(0.2, True)]
        sequence += [nn.Conv2d(64 * nf_mult, 512, kernel_size=4, stride=1, padding=1, bias=False),
                     nn.BatchNorm2d(512), nn.LeakyReLU(0.2, True)]
        sequence += [nn.Conv2d(512, 1, kernel_size=4, stride=1, padding=1)]
        self.model = nn.Sequential(*sequence)

    def param_dict(self):
        sd = dict(self.named_parameters())
        return {k: sd[k] for k in PIX2PIX_DISC_KEYS}

    def buffer_dict(self):
        return dict(self.named_buffers())

    def forward(self, x):
        return _Pix2PixDiscriminatorFn.apply(self.buffer_dict(), self.training, x, *self.param_dict().values())
