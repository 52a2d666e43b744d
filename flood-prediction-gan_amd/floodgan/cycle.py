"""The AttentionGAN cycle training iteration (models/model.py:660-758, Model.train_cycle) on the
native executors -- SURVEY.md §8(f) row 1.

AttentionGAN's generator is layer for layer the PairedAttention generator and its PatchGAN is
the same network over `input_channels`, so the cycle step reuses every kernel of the paired
path.  What is new on this path:

* the generator's input gradient (executor.gen_backward(input_grad=...)): the recreated images
  G'(cat(G(x), conditions)) back-propagate through one generator into the other;
* a generator applied several times per iteration (x, the synthetic image, the identity
  image) accumulates its weight gradients (gen_backward(accumulate=True));
* the `torch.cat((image, conditions), 1)` inputs (models/model.py:682-689) are packed straight
  into the generator's / discriminator's padded NHWC input, never materialised;
* the discriminator input gradient lands directly in the channels 0..2 of the downstream
  generator's input gradient (the `cat` adjoint), so d/d(synthetic image) is summed in place;
* the image pool (get_buffer_image, models/model.py:275-294) stays on the device instead of
  the reference's `.cpu()` round trip.

As in the paired step there is no autograd graph; `CycleStep` returns the loss values in the
reference's `losses` dict order (models/model.py:189-199 / :741-752).
"""
import random

import torch

from . import executor as X
from . import ops
from .parallel import FlatGrads, world

LOSS_KEYS = ["losses_generator_post", "losses_generator_pre", "losses_pre_to_post_cycle", "losses_post_to_pre_cycle",
             "losses_discriminator_pre_real", "losses_discriminator_post_real", "losses_discriminator_pre_synthetic",
             "losses_discriminator_post_synthetic"]
IDENTITY_KEYS = ["losses_identity_post", "losses_identity_pre"]
# the reference's loss multipliers (models/model.py:698-711): cycle x10, identity x5
_SCALE = [1.0, 1.0, 10.0, 10.0, 1.0, 1.0, 1.0, 1.0, 5.0, 5.0]


class ImagePool:
    """models/model.py:275-294 on the device: while fewer than `size` images are stored, store and
    return the new one; afterwards with probability 1/2 swap it for a random stored one.  The
    reference draws from the unseeded global `random`; pass `rng` for a reproducible pool.
    Images are (synthetic [N,3,H,W], conditions [N,C-3,H,W]) pairs -- the cat of the reference."""

    def __init__(self, size=50, rng=None):
        self.size, self.images, self.rng = size, [], rng or random

    def __call__(self, image, conditions):
        # the caller may reuse its input tensor next step; conditions is None without topography
        item = (image, None if conditions is None else conditions.clone())
        if len(self.images) < self.size:
            self.images.append(item)
            return image, conditions
        if self.rng.uniform(0, 1) > 0.5:
            i = self.rng.randint(0, self.size - 1)
            old, self.images[i] = self.images[i], item
            return old
        return image, conditions


class CycleStep:
    """One AttentionGAN cycle iteration on device tensors input_stack [N,C,H,W] (pre-flood RGB +
    conditions) and output_image [N,3,H,W] (post-flood RGB), models/model.py:677-752."""

    def __init__(self, g_pre_to_post, g_post_to_pre, d_pre, d_post, opt_g, opt_d, identity=False, pool_rng=None,
                 group=None):
        self.g1, self.g2 = g_pre_to_post.param_dict(), g_post_to_pre.param_dict()
        self.dpre, self.dpost = d_pre.param_dict(), d_post.param_dict()
        self.opt_g, self.opt_d = opt_g, opt_d
        self.identity, self.group = identity, group
        # one flat gradient buffer per optimiser group, laid out bucket by bucket in the order the
        # backward completes them (each generator's buckets complete in its LAST backward pass of
        # the iteration, each discriminator's in its D-step backward); each bucket's all-reduce
        # starts as soon as it is written (parallel.FlatGrads)
        gnamed = {f"{t}.{k}": v for t, P in (("g1", self.g1), ("g2", self.g2)) for k, v in P.items()}
        gb = [[f"{t}.{n}" for n in b] for t in ("g1", "g2") for b in X.gen_bucket_names(self.g1)]
        self.gflat = FlatGrads(gnamed, gb)
        dnamed = {f"{t}.{k}": v for t, P in (("dpre", self.dpre), ("dpost", self.dpost)) for k, v in P.items()}
        db = [[f"{t}.{n}" for n in b] for t in ("dpre", "dpost") for b in X.disc_bucket_names()]
        self.dflat = FlatGrads(dnamed, db)
        self.pre_pool, self.post_pool = ImagePool(rng=pool_rng), ImagePool(rng=pool_rng)
        self.last = {}
        # test instrumentation: when True, each call stores every network pass's activation decisions
        # in self.decisions, keyed like the oracle's networks, each list in that network's call order
        self.record_decisions = False
        self.decisions = None

    @staticmethod
    def _grads(params):
        return {k: p.grad for k, p in params.items()}

    def __call__(self, x, y):
        ws, _ = world()
        inv = 1.0 / ws
        N, C, H, W = x.shape
        dev = x.device
        # models/model.py:682-689: with topography the conditions (input channels 3..) are cat'ed to
        # every image a generator or discriminator sees; without (C == 3) nothing is cat'ed
        cond = x[:, 3:] if C > 3 else None
        losses = torch.zeros(10, dtype=torch.float32, device=dev)

        def ready(flat, tag):
            return lambda name: flat.ready(f"{tag}.{name}")
        # ---- generators forward                                                 (:685-692)
        sp, mask_p, S_a = X.gen_forward(self.g1, x)                       # synthetic post
        spre, mask_q, S_b = X.gen_forward(self.g2, y, x_extra=cond)       # synthetic pre
        rp, _, S_c = X.gen_forward(self.g1, spre, x_extra=cond)           # recreated post
        rq, _, S_d = X.gen_forward(self.g2, sp, x_extra=cond)             # recreated pre
        # ---- generator losses (discriminators frozen)                           (:694-712)
        g_rq = torch.empty(N, 3, H, W, dtype=torch.float32, device=dev)
        ops.l1(rq, x[:, :3], 10.0 * inv, losses[2:3], g_rq)
        g_rp = torch.empty_like(g_rq)
        ops.l1(rp, y, 10.0 * inv, losses[3:4], g_rp)
        rec = None
        if self.record_decisions:
            rec = {"pre_to_post": [X.gen_act_decisions(S_a), X.gen_act_decisions(S_c)],
                   "post_to_pre": [X.gen_act_decisions(S_b), X.gen_act_decisions(S_d)], "pre_d": [], "post_d": []}
        preds = []
        for params, img, slot, net in ((self.dpost, sp, 0, "post_d"), (self.dpre, spre, 1, "pre_d")):
            pred, dS = X.disc_forward(params, X.disc_pack([(img, cond)], C), save=True)
            g_pred = torch.empty_like(pred)
            ops.mse_const(pred, 1.0, inv, losses[slot:slot + 1], g_pred)
            preds.append((params, dS, g_pred))
            if rec is not None:
                rec[net].append(X.disc_act_decisions(dS))
        # ---- generator backward: second round first; its input gradient, plus the frozen
        # discriminator's, is d/d(first-round output).  A generator's gradient buckets are complete
        # (and start their all-reduce) in its last backward of the iteration.
        # the flat gradient views, attached once the forward is queued (the host checks overlap the GPU's work)
        self.gflat.attach()
        self.dflat.attach()
        g1g, g2g = self._grads(self.g1), self._grads(self.g2)
        self.gflat.begin(self.group)
        last1 = None if self.identity else ready(self.gflat, "g1")
        last2 = None if self.identity else ready(self.gflat, "g2")
        gx_d = torch.empty(N, C, H, W, dtype=torch.float32, device=dev)
        X.gen_backward(self.g2, S_d, g_rq, grads_into=g2g, input_grad=gx_d)
        del S_d
        params, dS, g_pred = preds[0]
        X.disc_backward(params, dS, g_pred, param_grads=False, input_grad=gx_d, input_grad_channels=(0, 3),
                        input_grad_accumulate=True)
        gx_c = torch.empty(N, C, H, W, dtype=torch.float32, device=dev)
        X.gen_backward(self.g1, S_c, g_rp, grads_into=g1g, input_grad=gx_c)
        del S_c
        params, dS, g_pred = preds[1]
        X.disc_backward(params, dS, g_pred, param_grads=False, input_grad=gx_c, input_grad_channels=(0, 3),
                        input_grad_accumulate=True)
        del preds, dS
        X.gen_backward(self.g1, S_a, gx_d[:, :3], grads_into=g1g, accumulate=True, ready=last1)
        del S_a
        X.gen_backward(self.g2, S_b, gx_c[:, :3], grads_into=g2g, accumulate=True, ready=last2)
        del S_b, gx_c, gx_d
        if self.identity:                                                     # (:700-702)
            for params, grads, a, b, target, slot, tag in ((self.g1, g1g, y, cond, y, 8, "g1"),
                                                           (self.g2, g2g, x, None, x[:, :3], 9, "g2")):
                out, _, S_i = X.gen_forward(params, a, x_extra=b)
                if rec is not None:
                    rec["pre_to_post" if tag == "g1" else "post_to_pre"].append(X.gen_act_decisions(S_i))
                g_i = torch.empty_like(g_rq)
                ops.l1(out, target, 5.0 * inv, losses[slot:slot + 1], g_i)
                X.gen_backward(params, S_i, g_i, grads_into=grads, accumulate=True, ready=ready(self.gflat, tag))
                del S_i
        self.gflat.finish()
        self.opt_g.step()
        # ---- discriminators: real and pooled synthetic in one 2N batch each    (:715-739)
        spre_b, cq = self.pre_pool(spre, cond)
        sp_b, cp = self.post_pool(sp, cond)
        self.dflat.begin(self.group)
        for params, real, real_extra, syn, syn_extra, slots, tag in (
                (self.dpre, x, None, spre_b, cq, (4, 6), "dpre"), (self.dpost, y, cond, sp_b, cp, (5, 7), "dpost")):
            pred, dS = X.disc_forward(params, X.disc_pack([(real, real_extra), (syn, syn_extra)], C), save=True)
            if rec is not None:
                rec[tag[1:] + "_d"] += [X.disc_act_decisions(dS, 0, N), X.disc_act_decisions(dS, N)]
            g_pred = torch.empty_like(pred)
            ops.mse_const(pred[:N], 1.0, 0.5 * inv, losses[slots[0]:slots[0] + 1], g_pred[:N])
            ops.mse_const(pred[N:], 0.0, 0.5 * inv, losses[slots[1]:slots[1] + 1], g_pred[N:])
            X.disc_backward(params, dS, g_pred, param_grads=True, grads_into=self._grads(params),
                            ready=ready(self.dflat, tag))
            del dS
        self.dflat.finish()
        self.opt_d.step()
        self.decisions = rec
        self.last = dict(synthetic_post=sp, synthetic_pre=spre, mask_pre_to_post=mask_p, mask_post_to_pre=mask_q,
                         recreated_post=rp, recreated_pre=rq)
        n = 10 if self.identity else 8
        return losses[:n] * torch.tensor(_SCALE[:n], device=dev)
