"""Training orchestration for the PairedAttention path, mirroring the reference's
`Model` (models/model.py:26-160) and `Model.train_paired` (models/model.py:598-658).

`PairedStep` is the fused device iteration: the exact sequence of models/model.py:615-646
(G forward; D step on fake(detached)+real with LSGAN MSE x0.5 and Adam(D); G step on the
UPDATED D with MSE(D(fake),1) + 100*L1 and Adam(G)) executed by the native executors with
no autograd graph, one fused 2N-image discriminator pass for the D step (InstanceNorm is
per-sample, so D(fake) and D(real) in one batch is the same computation), fused losses and
FusedAdam.  With torch.distributed initialised it performs batch-DP over RCCL.
"""
import itertools
import time

import numpy as np
import torch
from torch import nn
from torch.optim import lr_scheduler

from . import executor as X
from . import ops
from . import pix2pix as P2P
from .cycle import IDENTITY_KEYS, LOSS_KEYS, CycleStep
from .model_architectures import (AttentionGANDiscriminator, AttentionGANGenerator, CycleGANDiscriminator,
                                  CycleGANGenerator, PairedAttentionDiscriminator, PairedAttentionGenerator,
                                  Pix2PixDiscriminator, Pix2PixGenerator)
from .optim import FusedAdam
from .parallel import FlatGrads, world

TOPOGRAPHY_CHANNELS = {"all": 9, "map": 6, "dem": 4, "flow": 4, "river": 4, None: 3}


class PairedStep:
    """One paired-GAN training iteration on device tensors x [N,C,H,W], y [N,3,H,W].
    Returns a device tensor [D real, D synthetic, G synthetic, 100*L1] (models/model.py:648-651)."""

    def __init__(self, generator, discriminator, opt_g, opt_d, group=None):
        self.G, self.D = generator, discriminator
        self.opt_g, self.opt_d = opt_g, opt_d
        self.gp, self.dp = generator.param_dict(), discriminator.param_dict()
        # gradient buffers laid out in the order the backward completes them: each bucket's RCCL
        # all-reduce starts as soon as it is written and overlaps the rest of the backward
        self.gflat = FlatGrads(self.gp, X.gen_bucket_names())
        self.dflat = FlatGrads(self.dp, X.disc_bucket_names())
        self.group = group
        self.last_mask = None
        self.last_output = None
        # test instrumentation: when True, each call stores the activation decisions of its three
        # networks' passes in self.decisions ({"G": [...], "D": [fake, real, G-step]}, oracle order) and the
        # L1 term's sign decisions ({"L1": [{"l1": sign(fake - y)}]})
        self.record_decisions = False
        self.decisions = None
        # test instrumentation (teacher forcing): discriminator parameters {name: tensor} that replace the
        # result of Adam(D) before the G step, so that another implementation's G half can be compared on
        # the same discriminator (the oracle's d_after); the step's own Adam(D) result is kept in d_after_own
        self.d_after = None
        self.d_after_own = None

    def __call__(self, x, y):
        ws, _ = world()
        inv = 1.0 / ws
        N = x.shape[0]
        dev = x.device
        C = x.shape[1]
        losses = torch.empty(4, dtype=torch.float32, device=dev)
        # (the flat gradient views are attached right before each backward: the per-parameter checks then run on
        # the host while the GPU works through the forward instead of ahead of the step's first launch)
        # generator forward                                           (models/model.py:615)
        fake, mask, gS = X.gen_forward(self.gp, x, save=True)
        # ---- discriminator step: fake (detached) and real in one 2N batch   (:620-633)
        dinp = X.disc_pack([(x, fake), (x, y)], C + 3)
        pred, dS = X.disc_forward(self.dp, dinp, save=True)
        g_pred = torch.empty_like(pred)
        ops.mse_const(pred[:N], 0.0, 0.5 * inv, losses[1:2], g_pred[:N])
        ops.mse_const(pred[N:], 1.0, 0.5 * inv, losses[0:1], g_pred[N:])
        rec = {"G": [X.gen_act_decisions(gS)], "D": [X.disc_act_decisions(dS, 0, N), X.disc_act_decisions(dS, N)]} \
            if self.record_decisions else None
        self.dflat.attach()
        self.dflat.begin(self.group)
        X.disc_backward(self.dp, dS, g_pred, param_grads=True, grads_into=self._grads(self.dp),
                        ready=self.dflat.ready)
        del dS
        self.dflat.finish()
        self.opt_d.step()
        if self.d_after is not None:
            self.d_after_own = {k: p.detach().clone() for k, p in self.D.named_parameters()}
            with torch.no_grad():
                for k, p in self.D.named_parameters():
                    p.copy_(self.d_after[k])
        # ---- generator step against the updated discriminator                 (:636-646)
        dinp = X.disc_prefix(dinp, N)          # (x, fake): the D step's first half, unchanged since
        pred, dS = X.disc_forward(self.dp, dinp, save=True)
        g_pred = torch.empty_like(pred)
        ops.mse_const(pred, 1.0, inv, losses[2:3], g_pred)
        g_fake = torch.empty(N, 3, x.shape[2], x.shape[3], dtype=torch.float32, device=dev)
        ops.l1(fake, y, 100.0 * inv, losses[3:4], g_fake, loss_scale=100.0)     # logged as 100 * L1 (:643-651)
        X.disc_backward(self.dp, dS, g_pred, param_grads=False, input_grad=g_fake, input_grad_channels=(C, 3),
                        input_grad_accumulate=True)
        if rec is not None:
            rec["D"].append(X.disc_act_decisions(dS))
            rec["L1"] = [{"l1": torch.sign(fake.detach() - y)}]   # the L1 term's sign decisions (-1 / 0 / +1)
            self.decisions = rec
        del dS, dinp
        self.gflat.attach()
        self.gflat.begin(self.group)
        X.gen_backward(self.gp, gS, g_fake, grads_into=self._grads(self.gp), ready=self.gflat.ready)
        del gS
        self.gflat.finish()
        self.opt_g.step()
        self.last_mask, self.last_output = mask, fake
        return losses

    @staticmethod
    def _grads(params):
        return {k: p.grad for k, p in params.items()}


class Pix2PixStep(PairedStep):
    """The same iteration (models/model.py:611-651) for Pix2Pix: BatchNorm in training mode, so the D
    step's D(fake) and D(real) -- separate calls in the reference -- run as one 2N pass with two
    BatchNorm groups (per-half statistics, two running-stat updates in order), and the G step's D call
    updates the discriminator's running statistics a third time.  With dropout_rng "host" the generator's Dropout
    masks are torch's CPU stream in the reference's order, regenerated on the device (floodgan.torch_rng)."""

    def __init__(self, generator, discriminator, opt_g, opt_d, group=None):
        self.G, self.D = generator, discriminator
        self.opt_g, self.opt_d = opt_g, opt_d
        self.gp, self.dp = generator.param_dict(), discriminator.param_dict()
        self.gb, self.db = generator.buffer_dict(), discriminator.buffer_dict()
        self.gflat = FlatGrads(self.gp, P2P.gen_bucket_names())
        self.dflat = FlatGrads(self.dp, P2P.disc_bucket_names())
        self.group = group
        self.last_mask = None
        self.last_output = None
        self.record_decisions = False
        self.decisions = None
        self.masks = None        # test hook: dropout masks to use instead of drawing
        self.last_masks = None

    def __call__(self, x, y):
        N, C, H, W = x.shape
        commit = None
        if self.masks is not None:
            masks = self.masks
        elif self.G.dropout_rng == "host":
            masks, commit = P2P.draw_dropout_deferred(N, H, W, x.device)
        else:
            masks = P2P.draw_dropout(N, H, W, self.G.dropout_rng, x.device)
        self.last_masks = masks
        try:
            return self._iterate(x, y, masks)
        finally:
            # torch's CPU generator advanced past this iteration's Dropout draws -- also when the iteration raised
            # (its masks were drawn: a retry must not reuse them); commit() raises if anything drew in between
            if commit is not None:
                commit()

    def _iterate(self, x, y, masks):
        ws, _ = world()
        inv = 1.0 / ws
        N, C, H, W = x.shape
        dev = x.device
        losses = torch.empty(4, dtype=torch.float32, device=dev)
        fake, gS = P2P.gen_forward(self.gp, self.gb, x, masks=masks, training=True, save=True)
        dinp = X.disc_pack([(x, fake), (x, y)], C + 3)
        pred, dS = P2P.disc_forward(self.dp, self.db, dinp, groups=2, training=True, save=True)
        g_pred = torch.empty_like(pred)
        ops.mse_const(pred[:N], 0.0, 0.5 * inv, losses[1:2], g_pred[:N])
        ops.mse_const(pred[N:], 1.0, 0.5 * inv, losses[0:1], g_pred[N:])
        rec = {"G": [P2P.gen_act_decisions(gS)], "D": [P2P.disc_act_decisions(dS, 0, N),
                                                       P2P.disc_act_decisions(dS, N)]} \
            if self.record_decisions else None
        self.dflat.attach()
        self.dflat.begin(self.group)
        P2P.disc_backward(self.dp, dS, g_pred, param_grads=True, grads_into=self._grads(self.dp),
                          ready=self.dflat.ready)
        del dS
        self.dflat.finish()
        self.opt_d.step()
        dinp = X.disc_prefix(dinp, N)          # (x, fake): the D step's first half, unchanged since
        pred, dS = P2P.disc_forward(self.dp, self.db, dinp, groups=1, training=True, save=True)
        g_pred = torch.empty_like(pred)
        ops.mse_const(pred, 1.0, inv, losses[2:3], g_pred)
        g_fake = torch.empty(N, 3, H, W, dtype=torch.float32, device=dev)
        ops.l1(fake, y, 100.0 * inv, losses[3:4], g_fake, loss_scale=100.0)     # logged as 100 * L1 (:643-651)
        P2P.disc_backward(self.dp, dS, g_pred, param_grads=False, input_grad=g_fake, input_grad_channels=(C, 3),
                          input_grad_accumulate=True)
        if rec is not None:
            rec["D"].append(P2P.disc_act_decisions(dS))
            rec["L1"] = [{"l1": torch.sign(fake.detach() - y)}]   # the L1 term's sign decisions (-1 / 0 / +1)
            self.decisions = rec
        del dS, dinp
        self.gflat.attach()
        self.gflat.begin(self.group)
        P2P.gen_backward(self.gp, gS, g_fake, grads_into=self._grads(self.gp), ready=self.gflat.ready)
        del gS
        self.gflat.finish()
        self.opt_g.step()
        self.last_output = fake
        return losses


class Model:
    """The reference's Model (models/model.py:26-160) with identical construction semantics (seed,
    initialise_weights, Adam(2e-4, (0.5, 0.999)), LambdaLR) for "PairedAttention" (train_paired,
    the hot path) and the cycle models "AttentionGAN" / "CycleGAN" (train_cycle)."""

    def __init__(self, model="PairedAttention", dataset_subset="all", dataset_dem="best", data_path=None,
                 num_epochs=1, topography="all", resize=256, crop=None, save_model_interval=0,
                 save_images_interval=0, verbose=False, load_pretrained_model=False, pretrained_model_path=None,
                 add_identity_loss=False, training_model=True, seed=47, device="cuda", train_loader=None,
                 val_loader=None, test_loader=None, batch_size=1, num_workers=0,
                 csv_path="metadata/dataset_split.csv"):
        saved = None
        if load_pretrained_model:
            # models/model.py:52-57: the checkpoint, not the `model` argument, names the architecture
            saved = torch.load(pretrained_model_path, map_location="cpu", weights_only=True)
            model = saved["model"]
        self.model = model.lower()
        if self.model not in ("pairedattention", "pix2pix", "attentiongan", "cyclegan"):
            raise NotImplementedError("Model must be one of: Pix2Pix, CycleGAN, AttentionGAN or PairedAttention")
        if saved is not None:
            self.num_epochs, self.topography = saved["num_epochs"], saved["topography"]
            self.add_identity_loss = saved["add_identity_loss"]
        else:
            self.num_epochs, self.topography, self.add_identity_loss = num_epochs, topography, add_identity_loss
        self.verbose, self.save_model_interval = verbose, save_model_interval
        self.save_images_interval = save_images_interval
        self.load_pretrained_model, self.data_path = load_pretrained_model, data_path
        self.dataset_subset, self.dataset_dem, self.resize, self.crop = dataset_subset, dataset_dem, resize, crop
        self.training_model, self.seed, self.device = training_model, seed, device
        self.model_is_cycle = self.model in ("attentiongan", "cyclegan")
        self.model_is_attention = self.model in ("pairedattention", "attentiongan")     # models/model.py:219-229

        input_channels = TOPOGRAPHY_CHANNELS[self.topography]
        torch.manual_seed(self.seed)
        if self.model_is_cycle:                                   # models/model.py:96-100, :108-115
            self._init_cycle(input_channels, device)
        else:
            gcls, dcls = ((Pix2PixGenerator, Pix2PixDiscriminator) if self.model == "pix2pix"
                          else (PairedAttentionGenerator, PairedAttentionDiscriminator))
            self.generator = gcls(input_channels=input_channels).apply(self.initialise_weights).to(device)
        if self.training_model and not self.model_is_cycle:
            self.discriminator = dcls(input_channels=input_channels).apply(self.initialise_weights).to(device)
            self.optimizer_discriminator = FusedAdam(self.discriminator.parameters(), lr=0.0002, betas=(0.5, 0.999))
            self.optimizer_generator = FusedAdam(self.generator.parameters(), lr=0.0002, betas=(0.5, 0.999))
        if self.training_model:
            self.scheduler_generator = lr_scheduler.LambdaLR(self.optimizer_generator, lr_lambda=self.lambda_rule)
            self.scheduler_discriminator = lr_scheduler.LambdaLR(self.optimizer_discriminator,
                                                                 lr_lambda=self.lambda_rule)
        if saved is not None and self.model_is_cycle:
            self.starting_epoch, self.all_losses = saved["starting_epoch"], saved["all_losses"]
            for name in self._cycle_nets():
                getattr(self, name).load_state_dict(saved[name])
            if self.training_model:
                for name in ("optimizer_generator", "optimizer_discriminator", "scheduler_generator",
                             "scheduler_discriminator"):
                    getattr(self, name).load_state_dict(saved[name])
        elif saved is not None:
            self.starting_epoch, self.all_losses = saved["starting_epoch"], saved["all_losses"]
            self.generator.load_state_dict(saved["generator"])
            if self.training_model:
                self.discriminator.load_state_dict(saved["discriminator"])
                self.optimizer_discriminator.load_state_dict(saved["optimizer_discriminator"])
                self.optimizer_generator.load_state_dict(saved["optimizer_generator"])
                self.scheduler_discriminator.load_state_dict(saved["scheduler_discriminator"])
                self.scheduler_generator.load_state_dict(saved["scheduler_generator"])
        else:
            self.starting_epoch = 1
            self.all_losses = self.initialise_loss_storage(overall=True)
        self.current_epoch = self.starting_epoch
        # the data (models/model.py:150-156): with a data_path the three loaders are built as the reference
        # builds them -- floodgan.data's staged TileLoaders over the same split table (csv_path: the
        # reference reads metadata/dataset_split.csv relative to the working directory), batch_size images
        # per step (the reference's is 1) and, under torch.distributed, this rank's shard of every global
        # batch.  Loaders passed in explicitly (any iterable of (input, target, names)) take precedence.
        self.batch_size = batch_size
        if data_path is not None and train_loader is None:
            from .data import create_flood_dataset
            ws, rank = world()
            train_loader, val_loader, test_loader = create_flood_dataset(
                dataset_subset, dataset_dem, data_path, self.topography, resize=resize, crop=crop,
                batch_size=batch_size, num_workers=num_workers, csv_path=csv_path, device=device, rank=rank, world=ws)
        self.train_loader, self.val_loader, self.test_loader = train_loader, val_loader, test_loader
        self._step = None

    def _cycle_nets(self):
        nets = ["pre_to_post_generator", "post_to_pre_generator"]
        return nets + (["pre_discriminator", "post_discriminator"] if self.training_model else [])

    def _init_cycle(self, input_channels, device):
        """models/model.py:96-100 (construction order = RNG order) and :108-115 (optimisers)."""
        gcls, dcls = ((AttentionGANGenerator, AttentionGANDiscriminator) if self.model == "attentiongan"
                      else (CycleGANGenerator, CycleGANDiscriminator))
        for name in self._cycle_nets():
            cls = gcls if name.endswith("generator") else dcls
            setattr(self, name, cls(input_channels=input_channels).apply(self.initialise_weights).to(device))
        if self.training_model:
            self.optimizer_generator = FusedAdam(itertools.chain(self.pre_to_post_generator.parameters(),
                                                                 self.post_to_pre_generator.parameters()),
                                                 lr=0.0002, betas=(0.5, 0.999))
            self.optimizer_discriminator = FusedAdam(itertools.chain(self.post_discriminator.parameters(),
                                                                     self.pre_discriminator.parameters()),
                                                     lr=0.0002, betas=(0.5, 0.999))

    @staticmethod
    def initialise_weights(m):
        """models/model.py:162-173"""
        classname = m.__class__.__name__
        if hasattr(m, "weight") and (classname.find("Conv") != -1 or classname.find("Linear") != -1):
            nn.init.normal_(m.weight.data, 0.0, 0.02)
            if hasattr(m, "bias") and m.bias is not None:
                nn.init.constant_(m.bias.data, 0.0)
        elif classname.find("BatchNorm2d") != -1:
            nn.init.normal_(m.weight.data, 1.0, 0.02)
            nn.init.constant_(m.bias.data, 0.0)

    def lambda_rule(self, epoch):
        """models/model.py:175-181"""
        return 1.0 - max(0, epoch + 1 - (self.num_epochs / 2)) / float((self.num_epochs / 2) + 1)

    def initialise_loss_storage(self, overall):
        """models/model.py:183-205"""
        pre = "all_" if overall else ""
        if self.model_is_cycle:
            keys = LOSS_KEYS + (IDENTITY_KEYS if self.add_identity_loss else [])
            return {pre + k: [] for k in keys}
        return {f"{pre}losses_discriminator_real": [], f"{pre}losses_discriminator_synthetic": [],
                f"{pre}losses_generator_synthetic": [], f"{pre}l1_losses_generator_synthetic": []}

    @property
    def step_fn(self):
        if self._step is None:
            cls = Pix2PixStep if self.model == "pix2pix" else PairedStep
            self._step = cls(self.generator, self.discriminator, self.optimizer_generator, self.optimizer_discriminator)
        return self._step

    def train_paired(self):
        """models/model.py:598-658 on the fused device step."""
        if self.train_loader is None:
            raise RuntimeError("no training data: pass data_path (floodgan.data loaders, as models/model.py:150-156) "
                               "or train_loader (an iterable of (input, target, names))")
        keys = ["losses_discriminator_real", "losses_discriminator_synthetic", "losses_generator_synthetic",
                "l1_losses_generator_synthetic"]
        for epoch in range(self.starting_epoch, self.num_epochs + 1):
            t0 = time.time()
            losses = self.initialise_loss_storage(overall=False)
            self.discriminator.train()
            self.generator.train()
            torch.manual_seed(epoch)
            for input_stack, output_image, _ in self.train_loader:
                input_stack = input_stack.to(self.device, non_blocking=True)
                output_image = output_image.to(self.device, non_blocking=True)
                vals = self.step_fn(input_stack, output_image).cpu().tolist()
                for k, v in zip(keys, vals):
                    losses[k].append(v)
            self.scheduler_discriminator.step()
            self.scheduler_generator.step()
            self.save_results(epoch, losses, t0)

    @property
    def cycle_step_fn(self):
        if self._step is None:
            self._step = CycleStep(self.pre_to_post_generator, self.post_to_pre_generator, self.pre_discriminator,
                                   self.post_discriminator, self.optimizer_generator, self.optimizer_discriminator,
                                   identity=self.add_identity_loss)
        return self._step

    def train_cycle(self):
        """models/model.py:660-758 on the fused device step (CycleStep)."""
        if not self.model_is_cycle:
            raise RuntimeError("train_cycle needs model='AttentionGAN' or 'CycleGAN'")
        if self.train_loader is None:
            raise RuntimeError("no training data: pass data_path (floodgan.data loaders, as models/model.py:150-156) "
                               "or train_loader (an iterable of (input, target, names))")
        for epoch in range(self.starting_epoch, self.num_epochs + 1):
            t0 = time.time()
            losses = self.initialise_loss_storage(overall=False)
            for name in self._cycle_nets():
                getattr(self, name).train()
            torch.manual_seed(epoch)
            for input_stack, output_image, _ in self.train_loader:
                input_stack = input_stack.to(self.device, non_blocking=True)
                output_image = output_image.to(self.device, non_blocking=True)
                vals = self.cycle_step_fn(input_stack, output_image).cpu().tolist()
                for k, v in zip(losses.keys(), vals):
                    losses[k].append(v)
            self.scheduler_generator.step()
            self.scheduler_discriminator.step()
            self.save_results(epoch, losses, t0)

    def calculate_metrics(self, use_test_data=False, seg_model_path=None, seg_model=None):
        """models/model.py:363-422 on the device (floodgan.evaluate): the generator (pre_to_post for the
        cycle models) over the validation / test loader, PSNR / SSIM / MS-SSIM of its [0, 1] outputs,
        the segmentation U-Net's flood masks of output and target and their binary metrics.  Returns
        the one-row DataFrame the reference prints (and writes it under data_path/metrics/ when set)."""
        import pandas as pd

        from .evaluate import calculate_metrics, segmentation_model
        loader = self.test_loader if use_test_data else self.val_loader
        if loader is None:
            raise RuntimeError("assign Model.val_loader / Model.test_loader first (floodgan.data.create_flood_dataset)")
        seg = seg_model if seg_model is not None else segmentation_model(seg_model_path, self.device)
        gen = self.pre_to_post_generator if self.model_is_cycle else self.generator
        res = calculate_metrics(gen, loader, seg, self.topography, self.device)
        # the reference's table (models/model.py:419-422): one row, a "0" index column, written to
        # create_path("metric")
        df = pd.DataFrame([(k, v) for k, v in res.items()]).set_index(0).transpose()
        if self.verbose:
            print(df)
        if self.data_path:
            import os
            path = self.create_path("metric")
            os.makedirs(os.path.dirname(path), exist_ok=True)
            df.to_csv(path)
        return df

    def prettify_model_name(self, model_name=None):
        """models/model.py:231-239"""
        pretty = {"pix2pix": "Pix2Pix", "cyclegan": "CycleGAN", "attentiongan": "AttentionGAN",
                  "pairedattention": "PairedAttention"}
        return pretty[model_name.lower()] if model_name else pretty[self.model]

    def create_path(self, save_type, info=""):
        """models/model.py:241-258: the reference's file naming for models, metrics and images"""
        from datetime import datetime
        ext = {"image": ".png", "figure": ".png", "model": ".pth.tar", "metric": ".csv"}[save_type]
        now = str(datetime.now())[:-7].replace(" ", "-").replace(":", "-")
        identity = f"identity{self.add_identity_loss}" if self.model_is_cycle else ""
        path = (f"{self.data_path}/{save_type}s/"
                f"{self.prettify_model_name()}_{info}_epoch"
                f"{self.current_epoch if self.training_model else self.current_epoch - 1}_"
                f"{self.topography}Topography_{identity}_"
                f"{self.dataset_subset}Data_{self.dataset_dem}DEM_"
                f"resize{self.resize}_crop{self.crop}_"
                f"date{now}{ext}")
        return path.replace("__", "_")

    def save_results(self, epoch, losses, epoch_start_time):
        """models/model.py:322-358 (loss bookkeeping + checkpoint; plots are out of scope)."""
        self.current_epoch = epoch
        for key in self.all_losses.keys():
            self.all_losses[key].append(float(np.mean(losses[key[4:]])))
        if self.verbose:
            print(f"Epoch {epoch} ({time.time() - epoch_start_time:.2f} seconds) | "
                  + " | ".join(f"{k} = {v[-1]:.2f}" for k, v in self.all_losses.items()))
        if self.save_model_interval != 0 and epoch % self.save_model_interval == 0:
            path = self.create_path("model")                      # models/model.py:355-357
            if self.verbose:
                print(f"Saving {self.prettify_model_name()} model to {path}")
            torch.save(self.checkpoint(epoch), path)

    def checkpoint(self, epoch):
        if self.model_is_cycle:                                   # models/model.py:335-355 (cycle keys)
            ck = {"model": self.model, "starting_epoch": epoch + 1, "num_epochs": self.num_epochs,
                  "topography": self.topography, "all_losses": self.all_losses,
                  "add_identity_loss": self.add_identity_loss}
            for name in self._cycle_nets() + ["optimizer_generator", "optimizer_discriminator",
                                              "scheduler_generator", "scheduler_discriminator"]:
                ck[name] = getattr(self, name).state_dict()
            return ck
        return {"model": self.model, "starting_epoch": epoch + 1, "num_epochs": self.num_epochs,
                "topography": self.topography,
                "optimizer_generator": self.optimizer_generator.state_dict(),
                "optimizer_discriminator": self.optimizer_discriminator.state_dict(),
                "scheduler_generator": self.scheduler_generator.state_dict(),
                "scheduler_discriminator": self.scheduler_discriminator.state_dict(),
                "all_losses": self.all_losses, "add_identity_loss": self.add_identity_loss,
                "discriminator": self.discriminator.state_dict(), "generator": self.generator.state_dict()}
