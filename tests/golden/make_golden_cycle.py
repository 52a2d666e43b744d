"""Generate golden vectors for the AttentionGAN cycle training step from the REAL reference.

Runs only in the build container (the reference is mounted read-only at /root/reference),
with the same inert stand-ins for tifffile / torchvision.transforms / torchmetrics as
make_golden.py.  It builds `Model(model="attentiongan", topography="all", ...)` and drives
the UNMODIFIED `Model.train_cycle()` (models/model.py:660-758) over synthetic tiles.

Only numeric results are written (tests/golden/cycle_step_<R>[_id].npz for AttentionGAN,
tests/golden/cyclegan_step_<R>.npz for CycleGAN (models/model_architectures.py:91-157); no pickles).

Recorded per case (R = 32, batch N = 2, input_channels = 9, seed 47):
  * inputs x0, y0, x1, y1 ~ U[-1, 1) from torch.Generator().manual_seed(1234)
  * pre_to_post(x0), post_to_pre(cat(y0, x0[:, 3:])) and both attention masks, D_pre(x0),
    D_post(cat(y0, x0[:, 3:])) at initialisation
  * per-parameter init checksums of the four networks (same format as make_golden.py)
  * per iteration (two epochs of one batch each, lr 2e-4 then 1e-4): the loss values the
    reference appends (models/model.py:741-752) in its `losses` dict order, and the outputs
    and checksums after the iteration.  The image buffers (get_buffer_image,
    models/model.py:275-294) hold < 50 images throughout, so they return the new image and
    the unseeded `random` draw is never reached: the run is deterministic.

Usage:  python tests/golden/make_golden_cycle.py   (~1 minute on 8 vCPU)
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF, _install_stubs, checksums, synth  # noqa: E402

NETS = ("pre_to_post_generator", "post_to_pre_generator", "pre_discriminator", "post_discriminator")


def _eval(m, x0, y0, rec, pre):
    post = torch.cat((y0, x0[:, 3:]), 1)
    with torch.no_grad():
        rec[pre + "g_pre_to_post"] = m.pre_to_post_generator(x0).numpy()
        if m.model == "attentiongan":
            rec[pre + "mask_pre_to_post"] = m.pre_to_post_generator.last_attention_mask.numpy()
        rec[pre + "g_post_to_pre"] = m.post_to_pre_generator(post).numpy()
        if m.model == "attentiongan":
            rec[pre + "mask_post_to_pre"] = m.post_to_pre_generator.last_attention_mask.numpy()
        rec[pre + "d_pre"] = m.pre_discriminator(x0).numpy()
        rec[pre + "d_post"] = m.post_discriminator(post).numpy()
    for net in NETS:
        for k, v in checksums(getattr(m, net)).items():
            rec[f"{pre}{net}/{k}"] = v


def run(R, N=2, identity=False, model="attentiongan"):
    from models import model as M  # noqa: E402  (reference, imported read-only)

    torch.set_num_threads(8)
    m = M.Model(model=model, dataset_subset="usa", dataset_dem="same", data_path="/nonexistent",
                num_epochs=2, topography="all", resize=R, verbose=False, add_identity_loss=identity)
    gen = torch.Generator().manual_seed(1234)
    x0, y0 = synth(R, N, gen)
    x1, y1 = synth(R, N, gen)
    rec = {}
    rec["x0"], rec["y0"], rec["x1"], rec["y1"] = (t.numpy() for t in (x0, y0, x1, y1))
    _eval(m, x0, y0, rec, "init_")

    class _PerEpochLoader:
        def __init__(self, batches):
            self.batches, self.calls = batches, 0

        def __iter__(self):
            b = self.batches[self.calls]
            self.calls += 1
            return iter([b])

        def __len__(self):
            return 1

    m.train_loader = _PerEpochLoader([(x0, y0, ["synthetic"] * N), (x1, y1, ["synthetic"] * N)])
    orig_save = m.save_results
    keys = []

    def _record(epoch, losses, epoch_start_time):
        it = epoch - 1
        if not keys:
            keys.extend(losses.keys())
        rec[f"it{it}_losses"] = np.array([losses[k][-1] for k in keys])
        # train_cycle steps the LambdaLR schedulers before save_results (models/model.py:754-759)
        rec[f"it{it}_lr_after"] = np.array([m.optimizer_generator.param_groups[0]["lr"]])
        _eval(m, x0, y0, rec, f"it{it}_")
        orig_save(epoch=epoch, losses=losses, epoch_start_time=epoch_start_time)

    m.save_results = _record
    m.train_cycle()
    rec["loss_keys"] = np.array(keys)
    rec["meta"] = np.array([R, N, 47, 2, 1234, int(identity)], dtype=np.int64)
    return rec


def main():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    _install_stubs()
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(REF)  # models/data.py reads metadata/dataset_split.csv relative to cwd
    try:
        for model, R, identity in (("attentiongan", 32, False), ("attentiongan", 32, True), ("cyclegan", 32, False)):
            rec = run(R, identity=identity, model=model)
            kind = "cycle_step" if model == "attentiongan" else "cyclegan_step"
            out = os.path.join(HERE, f"{kind}_{R}{'_id' if identity else ''}.npz")
            np.savez_compressed(out, **{k.replace(".", "__"): v for k, v in rec.items()})
            print("wrote", out, "losses it0", rec["it0_losses"], "it1", rec["it1_losses"])
    finally:
        os.chdir(cwd)


if __name__ == "__main__":
    main()
