"""Generate golden vectors for the PairedAttention training step from the REAL reference.

Runs only in the build container, where the reference is mounted read-only at
/root/reference.  It imports the reference's own `models/model.py` (third-party modules the
hot path never touches -- tifffile, torchvision.transforms, torchmetrics -- are replaced by
inert stand-ins), builds `Model(model="pairedattention", ...)` and
drives the UNMODIFIED `Model.train_paired()` (models/model.py:598-658) over synthetic tiles.

Nothing from the reference is copied into this repository: only the numeric results are
written, to tests/golden/paired_step_<R>.npz (numpy, no pickles).

Recorded per resolution R (batch N=2, input_channels=9, seed 47):
  * inputs x0, y0, x1, y1 (two iterations) ~ U[-1, 1) from torch.Generator().manual_seed(1234)
  * G(x0), last_attention_mask, D(cat(x0, y0)) at initialisation
  * per-parameter init checksums (float64 sum, abs-sum, first 8 values, 16 strided samples)
  * the four per-iteration losses of two training iterations (epochs 1 and 2 of one
    train_paired() call, one batch per epoch, lr 2e-4 then 1e-4 from the reference's LambdaLR);
    the L1 entry is the raw mean |fake - y| (the reference multiplies it by 100)
  * G(x0), D(cat(x0,y0)) and parameter checksums after each iteration

Usage:  python tests/golden/make_golden.py   (takes ~1 minute on 8 vCPU)
"""
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _install_stubs():
    class _Dummy:
        def __init__(self, *a, **k):
            pass

        def to(self, *a, **k):
            return self

        def __call__(self, *a, **k):
            raise RuntimeError("stubbed third-party callable invoked")

    def mod(name, **attrs):
        m = types.ModuleType(name)
        for k, v in attrs.items():
            setattr(m, k, v)
        sys.modules[name] = m
        return m

    mod("tifffile", imread=_Dummy(), imsave=_Dummy(), imwrite=_Dummy())
    tv = mod("torchvision")
    tvt = mod("torchvision.transforms", Resize=_Dummy, Normalize=_Dummy,
              InterpolationMode=types.SimpleNamespace(BICUBIC=3, BILINEAR=2, NEAREST=0))
    tv.transforms = tvt
    tm = mod("torchmetrics")
    tm.regression = mod("torchmetrics.regression", MeanSquaredError=_Dummy)
    tm.image = mod("torchmetrics.image", PeakSignalNoiseRatio=_Dummy,
                   StructuralSimilarityIndexMeasure=_Dummy,
                   MultiScaleStructuralSimilarityIndexMeasure=_Dummy)
    tm.image.lpip = mod("torchmetrics.image.lpip", LearnedPerceptualImagePatchSimilarity=_Dummy)
    tm.classification = mod("torchmetrics.classification", BinaryAccuracy=_Dummy,
                            BinaryF1Score=_Dummy, BinaryPrecision=_Dummy, BinaryRecall=_Dummy)


def checksums(module):
    out = {}
    for name, p in module.state_dict().items():
        t = p.detach().double().flatten()
        idx = torch.linspace(0, t.numel() - 1, 16).long()
        out[name] = np.concatenate([[t.sum().item(), t.abs().sum().item()],
                                    t[:8].numpy(), t[idx].numpy()]).astype(np.float64)
    return out


class _Recorder:
    """Wraps nn.MSELoss / nn.L1Loss instances to record every value they return."""

    def __init__(self, fn, log):
        self.fn, self.log = fn, log

    def __call__(self, *a):
        v = self.fn(*a)
        self.log.append(float(v.detach()))
        return v


def synth(R, N, gen):
    x = torch.rand((N, 9, R, R), generator=gen) * 2 - 1
    y = torch.rand((N, 3, R, R), generator=gen) * 2 - 1
    return x, y


def run(R, N=2):
    from models import model as M  # noqa: E402  (reference, imported read-only)

    torch.set_num_threads(8)
    m = M.Model(model="pairedattention", dataset_subset="usa", dataset_dem="same",
                data_path="/nonexistent", num_epochs=2, topography="all", resize=R,
                verbose=False)
    gen = torch.Generator().manual_seed(1234)
    x0, y0 = synth(R, N, gen)
    x1, y1 = synth(R, N, gen)
    rec = {}
    rec["x0"], rec["y0"], rec["x1"], rec["y1"] = (t.numpy() for t in (x0, y0, x1, y1))

    G, D = m.generator, m.discriminator
    with torch.no_grad():
        rec["init_g_out"] = G(x0).numpy()
        rec["init_mask"] = G.last_attention_mask.numpy()
        rec["init_d_out"] = D(torch.cat((x0, y0), 1)).numpy()
    for k, v in checksums(G).items():
        rec["init_G/" + k] = v
    for k, v in checksums(D).items():
        rec["init_D/" + k] = v

    mse_log, l1_log = [], []
    m.loss_func = _Recorder(m.loss_func, mse_log)
    m.l1_loss = _Recorder(m.l1_loss, l1_log)

    class _PerEpochLoader:
        """epoch e (1-based) sees the single batch (x_{e-1}, y_{e-1})"""

        def __init__(self, batches):
            self.batches, self.calls = batches, 0

        def __iter__(self):
            b = self.batches[self.calls]
            self.calls += 1
            return iter([b])

        def __len__(self):
            return 1

    m.train_loader = _PerEpochLoader([(x0, y0, ["synthetic"] * N), (x1, y1, ["synthetic"] * N)])
    lrs = []
    orig_save = m.save_results

    def _record(epoch, losses, epoch_start_time):
        it = epoch - 1
        # call order inside one iteration: D(fake) vs 0, D(real) vs 1, D(fake) vs 1 (+ l1)
        d_syn, d_real, g_syn = mse_log[-3:]
        rec[f"it{it}_lr"] = np.array([lrs[it]])
        rec[f"it{it}_losses"] = np.array([d_real, d_syn, g_syn, l1_log[-1]])
        with torch.no_grad():
            rec[f"it{it}_g_out"] = G(x0).numpy()
            rec[f"it{it}_mask"] = G.last_attention_mask.numpy()
            rec[f"it{it}_d_out"] = D(torch.cat((x0, y0), 1)).numpy()
        for k, v in checksums(G).items():
            rec[f"it{it}_G/" + k] = v
        for k, v in checksums(D).items():
            rec[f"it{it}_D/" + k] = v
        orig_save(epoch=epoch, losses=losses, epoch_start_time=epoch_start_time)
        lrs.append(m.optimizer_generator.param_groups[0]["lr"])

    m.save_results = _record
    lrs.append(m.optimizer_generator.param_groups[0]["lr"])
    # epochs 1 and 2 of the unmodified loop; LambdaLR (num_epochs=2): lr 2e-4 then 1e-4
    m.train_paired()
    rec["meta"] = np.array([R, N, 47, 2, 1234], dtype=np.int64)
    return rec


def main():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    _install_stubs()
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(REF)  # models/data.py reads metadata/dataset_split.csv relative to cwd
    try:
        for R in (32, 64):
            rec = run(R)
            out = os.path.join(HERE, f"paired_step_{R}.npz")
            np.savez_compressed(out, **{k.replace(".", "__"): v for k, v in rec.items()})
            print("wrote", out, "losses it0", rec["it0_losses"], "it1", rec["it1_losses"])
    finally:
        os.chdir(cwd)


if __name__ == "__main__":
    main()
