"""Generate golden vectors for the Pix2Pix training step from the REAL reference.

Runs only in the build container (the reference is mounted read-only at /root/reference): imports the
reference's own models/model.py with the same inert stand-ins as make_golden.py, builds
Model(model="pix2pix", ...) and drives the UNMODIFIED Model.train_paired() (models/model.py:598-658)
over synthetic tiles.  Only numeric results are written (tests/golden/pix2pix_step_256.npz, no pickles).

Recorded (R=256 -- the U-Net-256's smallest input --, batch N=2, input_channels=9, seed 47):
  * inputs x0, y0, x1, y1 ~ U[-1, 1) from torch.Generator().manual_seed(1234) (regenerated, not stored)
  * state_dict checksums at initialisation (parameters AND BatchNorm buffers)
  * the four per-iteration losses of two training iterations (epochs 1 and 2: train_paired reseeds
    torch.manual_seed(epoch) at each epoch, which fixes the Dropout masks); L1 is the raw mean
  * state_dict checksums after each iteration (running statistics: three BatchNorm calls per
    iteration in the discriminator, one in the generator)
  * G(x0) and D(cat(x0, y0)) at init and after each iteration, evaluated in training mode on a deep
    copy under torch.manual_seed(99) inside fork_rng (G(x0) as sum, abs-sum and
    8192 strided samples) -- the model's own state and the training RNG
    stream are untouched by the recording

A second fixture, pix2pix_step_256_rgb_bs1.npz, records the same quantities for BASELINE.json configs[0]:
topography=None (3-ch RGB input, D over 3 + 3 channels), batch N=1, x ~ U[-1, 1)^(1,3,R,R) then
y ~ U[-1, 1)^(1,3,R,R) from the same generator.

Usage:  python tests/golden/make_golden_pix2pix.py [all|rgb]   (~1 minute each on 8 vCPU)
"""
import copy
import os
import sys

import numpy as np
import torch

from make_golden import REF, HERE, _install_stubs, _Recorder, checksums, synth

PROBE_SEED = 99
PROBE_SAMPLES = 8192


def probe(G, D, x0, y0):
    with torch.no_grad(), torch.random.fork_rng(devices=[]):
        torch.manual_seed(PROBE_SEED)
        g = copy.deepcopy(G)(x0).double().flatten()
        d = copy.deepcopy(D)(torch.cat((x0, y0), 1)).numpy()
    # the generator output as (sum, abs-sum, 8192 strided samples): the whole tensor would be 1.5 MB
    idx = torch.linspace(0, g.numel() - 1, PROBE_SAMPLES).long()
    return np.concatenate([[g.sum().item(), g.abs().sum().item()], g[idx].numpy()]), d


def synth_c(R, N, C, gen):
    x = torch.rand((N, C, R, R), generator=gen) * 2 - 1
    y = torch.rand((N, 3, R, R), generator=gen) * 2 - 1
    return x, y


def run(R=256, N=2, topography="all"):
    from models import model as M  # noqa: E402  (reference, imported read-only)

    torch.set_num_threads(8)
    m = M.Model(model="pix2pix", dataset_subset="usa", dataset_dem="same", data_path="/nonexistent",
                num_epochs=2, topography=topography, resize=R, verbose=False)
    gen = torch.Generator().manual_seed(1234)
    if topography == "all":
        x0, y0 = synth(R, N, gen)
        x1, y1 = synth(R, N, gen)
    else:
        C = m.generator.model.model[0].weight.shape[1]
        x0, y0 = synth_c(R, N, C, gen)
        x1, y1 = synth_c(R, N, C, gen)
    rec = {}   # the inputs are not stored: torch.Generator().manual_seed(1234) regenerates them
    G, D = m.generator, m.discriminator
    rec["init_g_out"], rec["init_d_out"] = probe(G, D, x0, y0)
    for k, v in checksums(G).items():
        rec["init_G/" + k] = v
    for k, v in checksums(D).items():
        rec["init_D/" + k] = v

    mse_log, l1_log = [], []
    m.loss_func = _Recorder(m.loss_func, mse_log)
    m.l1_loss = _Recorder(m.l1_loss, l1_log)

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
    lrs = [m.optimizer_generator.param_groups[0]["lr"]]
    orig_save = m.save_results

    def _record(epoch, losses, epoch_start_time):
        it = epoch - 1
        d_syn, d_real, g_syn = mse_log[-3:]
        rec[f"it{it}_lr"] = np.array([lrs[it]])
        rec[f"it{it}_losses"] = np.array([d_real, d_syn, g_syn, l1_log[-1]])
        rec[f"it{it}_g_out"], rec[f"it{it}_d_out"] = probe(G, D, x0, y0)
        for k, v in checksums(G).items():
            rec[f"it{it}_G/" + k] = v
        for k, v in checksums(D).items():
            rec[f"it{it}_D/" + k] = v
        orig_save(epoch=epoch, losses=losses, epoch_start_time=epoch_start_time)
        lrs.append(m.optimizer_generator.param_groups[0]["lr"])

    m.save_results = _record
    m.train_paired()
    rec["meta"] = np.array([R, N, 47, 2, 1234, PROBE_SEED], dtype=np.int64)
    return rec


def main():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    _install_stubs()
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(REF)
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    try:
        rec = run() if which == "all" else run(N=1, topography=None)
        out = os.path.join(HERE, "pix2pix_step_256.npz" if which == "all" else "pix2pix_step_256_rgb_bs1.npz")
        np.savez_compressed(out, **{k.replace(".", "__"): v for k, v in rec.items()})
        print("wrote", out, "losses it0", rec["it0_losses"], "it1", rec["it1_losses"])
    finally:
        os.chdir(cwd)


if __name__ == "__main__":
    main()
