"""Tile data path on the GPU: libfloodgan's batch transform and the staged
TileLoader against the reference's per-item pipeline restated with torch CPU ops -- np.fliplr of the
decoded HWC tile (models/data.py:63-65), topography channel selection, torchvision Resize(resize,
BICUBIC, antialias=True) = F.interpolate(mode="bicubic", antialias=True) on the CHW tensor, quadrant
crop and Normalize(0.5, 0.5) (models/utils.py:30-61).  Tolerance 1e-5 (max abs, values in [-1, 1])."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from tiff_util import write_tiff

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-5


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def reference_item(x_hwc, y_hwc, flip, topography, resize, crop, crop_index):
    from floodgan.data import TOPOGRAPHY_SOURCE_CHANNELS, crop_window
    if flip:
        x_hwc, y_hwc = np.fliplr(x_hwc).copy(), np.fliplr(y_hwc).copy()
    x = torch.from_numpy(x_hwc.transpose(2, 0, 1).copy())[TOPOGRAPHY_SOURCE_CHANNELS[topography]]
    y = torch.from_numpy(y_hwc.transpose(2, 0, 1).copy())
    if resize:
        size = (resize, resize) if x.shape[1] == x.shape[2] else None
        x = F.interpolate(x[None], size=size, mode="bicubic", antialias=True, align_corners=False)[0]
        y = F.interpolate(y[None], size=size, mode="bicubic", antialias=True, align_corners=False)[0]
    r0, c0, rs, cs = crop_window(x.shape[1], x.shape[2], crop, crop_index)
    x, y = x[:, r0:r0 + rs, c0:c0 + cs], y[:, r0:r0 + rs, c0:c0 + cs]
    return (x - 0.5) / 0.5, (y - 0.5) / 0.5


@pytest.mark.parametrize("h,resize,crop", [(96, 64, 4), (40, 64, None), (64, None, 4), (128, 40, 4), (64, 64, None)])
def test_transform_batch_vs_reference(h, resize, crop):
    from floodgan.data import TOPOGRAPHY_SOURCE_CHANNELS, crop_window, resized_size, transform_batch
    rng = np.random.default_rng(h)
    n = 3
    xs = rng.random((n, h, h, 9)).astype(np.float32)
    ys = rng.random((n, h, h, 3)).astype(np.float32)
    flips, crops = [0, 1, 0], [0, 3, 1]
    rh, rw = resized_size(h, h, resize)
    _, _, oh, ow = crop_window(rh, rw, crop, 0)
    for topo in ("all", "map", None):
        chan = TOPOGRAPHY_SOURCE_CHANNELS[topo]
        xo = torch.empty((n, len(chan), oh, ow), device=DEV, memory_format=torch.channels_last)
        yo = torch.empty((n, 3, oh, ow), device=DEV)
        f = torch.tensor(flips, dtype=torch.int32, device=DEV)
        transform_batch(torch.from_numpy(xs).to(DEV), f, crops, chan, resize, crop, xo)
        transform_batch(torch.from_numpy(ys).to(DEV), f, crops, [0, 1, 2], resize, crop, yo)
        torch.cuda.synchronize()
        for k in range(n):
            rx, ry = reference_item(xs[k], ys[k], flips[k], topo, resize, crop, crops[k])
            assert float((xo[k].cpu() - rx).abs().max()) < TOL, (topo, k)
            assert float((yo[k].cpu() - ry).abs().max()) < TOL, (topo, k)


def _dataset_dir(root, n_img=7, h=64):
    """a synthetic dataset in the reference's layout: dataset_input/<image>_<DEM>.tif (9-ch float32),
    dataset_output/<image>.tif (3-ch float32), metadata/dataset_split.csv"""
    rng = np.random.default_rng(11)
    os.makedirs(os.path.join(root, "dataset_input"))
    os.makedirs(os.path.join(root, "dataset_output"))
    os.makedirs(os.path.join(root, "metadata"))
    rows = ["image,best_DEM,same_DEM,version,split,disaster,country"]
    arrays = {}
    for i in range(n_img):
        name = f"hurricane-harvey_{i:08d}"
        x = rng.random((h, h, 9)).astype(np.float32)
        y = rng.random((h, h, 3)).astype(np.float32)
        write_tiff(os.path.join(root, "dataset_input", f"{name}_10m.tif"), x, rows_per_strip=16)
        write_tiff(os.path.join(root, "dataset_output", f"{name}.tif"), y)
        arrays[name] = (x, y)
        rows.append(f"{name},10m,10m,original,train,hurricane-harvey,usa")
        if i % 3 == 0:
            rows.append(f"{name},10m,10m,flipped,train,hurricane-harvey,usa")
    with open(os.path.join(root, "metadata", "dataset_split.csv"), "w") as f:
        f.write("\n".join(rows) + "\n")
    return arrays


@pytest.mark.parametrize("crop,resize,topo", [(4, 48, "map"), (None, None, "all")])
def test_tile_loader_vs_reference_items(tmp_path, crop, resize, topo):
    """The staged loader: the item order of DataLoader(shuffle=True) under the same global seed, every
    batch equal to the reference's per-item pipeline, names with the crop suffix (models/utils.py:56),
    and data-parallel sharding of each global batch (rank order)."""
    from floodgan.data import create_flood_dataset
    from torch.utils.data import DataLoader
    root = str(tmp_path)
    arrays = _dataset_dir(root)
    csv = os.path.join(root, "metadata", "dataset_split.csv")
    train, _, _ = create_flood_dataset("hurricane-harvey", "same", root, topo, resize=resize, crop=crop, batch_size=3,
                                       csv_path=csv, prefetch=2)
    ds = train.ds
    torch.manual_seed(5)
    # the reference's own loader form (models/data.py:28-32: batch_size 1, shuffle=True) over the item indices
    order = [int(i) for b in DataLoader(range(len(ds)), batch_size=1, shuffle=True) for i in b]
    torch.manual_seed(5)
    seen = []
    for xb, yb, names in train:
        assert xb.is_contiguous(memory_format=torch.channels_last)
        for k, name in enumerate(names):
            idx = order[len(seen)]
            _, _, flip, ci, want = ds.item(idx)
            assert name == want
            x, y = arrays[want[:len("hurricane-harvey_00000000")]]
            rx, ry = reference_item(x, y, flip, topo, resize, crop, ci)
            assert float((xb[k].cpu() - rx).abs().max()) < TOL and float((yb[k].cpu() - ry).abs().max()) < TOL
            seen.append(idx)
    assert seen == order and len(seen) == len(ds)
    # two ranks: each global batch of 2 x 2 items is split in rank order, the short tail dropped
    shards = []
    for rank in range(2):
        tr, _, _ = create_flood_dataset("hurricane-harvey", "same", root, topo, resize=resize, crop=crop, batch_size=2,
                                        csv_path=csv, rank=rank, world=2)
        torch.manual_seed(9)
        shards.append([n for _, _, names in tr for n in names])
    torch.manual_seed(9)
    flat = [int(i) for b in DataLoader(range(len(ds)), batch_size=1, shuffle=True) for i in b]
    glob = [flat[i:i + 4] for i in range(0, len(flat) - 3, 4)]
    assert shards[0] == [ds.item(i)[4] for b in glob for i in b[:2]]
    assert shards[1] == [ds.item(i)[4] for b in glob for i in b[2:]]


def test_cycle_training_through_the_loader(tmp_path):
    """BASELINE configs[4]'s pipeline in miniature: AttentionGAN train_cycle fed by the staged loader
    with crop=4 (models/model.py:151-156 -> :660-758)."""
    from floodgan.data import create_flood_dataset
    from floodgan.model import Model
    root = str(tmp_path)
    _dataset_dir(root, n_img=3, h=64)
    train, _, _ = create_flood_dataset("hurricane-harvey", "same", root, "all", resize=64, crop=4, batch_size=4,
                                       csv_path=os.path.join(root, "metadata", "dataset_split.csv"))
    m = Model(model="AttentionGAN", num_epochs=1, topography="all", train_loader=train)
    m.train_cycle()
    vals = [v[-1] for v in m.all_losses.values()]
    assert len(vals) == 8 and all(np.isfinite(vals))


def test_model_builds_its_loaders_like_train_py(tmp_path, monkeypatch):
    """train.py's own call (models/model.py:150-156 via train.py:33-38): Model(**vars(args)) with the
    reference's argument set over a dataset on disk -- the Model builds its train / validation / test loaders
    from data_path (metadata/dataset_split.csv read relative to the working directory, as the reference
    does) and train_paired runs on them.  Its per-epoch losses equal the same batches (the same
    torch.manual_seed(epoch) order) fed to a fresh Model's fused step, and so do the trained weights."""
    import argparse

    from floodgan.model import Model
    root = str(tmp_path)
    _dataset_dir(root, n_img=5, h=64)
    monkeypatch.chdir(root)
    args = argparse.Namespace(model="pairedattention", dataset_subset="hurricane-harvey", dataset_dem="same",
                              data_path=root, num_epochs=2, topography="all", resize=32, crop=None,
                              save_model_interval=0, save_images_interval=0, verbose=False,
                              load_pretrained_model=False, pretrained_model_path=None, add_identity_loss=False,
                              seed=47)
    args.training_model = True
    m = Model(**vars(args), batch_size=2)
    assert len(m.train_loader) == 4 and m.val_loader is not None and m.test_loader is not None   # 7 items, bs 2
    m.train_paired()
    ref = Model(**vars(args), batch_size=2)
    keys = ["losses_discriminator_real", "losses_discriminator_synthetic", "losses_generator_synthetic",
            "l1_losses_generator_synthetic"]
    means = {k: [] for k in keys}
    for epoch in (1, 2):
        torch.manual_seed(epoch)                        # models/model.py:609
        per = {k: [] for k in keys}
        for xb, yb, names in ref.train_loader:
            assert xb.shape[1:] == (9, 32, 32) and yb.shape[1:] == (3, 32, 32)
            for k, v in zip(keys, ref.step_fn(xb, yb).cpu().tolist()):
                per[k].append(v)
        for k in keys:
            means[k].append(float(np.mean(per[k])))
        ref.scheduler_discriminator.step()
        ref.scheduler_generator.step()
    for k in keys:
        assert np.allclose(m.all_losses["all_" + k], means[k], rtol=1e-6, atol=0), (k, m.all_losses["all_" + k], means[k])
    for (k, a), (_, b) in zip(m.generator.named_parameters(), ref.generator.named_parameters()):
        assert torch.equal(a, b), k


def test_configs4_attentiongan_crop4_256_tiles_vs_reference(tmp_path, report):
    """BASELINE.json configs[4] at its tile shape: the reference's README recipe --resize=512 --crop=4
    (models/utils.py:41-56) gives 256x256 quadrant tiles; AttentionGAN's train_cycle (models/model.py:660-758)
    fed by the staged TileLoader at batch 8.  Every loader batch equals the reference's per-item pipeline
    (fliplr version, Resize(512, bicubic, antialias), quadrant, Normalize; 1e-5), and the eight iteration-0
    losses of the fused cycle step on the first batch (all evaluated before any update) equal the fp32
    oracle's on that same batch (1e-5, as test_cycle_p1_losses_512)."""
    import torch.nn.functional as F

    from floodgan.data import create_flood_dataset
    from floodgan.model import Model
    from oracle import attention_cycle as OC
    from oracle import paired_attention as O
    root = str(tmp_path)
    arrays = _dataset_dir(root, n_img=3, h=640)           # raw tiles larger than the resize (downscaling taps)
    train, _, _ = create_flood_dataset("hurricane-harvey", "same", root, "all", resize=512, crop=4, batch_size=8,
                                       csv_path=os.path.join(root, "metadata", "dataset_split.csv"))
    ds = train.ds
    assert len(ds) == 16 and len(train) == 2                # (3 + 1 flipped) x 4 quadrants
    from torch.utils.data import DataLoader
    torch.manual_seed(1)                                    # models/model.py:676
    order = [int(i) for b in DataLoader(range(len(ds)), batch_size=1, shuffle=True) for i in b]
    torch.manual_seed(1)
    batches = []
    for xb, yb, names in train:
        assert xb.shape == (8, 9, 256, 256) and yb.shape == (8, 3, 256, 256)
        batches.append((xb, yb, names))
    worst = 0.0
    for bi, (xb, yb, names) in enumerate(batches):
        for k, name in enumerate(names):
            _, _, flip, ci, want = ds.item(order[bi * 8 + k])     # the original and flipped versions share a name
            assert name == want
            x, y = arrays[name[:len("hurricane-harvey_00000000")]]
            rx, ry = reference_item(x, y, flip, "all", 512, 4, ci)
            worst = max(worst, float((xb[k].cpu() - rx).abs().max()), float((yb[k].cpu() - ry).abs().max()))
    assert worst < TOL, worst
    # iteration-0 losses of the cycle step on the first batch vs the fp32 oracle's forwards
    x, y = batches[0][0], batches[0][1]
    m = Model(model="AttentionGAN", num_epochs=2, topography="all")
    losses = m.cycle_step_fn(x, y).cpu().numpy().astype(np.float64)
    xc, yc = x.cpu().contiguous(), y.cpu().contiguous()
    P = OC.init_cycle_params(model="attentiongan")
    D = O.discriminator_forward
    cond = xc[:, 3:]
    with torch.no_grad():
        def gen(p, t):
            return O.generator_forward(p, t)[0]
        post_real = torch.cat((yc, cond), 1)
        sp = torch.cat((gen(P["pre_to_post"], xc), cond), 1)
        spre = torch.cat((gen(P["post_to_pre"], post_real), cond), 1)
        rp = gen(P["pre_to_post"], spre)
        rq = gen(P["post_to_pre"], sp)

        def mse(p, t):
            return float(F.mse_loss(p, torch.full_like(p, t)))
        ref = np.array([mse(D(P["post_d"], sp), 1), mse(D(P["pre_d"], spre), 1), 10 * float(F.l1_loss(rq, xc[:, :3])),
                        10 * float(F.l1_loss(rp, yc)), mse(D(P["pre_d"], xc), 1), mse(D(P["post_d"], post_real), 1),
                        mse(D(P["pre_d"], spre), 0), mse(D(P["post_d"], sp), 0)])
    lrel = np.abs(losses - ref) / np.abs(ref)
    report("configs4_attentiongan_crop4_256", loader_vs_reference_items=worst, loss_rel=lrel.tolist())
    assert lrel.max() < 1e-5, lrel
