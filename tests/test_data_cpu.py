"""Host side of the tile data path on the CPU: split selection vs the
reference's own determine_flood_dataset (golden lists from tests/golden/make_golden_data.py),
libfloodgan's TIFF decoder vs known arrays (this repo's tifffile-layout writer and PIL), and the
antialias bicubic tap tables vs torch.nn.functional.interpolate (the op torchvision's tensor
Resize(antialias=True) dispatches to, models/utils.py:41-43).  TIFF decode parity against the
reference's tifffile is unpinned (tifffile is not installed; the reference ships no tiles)."""
import gzip
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from tiff_util import write_tiff

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def splits():
    with gzip.open(os.path.join(GOLDEN, "dataset_splits.json.gz"), "rt") as f:
        return json.load(f)


def test_split_selection_matches_reference(splits):
    from floodgan.data import determine_flood_dataset
    csv = os.path.join(GOLDEN, "dataset_split.csv")
    for key, ref in splits.items():
        subset, dem, crop = key.split("|")
        got = determine_flood_dataset(subset, dem, None if crop == "None" else int(crop), csv_path=csv)
        for part in ("train", "validation", "test"):
            assert [list(t) for t in got[part]] == ref[part], (key, part)
    with pytest.raises(NotImplementedError):
        determine_flood_dataset("mars", "best", csv_path=csv)
    with pytest.raises(NotImplementedError):
        determine_flood_dataset("usa", "worst", csv_path=csv)


@pytest.mark.parametrize("dtype,big,rps,shape", [(np.float32, False, None, (37, 23, 9)), (np.float32, True, 5, (16, 20, 9)),
                                                 (np.float64, False, 7, (9, 11, 3)), (np.uint8, False, None, (10, 12, 3)),
                                                 (np.uint16, True, 3, (8, 5, 1))])
def test_tiff_decoder_roundtrip(tmp_path, dtype, big, rps, shape):
    from floodgan.data import read_tile, tiff_probe
    rng = np.random.default_rng(1)
    a = (rng.random(shape) * (200 if dtype in (np.uint8, np.uint16) else 1)).astype(dtype)
    p = str(tmp_path / "t.tif")
    write_tiff(p, a, big_endian=big, rows_per_strip=rps)
    h, w, c, _ = tiff_probe(p)
    assert (h, w, c) == shape
    got = read_tile(p)
    assert got.dtype == np.float32 and got.shape == shape
    assert np.array_equal(got, a.astype(np.float32))


def test_tiff_decoder_reads_pil_files(tmp_path):
    """an independent writer: PIL's TIFF encoder (single-band float32 and RGB uint8)"""
    from PIL import Image
    from floodgan.data import read_tile
    rng = np.random.default_rng(2)
    f = rng.random((19, 13)).astype(np.float32)
    Image.fromarray(f, mode="F").save(tmp_path / "f.tif")
    assert np.array_equal(read_tile(str(tmp_path / "f.tif"))[..., 0], f)
    rgb = (rng.random((11, 17, 3)) * 255).astype(np.uint8)
    Image.fromarray(rgb, mode="RGB").save(tmp_path / "rgb.tif")
    assert np.array_equal(read_tile(str(tmp_path / "rgb.tif")), rgb.astype(np.float32))


def test_tiff_decoder_rejects_what_it_cannot_read(tmp_path):
    from PIL import Image
    from floodgan.data import read_tile
    rgb = (np.random.default_rng(3).random((8, 8, 3)) * 255).astype(np.uint8)
    Image.fromarray(rgb, mode="RGB").save(tmp_path / "lzw.tif", compression="tiff_lzw")
    with pytest.raises(RuntimeError, match="compression"):
        read_tile(str(tmp_path / "lzw.tif"))
    (tmp_path / "junk.tif").write_bytes(b"not a tiff at all")
    with pytest.raises(RuntimeError):
        read_tile(str(tmp_path / "junk.tif"))


def _emulate(x, n_out_h, n_out_w):
    """the engine's two separable passes (width, then height) over the tap tables, in float64"""
    from floodgan.data import aa_bicubic_taps
    c, h, w = x.shape
    xi, xw = aa_bicubic_taps(w, n_out_w)
    yi, yw = aa_bicubic_taps(h, n_out_h)
    t = np.zeros((c, h, n_out_w))
    for j in range(n_out_w):
        for k in range(xw.shape[1]):
            if xw[j, k] != 0:
                t[:, :, j] += xw[j, k] * x[:, :, xi[j] + k]
    out = np.zeros((c, n_out_h, n_out_w))
    for i in range(n_out_h):
        for k in range(yw.shape[1]):
            if yw[i, k] != 0:
                out[:, i, :] += yw[i, k] * t[:, yi[i] + k, :]
    return out


@pytest.mark.parametrize("n_in,n_out", [(64, 32), (64, 16), (48, 40), (30, 51), (40, 40), (1024, 512)])
def test_antialias_bicubic_taps_match_torch(n_in, n_out):
    torch.manual_seed(n_in + n_out)
    x = torch.rand(3, n_in, n_in, dtype=torch.float64)
    ref = F.interpolate(x[None], size=(n_out, n_out), mode="bicubic", antialias=True, align_corners=False)[0]
    if n_in > 256:     # keep the pure-numpy emulation cheap: a width-only resize, a few output columns
        from floodgan.data import aa_bicubic_taps
        xi, xw = aa_bicubic_taps(n_in, n_out)
        wide = F.interpolate(x[None], size=(n_in, n_out), mode="bicubic", antialias=True)[0]
        for j in (0, 1, 255, 511):
            col = sum(xw[j, k] * x[:, :, xi[j] + k] for k in range(xw.shape[1]) if xw[j, k] != 0)
            assert float((col - wide[:, :, j]).abs().max()) < 1e-6
        return
    got = torch.from_numpy(_emulate(x.numpy(), n_out, n_out))
    assert float((got - ref).abs().max()) < 1e-6, float((got - ref).abs().max())


def test_crop_window_and_resize_size():
    from floodgan.data import crop_window, resized_size
    assert resized_size(1024, 1024, 512) == (512, 512)
    assert resized_size(1024, 2048, 256) == (256, 512) and resized_size(300, 200, 100) == (150, 100)
    assert resized_size(64, 64, None) == (64, 64)
    # models/utils.py:45-56: crop=4 -> quadrants in row-major order
    assert [crop_window(512, 512, 4, i) for i in range(4)] == [(0, 0, 256, 256), (0, 256, 256, 256),
                                                              (256, 0, 256, 256), (256, 256, 256, 256)]
    assert crop_window(512, 512, None, 0) == (0, 0, 512, 512)


class _Items:
    """a dataset stand-in: only its length matters to the loader's index order"""

    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


@pytest.mark.parametrize("n,bs,world", [(20, 1, 1), (20, 3, 1), (23, 2, 2), (7, 4, 1)])
def test_tile_loader_order_is_the_reference_dataloaders(n, bs, world):
    """TileLoader's item order under torch.manual_seed(epoch) (models/model.py:609) is the order of the
    reference's DataLoader(batch_size=1, shuffle=True) (models/data.py:28-32): its iterator draws a base
    seed from the global generator before RandomSampler draws its own; DP ranks take consecutive slices
    of each global batch.  The global generator is left in the same state too."""
    import torch
    from torch.utils.data import DataLoader

    from floodgan.data import TileLoader
    ld = [TileLoader(_Items(n), batch_size=bs, device="cpu", rank=r, world=world) for r in range(world)]
    torch.manual_seed(5)
    flat = [int(i) for b in DataLoader(range(n), batch_size=1, shuffle=True) for i in b]
    after = torch.rand(1)
    g = bs * world
    for r in range(world):
        torch.manual_seed(5)
        got = list(ld[r]._batches())
        assert torch.equal(torch.rand(1), after)
        glob = [flat[i:i + g] for i in range(0, n, g)]
        if world > 1:
            glob = [b for b in glob if len(b) == g]
        assert got == [b[r * bs:(r + 1) * bs] for b in glob]


def test_model_builds_loaders_from_data_path(tmp_path, monkeypatch):
    """Model(**train.py's args) builds its three loaders from data_path (models/model.py:150-156): the split
    table read relative to the working directory, the batch size, the topography channels, the crop
    suffixes, and under DP the shard of this rank (here world 1).  Construction only (no compute)."""
    import numpy as np

    from floodgan.model import Model
    from tiff_util import write_tiff
    root = tmp_path
    for d in ("dataset_input", "dataset_output", "metadata"):
        (root / d).mkdir()
    rows = ["image,best_DEM,same_DEM,version,split,disaster,country"]
    for i, split in enumerate(["train"] * 5 + ["validation"] * 2 + ["test"]):
        name = f"hurricane-harvey_{i:08d}"
        write_tiff(str(root / "dataset_input" / f"{name}_10m.tif"), np.zeros((16, 16, 9), np.float32))
        write_tiff(str(root / "dataset_output" / f"{name}.tif"), np.zeros((16, 16, 3), np.float32))
        rows.append(f"{name},10m,10m,original,{split},hurricane-harvey,usa")
    (root / "metadata" / "dataset_split.csv").write_text("\n".join(rows) + "\n")
    monkeypatch.chdir(root)
    m = Model(model="pairedattention", dataset_subset="hurricane-harvey", dataset_dem="same", data_path=str(root),
              num_epochs=1, topography="map", resize=None, crop=4, device="cpu", batch_size=3)
    assert (len(m.train_loader.ds), len(m.val_loader.ds), len(m.test_loader.ds)) == (20, 8, 4)   # x4 crops
    assert m.train_loader.bs == 3 and len(m.train_loader) == 7
    assert m.train_loader.ds.item(0)[4].endswith(("_0", "_1", "_2", "_3"))
    assert m.train_loader.ds.chan == [0, 1, 2, 6, 7, 8]
    # explicit loaders still take precedence (the bench / tests feed resident batches)
    m2 = Model(model="pairedattention", data_path=str(root), device="cpu", train_loader=[1])
    assert m2.train_loader == [1] and m2.val_loader is None
