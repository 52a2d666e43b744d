"""Tile data path: split selection, TIFF decode, async H2D staging and the
device-side transform of the reference's dataset (models/data.py:11-146, models/utils.py:19-67).

  determine_flood_dataset   models/data.py:83-146 (metadata/dataset_split.csv -> file lists)
  read_tile                 tifffile.imread (models/data.py:64-68): libfloodgan's host TIFF decoder
  FloodDataset              models/data.py:46-81: (input [C,R,R], target [3,R,R], name) per item
  TileLoader                the DataLoader of models/data.py:28-42 (the index order of a real DataLoader,
                            so the order under torch.manual_seed(epoch) is the reference's), but
                            batches come out on the device: decode into a pinned-host ring, H2D on
                            a copy stream, then one HIP transform per batch (fg_tile_transform:
                            np.fliplr, topography channels, bicubic antialias Resize, quadrant
                            crop, Normalize(0.5, 0.5)) writing channels-last tensors
  create_flood_dataset      models/data.py:11-44

There is no CPU transform path: the loader needs a HIP device, like the rest of floodgan.
"""
import concurrent.futures as cf
import ctypes as C
import math
import os
import queue
import struct
import threading

import numpy as np
import torch
from torch.utils.data import DataLoader

from . import _lib as L

# models/utils.py:30-39 and :58 -- the input-stack channels each topography keeps
TOPOGRAPHY_SOURCE_CHANNELS = {"all": list(range(9)), "dem": [0, 1, 2, 3], "flow": [0, 1, 2, 4],
                              "river": [0, 1, 2, 5], "map": [0, 1, 2, 6, 7, 8], None: [0, 1, 2]}
LOCATIONS = ["usa", "india"]
DISASTERS = ["hurricane-harvey", "hurricane-florence", "midwest-flooding", "nepal-flooding"]


# ------------------------------------------------------------------------------------------ splits

def determine_flood_dataset(subset, dem, crop=None, csv_path="metadata/dataset_split.csv"):
    """models/data.py:83-146: {"train"|"validation"|"test": [(file_name, version[, crop_index]), ...]}
    from the split table (the reference reads metadata/dataset_split.csv relative to the working
    directory; csv_path defaults to the same)."""
    import pandas as pd
    split = pd.read_csv(csv_path)
    s = subset.lower()
    if s in LOCATIONS:
        ds = split[split["country"] == s].copy()
    elif s in DISASTERS:
        ds = split[split["disaster"] == s].copy()
    elif s in ("harveyflorence", "harveyonflorence"):
        ds = _cross_disaster(split, s)
    elif s == "testing":
        ds = split[split["disaster"] == "hurricane-harvey"].copy()
        ds = ds[ds["version"] == "original"]
        ds = ds.sample(n=50, random_state=47)
    elif s == "all":
        ds = split.copy()
    else:
        raise NotImplementedError("Unrecognised dataset subset name")
    if dem not in ("best", "same"):
        raise NotImplementedError("Unrecognised DEM name - provide 'best' or 'same'")
    ds["file_name"] = ds["image"] + "_" + ds[f"{dem}_DEM"] + ".tif"
    ds = ds.sample(frac=1, random_state=47)
    names = ("train", "validation", "test")
    if crop:
        parts = []
        for i in range(crop):
            part = ds.copy()
            part["crop"] = i
            parts.append(part)
        ds = pd.concat(parts)
        out = {n: list(zip(ds[ds["split"] == n]["file_name"], ds[ds["split"] == n]["version"],
                           ds[ds["split"] == n]["crop"])) for n in names}
    else:
        out = {n: list(zip(ds[ds["split"] == n]["file_name"], ds[ds["split"] == n]["version"])) for n in names}
    return out


def _cross_disaster(split, s):
    """the two cross-disaster subsets of models/data.py:95-116: train on one disaster set (plus the
    flipped copies of its test images), validate and test on the other"""
    import pandas as pd
    if s == "harveyflorence":
        ds = split[split["country"] == "usa"].copy()
        train = (ds["disaster"] == "hurricane-harvey") | (ds["disaster"] == "hurricane-florence")
        flipped = ds[train & (ds["split"] == "test")].copy()
        held_out = "midwest-flooding"
    else:
        ds = split[(split["disaster"] == "hurricane-harvey") | (split["disaster"] == "hurricane-florence")].copy()
        flipped = ds[(ds["disaster"] == "hurricane-harvey") & (ds["split"] == "test")].copy()
        held_out = "hurricane-florence"
    flipped["version"] = "flipped"
    ds = pd.concat([ds, flipped], axis=0)
    if s == "harveyflorence":
        ds.loc[(ds["disaster"] == "hurricane-harvey") | (ds["disaster"] == "hurricane-florence"), "split"] = "train"
    else:
        ds.loc[ds["disaster"] == "hurricane-harvey", "split"] = "train"
    ds.loc[ds["disaster"] == held_out, "split"] = "validation"
    test = ds[ds["disaster"] == held_out].copy()
    test["split"] = "test"
    ds = pd.concat([ds, test], axis=0).reset_index(drop=True)
    return ds.drop(ds[((ds["split"] == "test") | (ds["split"] == "validation")) & (ds["version"] == "flipped")].index)


# ------------------------------------------------------------------------------------------ decode

def tiff_probe(path):
    """(height, width, channels, sample code) of a TIFF (libfloodgan host decoder)"""
    h, w, c, code = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    L.check(L.load().fg_tiff_probe(os.fsencode(path), C.byref(h), C.byref(w), C.byref(c), C.byref(code)),
            "tiff_probe")
    return h.value, w.value, c.value, code.value


def read_tile(path, out=None):
    """tifffile.imread of a dataset tile as float32 HWC (numpy), decoded by libfloodgan into `out`
    (e.g. a view of a pinned staging slot) when given."""
    h, w, c, _ = tiff_probe(path)
    if out is None:
        out = np.empty((h, w, c), dtype=np.float32)
    if out.size < h * w * c or out.dtype != np.float32 or not out.flags["C_CONTIGUOUS"]:
        raise ValueError(f"read_tile: destination must be contiguous float32 with >= {h * w * c} elements")
    L.check(L.load().fg_tiff_read(os.fsencode(path), out.ctypes.data_as(C.c_void_p), out.size), "tiff_read")
    return out.reshape(-1)[:h * w * c].reshape(h, w, c)


_FMT = {np.dtype(np.uint8): (1, 8), np.dtype(np.uint16): (1, 16), np.dtype(np.float32): (3, 32),
        np.dtype(np.float64): (3, 64)}


def write_tile(path, arr, big_endian=False, rows_per_strip=None):
    """tifffile.imsave(path, arr, planarconfig="contig") for a dataset tile (pre_processing/
    data_pre_processing.py:377-418): one IFD, uncompressed chunky strips; arr HWC (or HW) numpy
    uint8 / uint16 / float32 / float64.  Either byte order, any strip height."""
    a = np.asarray(arr)
    if a.ndim == 2:
        a = a[:, :, None]
    h, w, spp = a.shape
    fmt, bps = _FMT[a.dtype]
    e = ">" if big_endian else "<"
    data = a.astype(a.dtype.newbyteorder(e)).tobytes()
    rps = rows_per_strip or h
    row_bytes = w * spp * bps // 8
    strips = [data[i * rps * row_bytes:(i + 1) * rps * row_bytes] for i in range((h + rps - 1) // rps)]
    out = bytearray(b"MM\x00\x2a" if big_endian else b"II\x2a\x00")
    out += struct.pack(e + "I", 0)                      # IFD offset, patched below
    offsets = []
    for s in strips:
        offsets.append(len(out))
        out += s
    extra = bytearray()                                  # out-of-line arrays, after the IFD
    entries = []

    def entry(tag, typ, values):
        size = {3: 2, 4: 4}[typ]
        entries.append((tag, typ, values, size))
    entry(256, 4, [w])
    entry(257, 4, [h])
    entry(258, 3, [bps] * spp)
    entry(259, 3, [1])
    entry(262, 3, [2 if spp == 3 and fmt == 1 else 1])
    entry(273, 4, offsets)
    entry(277, 3, [spp])
    entry(278, 4, [rps])
    entry(279, 4, [len(s) for s in strips])
    entry(284, 3, [1])
    entry(339, 3, [fmt] * spp)
    ifd = len(out) + (len(out) & 1)
    out += b"\x00" * (ifd - len(out))
    struct.pack_into(e + "I", out, 4, ifd)
    n = len(entries)
    extra_base = ifd + 2 + 12 * n + 4
    body = bytearray(struct.pack(e + "H", n))
    for tag, typ, values, size in entries:
        body += struct.pack(e + "HHI", tag, typ, len(values))
        packed = b"".join(struct.pack(e + ("H" if size == 2 else "I"), v) for v in values)
        if len(packed) <= 4:
            body += packed + b"\x00" * (4 - len(packed))
        else:
            body += struct.pack(e + "I", extra_base + len(extra))
            extra += packed
    body += struct.pack(e + "I", 0)
    out += body + extra
    with open(path, "wb") as f:
        f.write(bytes(out))


# ------------------------------------------------------------------------------------------ resize

def aa_bicubic_taps(n_in, n_out):
    """Separable taps of torch.nn.functional.interpolate(mode="bicubic", antialias=True,
    align_corners=False) -- what torchvision's tensor Resize(antialias=True, BICUBIC) runs: Keys cubic
    with a = -0.5, support 2*scale when downscaling (scale = n_in / n_out), per-output weights
    normalized to sum 1.  Returns (first source index [n_out] int32, weights [n_out, taps] float32)."""
    scale = n_in / n_out
    support = 2.0 * scale if scale >= 1.0 else 2.0
    invscale = 1.0 / scale if scale >= 1.0 else 1.0

    def cubic(x):
        a = -0.5
        x = abs(x)
        if x < 1.0:
            return ((a + 2.0) * x - (a + 3.0)) * x * x + 1.0
        if x < 2.0:
            return (((x - 5.0) * x + 8.0) * x - 4.0) * a
        return 0.0
    taps = int(math.ceil(support)) * 2 + 1
    idx = np.zeros(n_out, dtype=np.int32)
    wts = np.zeros((n_out, taps), dtype=np.float64)
    for i in range(n_out):
        center = scale * (i + 0.5)
        xmin = max(int(center - support + 0.5), 0)
        xsize = min(int(center + support + 0.5), n_in) - xmin
        w = np.array([cubic((j + xmin - center + 0.5) * invscale) for j in range(xsize)])
        tot = w.sum()
        if tot != 0.0:
            w = w / tot
        idx[i] = xmin
        wts[i, :xsize] = w
    return idx, wts.astype(np.float32)


def resized_size(h, w, size):
    """torchvision Resize(int) output size: the shorter edge becomes `size`, aspect kept"""
    if size is None:
        return h, w
    if h <= w:
        return size, int(size * w / h)
    return int(size * h / w), size


def crop_window(rows, cols, crop, crop_index):
    """models/utils.py:45-56: (row0, col0, rows, cols) of quadrant crop_index of a rows x cols image"""
    if not crop:
        return 0, 0, rows, cols
    nd = int(np.sqrt(crop))
    rs, cs = rows // nd, cols // nd
    return (crop_index // nd) * rs, (crop_index % nd) * cs, rs, cs


class _Tables:
    """device tap tables per (n_in, n_out), cached"""

    def __init__(self):
        self.cache = {}

    def get(self, n_in, n_out, device):
        key = (n_in, n_out, str(device))
        if key not in self.cache:
            idx, w = aa_bicubic_taps(n_in, n_out)
            self.cache[key] = (torch.from_numpy(idx).to(device), torch.from_numpy(w).to(device), w.shape[1],
                               idx, w)
        return self.cache[key]


_TABLES = _Tables()


def transform_batch(raw, flips, crops, chan, resize, crop, out, tmp=None):
    """fg_tile_transform over a batch of raw HWC tiles already on the device.
    raw [n, h, w, c_src] fp32 (contiguous), flips [n] int (device), crops: per-tile crop indices (host
    list) or None; chan: source channel per output channel; out [n, len(chan), oh, ow] (any strides)."""
    L.require_device(raw, "raw tiles")
    n, h, w, c_src = raw.shape
    rh, rw = resized_size(h, w, resize)
    dev = raw.device
    xi, xw, xt, _, _ = _TABLES.get(w, rw, dev)
    yi, yw, yt, yi_h, _ = _TABLES.get(h, rh, dev)
    wins = [crop_window(rh, rw, crop, ci) for ci in (crops if crop else [0] * n)]
    oh, ow = wins[0][2], wins[0][3]
    assert tuple(out.shape) == (n, len(chan), oh, ow), (tuple(out.shape), (n, len(chan), oh, ow))
    # source rows each window's row taps reach; one common count so the workspace is regular
    lo = [int(yi_h[r0]) for r0, _, _, _ in wins]
    hi = [min(h, int(yi_h[r0 + oh - 1]) + yt) for r0, _, _, _ in wins]
    rows = min(h, max(b - a for a, b in zip(lo, hi)))
    lo = [min(a, h - rows) for a in lo]
    b = L.fg_tile_batch()
    b.src, b.tile_stride = raw.data_ptr(), h * w * c_src
    b.n, b.h_in, b.w_in, b.c_src = n, h, w, c_src
    b.flip = flips.data_ptr() if flips is not None else None
    b.c_out = len(chan)
    for o, c in enumerate(chan):
        b.chan[o] = c
    meta = torch.tensor([v for r0, c0, _, _ in wins for v in (r0, c0)] + lo, dtype=torch.int32).to(dev)
    b.crop, b.row_lo = meta.data_ptr(), meta.data_ptr() + 4 * 2 * n
    b.rows, b.out_h, b.out_w = rows, oh, ow
    b.x_idx0, b.x_w, b.x_taps = xi.data_ptr(), xw.data_ptr(), xt
    b.y_idx0, b.y_w, b.y_taps = yi.data_ptr(), yw.data_ptr(), yt
    need = n * rows * ow * len(chan)
    if tmp is None or tmp.numel() < need:
        tmp = torch.empty(need, dtype=torch.float32, device=dev)
    b.tmp = tmp.data_ptr()
    sn, sc, sy, sx = out.stride()
    b.dst = L.fg_wview(out.data_ptr(), sn, sc, sy, sx)
    L.check(L.load().fg_tile_transform(C.byref(b), L.stream_handle()), "tile_transform")
    return out, (meta, tmp)          # keep-alive of the per-call device buffers until the stream passes


# ------------------------------------------------------------------------------------------ dataset

class FloodDataset:
    """models/data.py:46-81 over libfloodgan's decoder and transform.  Items are
    (input [C,R,R], target [3,R,R], name) device tensors; `raw(index)` gives the decoded host arrays
    (what the staged loader batches)."""

    def __init__(self, dataset_subset, dataset_dem, split, path, topography, resize, crop,
                 csv_path="metadata/dataset_split.csv", files=None, device="cuda"):
        self.data_files = files if files is not None else \
            determine_flood_dataset(dataset_subset, dataset_dem, crop, csv_path)[split]
        self.resize, self.path, self.crop, self.topography = resize, path, crop, topography
        self.chan = TOPOGRAPHY_SOURCE_CHANNELS[topography]
        self.device = torch.device(device)

    def __len__(self):
        return len(self.data_files)

    def item(self, index):
        """(input path, output path, flipped, crop index, name) of item `index` (models/data.py:58-62)"""
        f = self.data_files[index]
        image_path, version = f[0], f[1]
        name = image_path[:-8]
        crop_index = f[2] if self.crop else 0
        return (os.path.join(self.path, "dataset_input", image_path), os.path.join(self.path, "dataset_output",
                                                                                     name + ".tif"),
                version == "flipped", crop_index, f"{name}_{crop_index}" if self.crop else name)

    def __getitem__(self, index):
        inp, outp, flip, ci, name = self.item(index)
        x, y = read_tile(inp), read_tile(outp)
        loader = TileLoader(self, batch_size=1, shuffle=False, device=self.device, prefetch=1, workers=1)
        xs, ys = loader._transform(torch.from_numpy(x)[None].to(self.device), torch.from_numpy(y)[None].to(self.device),
                                   [flip], [ci])
        return xs[0], ys[0], name


class _Slot:
    def __init__(self, n, h, w, cx, cy, device):
        self.hx = torch.empty((n, h, w, cx), dtype=torch.float32, pin_memory=True)
        self.hy = torch.empty((n, h, w, cy), dtype=torch.float32, pin_memory=True)
        self.dx = torch.empty((n, h, w, cx), dtype=torch.float32, device=device)
        self.dy = torch.empty((n, h, w, cy), dtype=torch.float32, device=device)
        self.h2d = torch.cuda.Event()          # host slot free again once this has passed
        self.consumed = torch.cuda.Event()     # device slot free again once this has passed
        self.h2d.record()
        self.consumed.record()


class TileLoader:
    """The reference's DataLoader (models/data.py:28-42: batch_size, shuffle=True, pin_memory=True) as an
    MI355X pipeline: a producer thread decodes each batch's tiles (libfloodgan, GIL released, `workers`
    threads) into a pinned-host ring slot and issues its H2D on a dedicated copy stream; the consumer's
    stream waits for that copy and runs the transform, so decode + PCIe of batch i+1 overlap the
    training step on batch i.  Yields (input [B,C,R,R], target [B,3,R,R], names), channels-last.

    Order: that of torch.utils.data.DataLoader(shuffle=True) over the item indices (the same draws from
    the global torch RNG when the iteration starts as the reference's loader).  Data parallelism: each global batch of
    batch_size * world items is split in rank order (every rank gets batch_size items; the last, short
    global batch is dropped when world > 1 so the shards stay equal)."""

    def __init__(self, dataset, batch_size=1, shuffle=True, device="cuda", prefetch=2, workers=4, rank=0, world=1,
                 drop_last=False):
        self.ds, self.bs, self.shuffle = dataset, batch_size, shuffle
        self.device = torch.device(device)
        self.prefetch, self.workers = max(1, prefetch), max(1, workers)
        self.rank, self.world = rank, world
        self.drop_last = drop_last or world > 1
        self._slots = None
        self._copy = None
        self._keep = []

    def __len__(self):
        n = len(self.ds) // (self.bs * self.world)
        if not self.drop_last and len(self.ds) % (self.bs * self.world):
            n += 1
        return n

    def _batches(self):
        # the index order of an actual DataLoader(shuffle=True) over the items: its iterator draws the
        # base seed from the global generator BEFORE RandomSampler draws its own, so a bare RandomSampler
        # would visit the items in another order than the reference's loader (models/data.py:28-42)
        order = DataLoader(range(len(self.ds)), batch_size=self.bs * self.world, shuffle=self.shuffle,
                           drop_last=self.drop_last, collate_fn=list)
        for b in order:
            shard = b[self.rank * self.bs:(self.rank + 1) * self.bs] if self.world > 1 else b
            if shard:
                yield shard

    def _ensure(self, first_index):
        if self._slots is not None:
            return
        inp, outp, _, _, _ = self.ds.item(first_index)
        h, w, cx, _ = tiff_probe(inp)
        hy, wy, cy, _ = tiff_probe(outp)
        if (hy, wy) != (h, w):
            raise RuntimeError(f"input {h}x{w} and target {hy}x{wy} tiles differ in size")
        self.geom = (h, w, cx, cy)
        self._slots = [_Slot(self.bs, h, w, cx, cy, self.device) for _ in range(self.prefetch + 1)]
        self._copy = torch.cuda.Stream(device=self.device)

    def _decode(self, pool, slot, items):
        h, w, cx, cy = self.geom

        def one(k):
            inp, outp, _, _, _ = items[k]
            if tiff_probe(inp)[:3] != (h, w, cx) or tiff_probe(outp)[:3] != (h, w, cy):
                raise RuntimeError(f"tile {inp} does not match the batch geometry {h}x{w}")
            read_tile(inp, slot.hx[k].numpy())
            read_tile(outp, slot.hy[k].numpy())
        list(pool.map(one, range(len(items))))

    def _transform(self, dx, dy, flips, crops):
        n = dx.shape[0]
        h, w = dx.shape[1], dx.shape[2]
        rh, rw = resized_size(h, w, self.ds.resize)
        _, _, oh, ow = crop_window(rh, rw, self.ds.crop, 0)
        f = torch.tensor([int(v) for v in flips], dtype=torch.int32).to(self.device, non_blocking=True)
        xo = torch.empty((n, len(self.ds.chan), oh, ow), dtype=torch.float32, device=self.device,
                         memory_format=torch.channels_last)
        yo = torch.empty((n, 3, oh, ow), dtype=torch.float32, device=self.device, memory_format=torch.channels_last)
        _, k1 = transform_batch(dx, f, crops, self.ds.chan, self.ds.resize, self.ds.crop, xo)
        _, k2 = transform_batch(dy, f, crops, [0, 1, 2], self.ds.resize, self.ds.crop, yo)
        self._keep = [f, k1, k2]
        return xo, yo

    def __iter__(self):
        batches = list(self._batches())
        if not batches:
            return
        self._ensure(batches[0][0])
        ready = queue.Queue(maxsize=self.prefetch)
        free = queue.Queue()
        for s in self._slots:
            free.put(s)
        stop = threading.Event()

        def produce():
            try:
                with cf.ThreadPoolExecutor(self.workers) as pool:
                    for b in batches:
                        if stop.is_set():
                            break
                        slot = free.get()
                        items = [self.ds.item(i) for i in b]
                        slot.h2d.synchronize()                 # its previous H2D has left the host slot
                        self._decode(pool, slot, items)
                        with torch.cuda.stream(self._copy):
                            self._copy.wait_event(slot.consumed)       # the device slot was transformed
                            n = len(items)
                            slot.dx[:n].copy_(slot.hx[:n], non_blocking=True)
                            slot.dy[:n].copy_(slot.hy[:n], non_blocking=True)
                            slot.h2d.record(self._copy)
                        ready.put((slot, items))
            except BaseException as e:      # surfaced on the consumer side
                ready.put(e)
            ready.put(None)

        th = threading.Thread(target=produce, daemon=True)
        th.start()
        try:
            while True:
                got = ready.get()
                if got is None:
                    break
                if isinstance(got, BaseException):
                    raise got
                slot, items = got
                cur = torch.cuda.current_stream(self.device)
                cur.wait_event(slot.h2d)
                n = len(items)
                xo, yo = self._transform(slot.dx[:n], slot.dy[:n], [it[2] for it in items], [it[3] for it in items])
                slot.consumed.record(cur)
                free.put(slot)
                yield xo, yo, [it[4] for it in items]
        finally:
            stop.set()
            while th.is_alive():
                try:
                    free.put(self._slots[0], timeout=0.01)
                    ready.get(timeout=0.01)
                except (queue.Empty, queue.Full):
                    pass
            th.join()


def create_flood_dataset(dataset_subset, dataset_dem, path, topography, resize=None, crop=None, batch_size=1,
                         num_workers=0, csv_path="metadata/dataset_split.csv", device="cuda", rank=0, world=1,
                         prefetch=2):
    """models/data.py:11-44: (train, validation, test) loaders, each shuffled."""
    splits = determine_flood_dataset(dataset_subset, dataset_dem, crop, csv_path)
    out = []
    for name in ("train", "validation", "test"):
        ds = FloodDataset(dataset_subset, dataset_dem, name, path, topography, resize, crop, files=splits[name],
                          device=device)
        out.append(TileLoader(ds, batch_size=batch_size, shuffle=True, device=device, prefetch=prefetch,
                              workers=max(1, num_workers) if num_workers else 4, rank=rank, world=world))
    return tuple(out)
