"""A minimal baseline-TIFF writer for the tests (tifffile is not installed here): the layout
tifffile.imsave(..., planarconfig="contig") produces for the reference's dataset tiles
(pre_processing/data_pre_processing.py:377-418) -- one IFD, uncompressed chunky strips -- in either
byte order, with a configurable strip height, so libfloodgan's decoder can be checked against
known arrays."""
import struct

import numpy as np

_FMT = {np.dtype(np.uint8): (1, 8), np.dtype(np.uint16): (1, 16), np.dtype(np.float32): (3, 32),
        np.dtype(np.float64): (3, 64)}


def write_tiff(path, arr, big_endian=False, rows_per_strip=None):
    """arr: HWC (or HW) numpy array of uint8 / uint16 / float32 / float64"""
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
