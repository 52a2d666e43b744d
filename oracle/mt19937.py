"""CPU restatement of the random stream behind the reference's Dropout (test infrastructure: the checker of
csrc/mt19937.hip; nothing on the product path imports it).

The reference's Pix2Pix generator applies nn.Dropout(0.5) in training mode
(/root/reference/models/model_architectures.py:52); on the CPU, F.dropout draws
`torch.empty_like(x).bernoulli_(1 - p)`.  torch 2.10's CPU `bernoulli_(p)` on a float tensor is a serial walk
over the elements in memory order; each element takes `random64()` from the global CPUGeneratorImpl (two
consecutive mt19937 outputs r1, r2 -> (r1 << 32) | r2), maps its low 53 bits to u = x * 2^-53 and keeps
u < p.  At p = 0.5 that is bit 20 of r1 == 0.  The generator is the standard MT19937 (ATen's at::mt19937:
624-word state, twist(u, v) = ((u & 0x80000000 | v & 0x7fffffff) >> 1) ^ (v & 1 ? 0x9908b0df : 0), the
standard tempering).  `torch.get_rng_state()` serialises it as CPUGeneratorImplState: the initial seed (u64),
left (i32), seeded (i32), next (u64), state[624] (u64 each), then the normal-sampler caches.

Pinned against torch itself by tests/test_mt19937_cpu.py (masks and the generator state after the draw)."""
import struct

import numpy as np

N, M = 624, 397
MATRIX_A, UPPER, LOWER = 0x9908B0DF, 0x80000000, 0x7FFFFFFF


def parse_state(state_bytes):
    """(state words [624] uint32, left, next) of a torch.get_rng_state() byte tensor"""
    b = bytes(state_bytes.numpy().tobytes()) if hasattr(state_bytes, "numpy") else bytes(state_bytes)
    _, left, _, nxt = struct.unpack_from("<QiiQ", b, 0)
    words = np.frombuffer(b, dtype="<u8", count=N, offset=24).astype(np.uint32)
    return words, left, nxt


def pack_state(state_bytes, words, left, nxt):
    """a torch.get_rng_state() byte tensor with the mt19937 fields replaced (seed, caches kept)"""
    import torch
    b = bytearray(state_bytes.numpy().tobytes())
    struct.pack_into("<i", b, 8, left)
    struct.pack_into("<Q", b, 16, nxt)
    b[24:24 + 8 * N] = np.asarray(words, dtype=np.uint32).astype("<u8").tobytes()
    return torch.frombuffer(b, dtype=torch.uint8).clone()


def first_index(left):
    """W index of the next output when the state words are W[0..623]: 625 - left (left = 1: a twist is due)"""
    return 625 - left


def extend(words, count):
    """W[0 .. count) of the word sequence whose first 624 words are `words`: the MT recurrence
    W[k + 624] = W[k + 397] ^ twist(W[k], W[k + 1]), computed 227 words at a time (numpy)"""
    w = np.zeros(max(count, N), dtype=np.uint32)
    w[:N] = words
    k = N
    while k < count:
        n = min(N - M, count - k)
        a, b, c = w[k - N:k - N + n], w[k - N + 1:k - N + 1 + n], w[k - N + M:k - N + M + n]
        y = (a & np.uint32(UPPER)) | (b & np.uint32(LOWER))
        w[k:k + n] = c ^ (y >> np.uint32(1)) ^ np.where(b & np.uint32(1), np.uint32(MATRIX_A), np.uint32(0))
        k += n
    return w[:count]


def temper(y):
    y = np.asarray(y, dtype=np.uint32)
    y = y ^ (y >> np.uint32(11))
    y = y ^ ((y << np.uint32(7)) & np.uint32(0x9D2C5680))
    y = y ^ ((y << np.uint32(15)) & np.uint32(0xEFC60000))
    return y ^ (y >> np.uint32(18))


def bernoulli_draw(state_bytes, sizes, p=0.5):
    """float32 0/1 arrays of the given element counts, drawn in order exactly as consecutive
    `torch.empty(n).bernoulli_(p)` calls draw them, and the generator state after the draws"""
    words, left, _ = parse_state(state_bytes)
    q0 = first_index(left)
    total = 2 * sum(sizes)
    w = extend(words, q0 + total + N)
    y = temper(w[q0:q0 + total]).astype(np.uint64)
    x = ((y[0::2] << np.uint64(32)) | y[1::2]) & np.uint64((1 << 53) - 1)
    keep = (x.astype(np.float64) * 2.0 ** -53 < p).astype(np.float32)
    out, o = [], 0
    for n in sizes:
        out.append(keep[o:o + n])
        o += n
    last = q0 + total - 1
    blk = last // N
    after = pack_state(state_bytes, w[blk * N:(blk + 1) * N], N - last % N, last % N + 1) if total else state_bytes
    return out, after
