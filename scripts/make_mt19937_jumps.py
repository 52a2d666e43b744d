"""Generate floodgan/data/mt19937_jumps.npz: the jump polynomials the device MT19937 (csrc/mt19937.hip) uses to
start its chunks of the stream in parallel.

MT19937's state transition is GF(2)-linear with an irreducible characteristic polynomial phi of degree 19937, so
every bit position of the word sequence W satisfies sum_i phi_i W[t + i] = 0.  With g = x^J mod phi,
W[J + t] = XOR over {i : g_i = 1} of W[i + t] (t = 0..623, and the top bit at t = 0): a chunk starting J words
after a known window is a fixed XOR-combination of the first 19937 + 624 words of the stream.

phi is found with Berlekamp-Massey over the top-bit sequence of a seeded stream (and checked on every bit
position of a second seed); the table holds g_c = x^(c * CHUNK) mod phi for c = 1..COUNT, CHUNK = 624 * 256
words.  Run: python scripts/make_mt19937_jumps.py (about a minute)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import mt19937 as MT  # noqa: E402

DEG = 19937
CHUNK = 624 * 256
COUNT = 128
OUT = os.path.join(ROOT, "flood-prediction-gan_amd", "floodgan", "data", "mt19937_jumps.npz")


def seeded(seed):
    """the 624 init words of std::mt19937(seed) (ATen's at::mt19937 initialisation)"""
    w = [seed & 0xFFFFFFFF]
    for i in range(1, 624):
        w.append((1812433253 * (w[-1] ^ (w[-1] >> 30)) + i) & 0xFFFFFFFF)
    return np.array(w, dtype=np.uint32)


def berlekamp_massey(bits):
    """connection polynomial C (bit i = c_i, c_0 = 1) and its length L: s[n] = sum_{i=1..L} c_i s[n-i]"""
    C, B, L, m = 1, 1, 0, 1
    R = 0                                     # bit i = s[n - i]
    for n, s in enumerate(bits):
        R = (R << 1) | s
        d = (C & R).bit_count() & 1
        if d == 0:
            m += 1
        elif 2 * L <= n:
            T = C
            C ^= B << m
            L, B, m = n + 1 - L, T, 1
        else:
            C ^= B << m
            m += 1
    return C, L


def polymod(r, phi):
    d = phi.bit_length() - 1
    while r.bit_length() - 1 >= d:
        r ^= phi << (r.bit_length() - 1 - d)
    return r


def mulmod(a, b, phi):
    r, i = 0, 0
    while b:
        if b & 1:
            r ^= a << i
        b >>= 1
        i += 1
    return polymod(r, phi)


def powmod_x(e, phi):
    r, base = 1, 2                           # polynomials as ints: 2 = x
    while e:
        if e & 1:
            r = mulmod(r, base, phi)
        base = mulmod(base, base, phi)
        e >>= 1
    return r


def to_words(poly):
    return np.array([(poly >> (32 * i)) & 0xFFFFFFFF for i in range(624)], dtype=np.uint32)


def apply_jump(w, g, t_count=624):
    acc = np.zeros(t_count, dtype=np.uint32)
    i = 0
    while g:
        if g & 1:
            acc ^= w[i:i + t_count]
        g >>= 1
        i += 1
    return acc


def main():
    w = MT.extend(seeded(5489), 2 * DEG + 2000)
    bits = [(int(v) >> 31) & 1 for v in w[1:2 * DEG + 1000]]
    C, L = berlekamp_massey(bits)
    assert L == DEG, L
    phi = 0                                   # reciprocal: phi_i = c_{L-i}
    for i in range(L + 1):
        if (C >> (L - i)) & 1:
            phi |= 1 << i
    # phi annihilates every bit position of another seed's stream
    w2 = MT.extend(seeded(20240), DEG + 4000)
    for t in (1, 7, 1000, 3000):
        assert not apply_jump(w2[t:], phi, 1).any() and not apply_jump(w2[t:], phi, 624)[1:].any()
    gs, g1 = [], powmod_x(CHUNK, phi)
    g = 1
    for c in range(1, COUNT + 1):
        g = mulmod(g, g1, phi)
        gs.append(to_words(g))
        if c <= 2:                            # check against sequential generation
            seq = MT.extend(seeded(99), c * CHUNK + 624)
            jumped = apply_jump(seq, g)
            assert np.array_equal(jumped[1:], seq[c * CHUNK + 1:c * CHUNK + 624]), c
            assert (jumped[0] >> 31) == (seq[c * CHUNK] >> 31), c
        print(f"jump {c}/{COUNT}", flush=True) if c % 16 == 0 else None
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez_compressed(OUT, phi=to_words(phi), jumps=np.stack(gs), chunk=np.array(CHUNK), deg=np.array(DEG))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
