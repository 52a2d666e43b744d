"""The Dropout random stream (oracle/mt19937.py, checker of csrc/mt19937.hip) pinned against torch itself, and
the jump polynomials of floodgan/data/mt19937_jumps.npz against sequential generation.  CPU only."""
import os

import numpy as np
import pytest
import torch

from oracle import mt19937 as MT

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "flood-prediction-gan_amd", "floodgan", "data", "mt19937_jumps.npz")


@pytest.mark.parametrize("seed,pre,sizes,p", [(47, 0, [262144, 1], 0.5), (47, 5, [1000, 4096, 77], 0.5),
                                               (3, 623, [312, 311], 0.5), (11, 1, [9999], 0.3),
                                               (0, 624, [2048, 2048], 0.5)])
def test_restatement_equals_torch_bernoulli(seed, pre, sizes, p):
    """torch.empty(n).bernoulli_(p) calls in a row (the reference's F.dropout draws) equal the restatement, and
    the generator state after them equals the restatement's"""
    torch.manual_seed(seed)
    if pre:
        torch.randint(0, 2 ** 31, (pre,), dtype=torch.int64)     # move the stream to an odd position
    state = torch.get_rng_state()
    outs, after = MT.bernoulli_draw(state, sizes, p)
    ref = [torch.empty(n).bernoulli_(p).numpy() for n in sizes]
    assert all(np.array_equal(a, b) for a, b in zip(outs, ref))
    assert torch.equal(after, torch.get_rng_state())


def test_jump_table_equals_sequential_generation():
    """W[c * chunk + t] = XOR of W[i + t] over the set exponents of x^(c * chunk) mod phi (t = 1..624, and the top
    bit at t = 0) for the first two table entries, from a generator state mid-stream; phi has degree 19937"""
    z = np.load(TABLE, allow_pickle=False)
    chunk = int(z["chunk"])
    assert chunk % 624 == 0 and z["jumps"].shape[1] == 624
    phi = int.from_bytes(z["phi"].astype("<u4").tobytes(), "little")
    assert phi.bit_length() - 1 == 19937
    torch.manual_seed(2024)
    torch.rand(1000)
    words, _, _ = MT.parse_state(torch.get_rng_state())
    w = MT.extend(words, 2 * chunk + 625)
    for c in (1, 2):
        g = int.from_bytes(z["jumps"][c - 1].astype("<u4").tobytes(), "little")
        acc = np.zeros(625, dtype=np.uint32)
        i = 0
        while g:
            if g & 1:
                acc ^= w[i:i + 625]
            g >>= 1
            i += 1
        assert np.array_equal(acc[1:], w[c * chunk + 1:c * chunk + 625]), c
        assert acc[0] >> 31 == w[c * chunk] >> 31, c
