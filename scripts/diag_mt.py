"""Diagnostic (GPU): the device Bernoulli stream vs torch's CPU draws, per chunk range (outputs prefilled with -1)."""
import ctypes as C
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "flood-prediction-gan_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from floodgan import _lib as L, torch_rng as T  # noqa: E402

lib = L.load()
for n in (200000, 600000):
    torch.manual_seed(5)
    st = torch.get_rng_state()
    raw = st.numpy().tobytes()
    left = struct.unpack_from("<i", raw, 8)[0]
    first = 625 - left
    words = np.frombuffer(raw, dtype="<u8", count=624, offset=24).astype(np.uint32)
    chunk = T._table()["chunk"]
    last = first + 2 * n - 1
    nch = 1 if last <= chunk else (last - 1) // chunk + 1
    jumps = T._jumps("cuda", nch - 1)
    work = torch.zeros(int(lib.fg_bernoulli_mt_workspace_words(nch)), dtype=torch.int32, device="cuda")
    sd = torch.from_numpy(words.view(np.int32)).cuda()
    out = torch.full((n,), -1.0, device="cuda")
    final = torch.zeros(624, dtype=torch.int32, device="cuda")
    optr = (C.c_void_p * 1)(out.data_ptr())
    sz = (C.c_longlong * 1)(n)
    rc = lib.fg_bernoulli_mt(sd.data_ptr(), first, n, jumps.data_ptr(), jumps.shape[0], chunk, 1, optr, sz, 0.5,
                             final.data_ptr(), work.data_ptr(), L.stream_handle())
    torch.cuda.synchronize()
    print("rc", rc, L.load().fg_last_error(), "chunks", nch, "first", first, flush=True)
    ref = torch.empty(n).bernoulli_(0.5)
    o = out.cpu()
    for c in range(nch):
        lo = 0 if c == 0 else ((c * chunk + 1 - first + 1) // 2)
        hi = min(n, ((c + 1) * chunk - first) // 2 + 1)
        seg, r = o[lo:hi], ref[lo:hi]
        bad = (seg != r).nonzero().flatten()
        print(f"chunk {c}: elements [{lo}, {hi}) unwritten {(seg == -1).sum().item()} mismatch {bad.numel()} "
              f"first bad {(bad[:4] + lo).tolist()} last bad {(bad[-4:] + lo).tolist()}", flush=True)
    base = work[:20562].cpu().numpy().view(np.uint32)
    sys.path.insert(0, ROOT)
    from oracle import mt19937 as MT
    wref = MT.extend(words, 20562)
    print("base mismatch", int((base != wref).sum()), "first", np.nonzero(base != wref)[0][:5].tolist(), flush=True)
    win = work[20562:20562 + nch * 640].cpu().numpy().view(np.uint32).reshape(nch, 640)
    wfull = MT.extend(words, nch * chunk + 700)
    for c in range(1, nch):
        d = np.nonzero(win[c, 1:625] != wfull[c * chunk + 1:c * chunk + 625])[0]
        print(f"window {c}: mismatch {d.size} first {d[:5].tolist()}", flush=True)
