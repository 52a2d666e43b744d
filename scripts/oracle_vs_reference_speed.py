"""Build-container check: the CPU oracle step (oracle/paired_attention.py, the
bench's cpu_baseline "port") runs at the speed of the reference's own Model.train_paired()
(models/model.py:598-658) on the same synthetic 512x512 tiles, threads and batch sizes, so the
bench's CPU number stands for the reference's CPU path.  Imports the reference read-only through
the stub harness of tests/golden/make_golden.py; writes nothing but its log.

  python scripts/oracle_vs_reference_speed.py > profiles/round2/oracle_vs_reference_speed.log
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import torch  # noqa: E402

from make_golden import REF, _install_stubs  # noqa: E402
from oracle import paired_attention as O  # noqa: E402

THREADS = int(os.environ.get("THREADS", "8"))
R = 512


class TimedLoader:
    """yields the same batch `n` times and stamps the wall clock at every yield"""

    def __init__(self, x, y, n):
        self.x, self.y, self.n, self.stamps = x, y, n, []

    def __iter__(self):
        for _ in range(self.n):
            self.stamps.append(time.perf_counter())
            yield self.x, self.y, ["synthetic"] * self.x.shape[0]
        self.stamps.append(time.perf_counter())

    def __len__(self):
        return self.n


def reference_rate(x, y, iters):
    from models import model as M     # the reference, imported read-only
    m = M.Model(model="pairedattention", dataset_subset="usa", dataset_dem="same", data_path="/nonexistent",
                num_epochs=1, topography="all", resize=R, verbose=False)
    m.save_results = lambda **k: None
    m.train_loader = TimedLoader(x, y, iters + 1)
    m.train_paired()
    st = m.train_loader.stamps
    return x.shape[0] * iters / (st[-1] - st[1])          # iteration 0 is the warm-up


def oracle_rate(x, y, iters):
    st = O.PairedStepOracle()
    st.step(x, y)
    t0 = time.perf_counter()
    for _ in range(iters):
        st.step(x, y)
    return x.shape[0] * iters / (time.perf_counter() - t0)


def main():
    torch.set_num_threads(THREADS)
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    _install_stubs()
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(REF)
    print(f"torch {torch.__version__}, {THREADS} threads, {os.cpu_count()} logical CPUs; 512x512 topography=all")
    try:
        for bs, iters in ((1, 3), (8, 2)):
            g = torch.Generator().manual_seed(4321)
            x = torch.rand((bs, 9, R, R), generator=g) * 2 - 1
            y = torch.rand((bs, 3, R, R), generator=g) * 2 - 1
            ref = reference_rate(x, y, iters)
            orc = oracle_rate(x, y, iters)
            print(f"batch {bs}: reference train_paired {ref:.4f} img/s, oracle step {orc:.4f} img/s, "
                  f"oracle/reference {orc / ref:.3f} ({iters} timed iterations after 1 warm-up)", flush=True)
    finally:
        os.chdir(cwd)


if __name__ == "__main__":
    main()
