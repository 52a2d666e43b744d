import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "flood-prediction-gan_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(R, kind="paired_step"):
        path = os.path.join(ROOT, "tests", "golden", f"{kind}_{R}.npz")
        z = np.load(path, allow_pickle=False)
        return {k.replace("__", "."): z[k] for k in z.files}

    return load


@pytest.fixture(scope="session")
def report():
    """Append measured parity numbers to gpurun_out/parity_report.jsonl (evidence for DESIGN.md)."""
    import json

    path = os.path.join(ROOT, "gpurun_out", "parity_report.jsonl")
    os.makedirs(os.path.dirname(path), exist_ok=True)

    def rec(name, **vals):
        with open(path, "a") as f:
            f.write(json.dumps({"test": name, **vals}) + "\n")

    return rec
