"""Golden split lists from the REFERENCE's own determine_flood_dataset (models/data.py:83-146).

Runs only in the build container (reference mounted read-only at /root/reference; its third-party
imports stubbed as in make_golden.py).  Writes tests/golden/dataset_splits.json.gz: for every subset x
DEM x crop the reference supports, the (file_name, version[, crop]) lists of train / validation /
test, and copies the split table the function reads (metadata/dataset_split.csv, a data file) to
tests/golden/dataset_split.csv as the fixture input.

Usage:  python tests/golden/make_golden_data.py
"""
import gzip
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF, _install_stubs  # noqa: E402

SUBSETS = ["usa", "india", "hurricane-harvey", "hurricane-florence", "midwest-flooding", "nepal-flooding",
           "harveyflorence", "harveyonflorence", "testing", "all"]


def main():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    _install_stubs()
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(REF)
    try:
        from models import data as D      # the reference, imported read-only
        out = {}
        for s in SUBSETS:
            for dem in ("best", "same"):
                for crop in (None, 4):
                    r = D.determine_flood_dataset(s, dem, crop)
                    out[f"{s}|{dem}|{crop}"] = {k: [list(map(lambda v: v if isinstance(v, str) else int(v), t))
                                                    for t in v] for k, v in r.items()}
        shutil.copyfile(os.path.join(REF, "metadata", "dataset_split.csv"), os.path.join(HERE, "dataset_split.csv"))
    finally:
        os.chdir(cwd)
    with gzip.open(os.path.join(HERE, "dataset_splits.json.gz"), "wt") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote", len(out), "split sets")


if __name__ == "__main__":
    main()
