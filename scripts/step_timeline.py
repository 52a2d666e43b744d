#!/usr/bin/env python3
"""The conv-family launches of ONE timed step of a bench.py kernel trace, in order, with duration and grid
(rocprofv3 --kernel-trace CSV; the warm-up steps are skipped as in kstats_timed.py).
  python scripts/step_timeline.py <prof_kernel_trace.csv> <warmup steps> [all]"""
import csv
import sys

from kstats_timed import timed_rows


def main():
    rows = timed_rows(list(csv.DictReader(open(sys.argv[1]))), int(sys.argv[2]))
    everything = len(sys.argv) > 3
    groups, conv_since = 0, True
    for r in rows:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        if "adam_kernel" in n:
            if conv_since:
                groups += 1
                conv_since = False
            if groups == 2:
                break
            continue
        if "conv" in n:
            conv_since = True
        if not everything and not any(k in n for k in ("conv", "win", "stem", "n1_", "head")):
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        blocks = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        print(f"{d:8.1f} us  grid {blocks:6d}x{r['Grid_Size_Y']:>3}  {n.split('(')[0][:90]}")


if __name__ == "__main__":
    main()
