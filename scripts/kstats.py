#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel_stats.csv: top kernels by total time (per-step if --steps)."""
import csv
import sys


def main():
    path = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total {tot / 1e6 / steps:.2f} ms per step ({steps:g} steps)")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
        print(f'{float(r["TotalDurationNs"]) / 1e6 / steps:8.3f} ms {int(r["Calls"]) / steps:7.1f}x '
              f'{float(r["AverageNs"]) / 1e3:8.1f}us  {r["Name"][:120]}')


if __name__ == "__main__":
    main()
