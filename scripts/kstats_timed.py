#!/usr/bin/env python3
"""Kernel statistics of bench.py's TIMED steps only, from a rocprofv3 --kernel-trace CSV (the --stats summary
also counts the warm-up steps: first-use weight packs, buffer fills).

A paired / cycle step ends with its optimiser launches: an Adam group is a run of adam_kernel launches with no
conv launch in between (Adam(D), then Adam(G)).  With W warm-up steps the timed region starts after the
2W-th group (the first non-Adam, non-pack launch after it).

  python scripts/kstats_timed.py <prof_kernel_trace.csv> <warmup steps> <timed steps> [out_stats.csv]

Prints per-step kernel time, launches per step, sub-15-us launches per step and the top kernels; writes a
kernel_stats-format CSV (Name, Calls, TotalDurationNs, AverageNs, Percentage) of the timed region."""
import csv
import sys


def timed_rows(rows, warmup, groups_per_step=2):
    rows = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
    groups, conv_since, start = 0, True, None
    for i, r in enumerate(rows):
        n = r["Kernel_Name"]
        if "adam_kernel" in n:
            if conv_since:
                groups += 1
                conv_since = False
            continue
        if "conv" in n:
            conv_since = True
        if groups >= warmup * groups_per_step and "pack" not in n and start is None:
            start = i
            break
    return rows[start:] if start is not None else []


def main():
    path, warmup, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    rows = timed_rows(list(csv.DictReader(open(path))), warmup)
    stats = {}
    for r in rows:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        s = stats.setdefault(r["Kernel_Name"], [0, 0])
        s[0] += 1
        s[1] += d
    tot = sum(v[1] for v in stats.values())
    small = sum(1 for r in rows if int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) < 15000)
    print(f"timed region: {len(rows)} launches over {steps} steps = {len(rows) / steps:.1f} per step; "
          f"kernel time {tot / 1e6 / steps:.2f} ms per step; launches under 15 us: {small / steps:.1f} per step")
    for name, (c, t) in sorted(stats.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f"{t / 1e6 / steps:8.3f} ms {c / steps:6.1f}x {t / c / 1e3:8.1f}us  "
              f"{name.replace('(anonymous namespace)::', '')[:110]}")
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for name, (c, t) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
                w.writerow([name, c, t, t / c, 100.0 * t / tot])


if __name__ == "__main__":
    main()
