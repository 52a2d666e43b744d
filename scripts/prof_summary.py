"""Per-step kernel time table from a rocprofv3 --stats kernel_stats.csv."""
import csv
import sys

path, steps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6 / steps:.1f} ms/step")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    n = r["Name"].replace("(anonymous namespace)::", "")[:100]
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:7.2f} ms/step {int(r['Calls']) // steps:4d} calls "
          f"{float(r['AverageNs']) / 1e3:8.1f} us  {n}")
