"""One training step's kernel dispatches, in order, from a rocprofv3 kernel_trace.csv (the last step
of a bench run): name, grid, duration; plus per-kernel totals and the resblock-forward launches.
  python scripts/trace_step.py gpurun_out/prof_X/prof_kernel_trace.csv [steps_in_trace]"""
import csv
import re
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    return n.replace("void ", "")[:60]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # a step = from the first dispatch after the previous step's last Adam launch to its own last
    # Adam launch; each step has exactly one tail_fwd (the generator's composite)
    tails = [i for i, r in enumerate(rows) if "tail_fwd_kernel" in r["Kernel_Name"]]
    adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    start = max(i for i in adam if i < tails[-1]) + 1
    end = max(adam)
    last = rows[start:end + 1]
    t0 = int(last[0]["Start_Timestamp"])
    tot = {}
    for r in last:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[short(r["Kernel_Name"])] = tot.get(short(r["Kernel_Name"]), 0) + d
        g = f'{r["Grid_Size_X"]}x{r["Grid_Size_Y"]}'
        print(f'{(int(r["Start_Timestamp"]) - t0) / 1e3:9.1f} us {d:8.1f} us  {g:>12s}  {short(r["Kernel_Name"])}')
    span = (int(last[-1]["End_Timestamp"]) - t0) / 1e3
    busy = sum(tot.values())
    print(f"\nstep span {span / 1e3:.2f} ms, kernel busy {busy / 1e3:.2f} ms, {len(last)} dispatches")
    for k, v in sorted(tot.items(), key=lambda t: -t[1])[:30]:
        print(f"{v / 1e3:7.2f} ms  {k}")


if __name__ == "__main__":
    main()
