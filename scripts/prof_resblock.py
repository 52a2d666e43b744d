#!/usr/bin/env python3
"""Separate the resblock-forward launches of conv_fwd_f3_kernel<256,256,...> in a rocprofv3 kernel trace
of bench.py, so the bench line's live roofline (avg_launch_ms over the same launches) can be checked
against the profiler.

Within one training step (between two Adam(G) launches) the generator forward runs first: its 18
conv_fwd_f3_kernel<256,256> launches before the first InstanceNorm-backward kernel are the 9 resblocks'
conv1 / conv2 (conv3 and the heads use other tile configs; the discriminator convs run after the
generator).  Prints their mean duration per step and overall.
  python scripts/prof_resblock.py gpurun_out/prof_<tag>/prof_kernel_trace.csv"""
import csv
import statistics
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # a forward segment starts after a run of Adam launches (the previous step's optimiser steps) and
    # ends at the first InstanceNorm backward (the discriminator's backward of the D step)
    per_step, cur, state = [], None, "idle"
    for r in rows:
        n = r["Kernel_Name"]
        if "adam_kernel" in n:
            state = "adam"
            continue
        if state == "adam":
            state, cur = "fwd", []
            per_step.append(cur)
        if state == "fwd":
            if "in_bwd" in n:
                state = "idle"
            elif "conv_fwd_f3_kernel<256, 256" in n:
                cur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    # the generator's 18 resblock convs come first among the 256x256 launches of the forward
    per_step = [s[:18] for s in per_step if len(s) >= 18]
    allv = [v for s in per_step for v in s]
    for i, s in enumerate(per_step):
        print(f"step {i}: {len(s)} resblock forward launches, mean {statistics.mean(s):.4f} ms")
    print(f"overall: {len(allv)} launches, mean {statistics.mean(allv):.4f} ms, median {statistics.median(allv):.4f} ms;"
          f" 154.6 GFLOP per launch -> {154.618822656 / statistics.mean(allv):.1f} TFLOP/s")


if __name__ == "__main__":
    main()
