#!/bin/bash
# Round-3 switches at HEAD, each an interleaved A/B in one process (scripts/ab_step.py), one box
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for sw in presplit ps_resid in_rows f3_fill wgrad_f3; do
  echo "== $sw"
  timeout -k 10 240 python -u scripts/ab_step.py $sw 3 5 2>&1 | grep "ms/step" || exit 1
done > gpurun_out/r3an_ab_all.log 2>&1
rc=$?; cat gpurun_out/r3an_ab_all.log; exit $rc
