#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for t in 512 256 512 128; do
  echo "== FG_IN_BWD_WG=$t"
  FG_IN_BWD_WG=$t timeout -k 10 200 python -u scripts/ab_step.py presplit 3 5 1 2>&1 | tail -1
done > gpurun_out/r3ai_bwd_wg.log 2>&1
cat gpurun_out/r3ai_bwd_wg.log
