#!/bin/bash
# Round-3 HEAD counter passes of the two resblock forward kinds the bench times (conv1: fp32 operand; conv2:
# FG_PRESPLIT operand), summarised into the files bench.py reads for roofline.traffic, then the bench.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for kind in fwd_stats fwd_stats_ps; do
  KIND=$kind scripts/gpu_pmc.sh r3x_$kind > gpurun_out/r3x_pmc_$kind.log 2>&1 || { echo "pmc $kind failed"; cat gpurun_out/r3x_pmc_$kind.log; exit 1; }
  python scripts/pmc_summary.py gpurun_out/pmc_r3x_$kind conv_fwd_f3 "conv_fwd_f3_kernel<256,256,...,STATS>" $kind \
      > gpurun_out/r3x_pmc_resblock_$kind.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r3x_pmc_resblock_$kind.json')); print('$kind', {k: d.get(k) for k in ('launch_s','clock_ghz','mfma_busy','hbm_bytes','l2_hit')})"
done
