#!/bin/bash
# kernel traces of the step with and without the fused attention head, then its bit-identity test and an A/B
cd "$(dirname "$0")/.." || exit 1
for v in 0 1; do
  FLOODGAN_FUSED_HEAD=$v STEPS=3 timeout -k 10 400 bash scripts/gpu_profile.sh r5f_head$v > /dev/null 2>&1 || { echo "prof $v failed"; exit 1; }
  python scripts/kstats.py $(find gpurun_out/prof_r5f_head$v -name "*kernel_stats.csv" | head -1) 2>/dev/null | head -0
  grep -hE "in_apply_rows|in_bwd_apply_rows|in_bwd_stats_u|conv1x1" $(find gpurun_out/prof_r5f_head$v -name "*kernel_stats.csv" | head -1) | cut -c1-160
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_northstar.py -k fused_attention_head 2>&1 | tail -2
timeout -k 10 400 python scripts/ab_step.py fused_head 4 5 > gpurun_out/r5f_ab_fused_head.log 2>&1 || exit 1
tail -2 gpurun_out/r5f_ab_fused_head.log
