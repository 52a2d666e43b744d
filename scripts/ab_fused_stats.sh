#!/bin/bash
# A/B of the InstanceNorm statistics fused into the conv epilogue (FLOODGAN_FUSED_IN_STATS), interleaved
# bench runs on one box; each step under its own time limit, stop at the first failure.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -m gpu -q -x --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k fused \
  > gpurun_out/ab_tests.log 2>&1 || { tail -20 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
i=0
for v in 0 1 0 1; do
  i=$((i + 1))
  FLOODGAN_FUSED_IN_STATS=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline \
    > gpurun_out/ab_${i}_fused$v.log 2>&1 || { tail -5 gpurun_out/ab_${i}_fused$v.log; exit 1; }
  echo "fused=$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_${i}_fused$v.log) $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/ab_${i}_fused$v.log)"
done
