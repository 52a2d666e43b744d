#!/bin/bash
# A/B of the f16x3 pack cache (FLOODGAN_PACK_CACHE), interleaved bench runs on one box, after the pack
# tests and the step parity tests; each step under its own time limit, stop at the first failure.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_northstar.py tests/test_gpu_cycle.py tests/test_gpu_pix2pix.py tests/test_gpu_custom_ops.py \
  > gpurun_out/abp_tests.log 2>&1 || { tail -30 gpurun_out/abp_tests.log; exit 1; }
tail -2 gpurun_out/abp_tests.log
i=0
for v in 0 1 0 1; do
  i=$((i + 1))
  FLOODGAN_PACK_CACHE=$v timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline \
    > gpurun_out/abp_${i}_cache$v.log 2>&1 || { tail -5 gpurun_out/abp_${i}_cache$v.log; exit 1; }
  echo "cache=$v $(grep -o '"value": [0-9.]*' gpurun_out/abp_${i}_cache$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abp_${i}_cache$v.log)"
done
