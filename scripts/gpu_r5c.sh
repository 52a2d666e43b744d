#!/bin/bash
# round 5: the Pix2Pix tests (device torch-stream masks bit-exact vs torch's CPU draws), the fused attention head's
# bit-identity test, the Pix2Pix bench in both dropout modes, an interleaved A/B of the fused head
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pix2pix.py \
    tests/test_gpu_northstar.py -k "pix2pix or torch_stream or host_dropout or fused_attention_head" \
    > gpurun_out/r5c_tests.log 2>&1
rc=$?; tail -25 gpurun_out/r5c_tests.log; [ $rc -eq 0 ] || exit $rc
for mode in host device; do
  timeout -k 10 300 python bench.py --workload pix2pix --dropout-rng $mode --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/r5c_pix_$mode.log 2>&1 || { tail -20 gpurun_out/r5c_pix_$mode.log; exit 1; }
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r5c_pix_$mode.log
done
timeout -k 10 400 python scripts/ab_step.py fused_head 4 5 > gpurun_out/r5c_ab_fused_head.log 2>&1 \
    || { tail -20 gpurun_out/r5c_ab_fused_head.log; exit 1; }
tail -3 gpurun_out/r5c_ab_fused_head.log
