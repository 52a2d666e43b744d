#!/bin/bash
# A/B run: micro-bench, GPU tests in bf16x6 mode, full bench in both maths.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/bench_conv.py > gpurun_out/bench_conv.log 2>&1 || { echo "bench_conv failed"; tail gpurun_out/bench_conv.log; exit 1; }
FLOODGAN_CONV_MATH=bf16x6 timeout -k 10 600 python -m pytest tests -m gpu -q --timeout=500 > gpurun_out/gpu_tests_x6.log 2>&1
rc=$?; echo "pytest(bf16x6) rc=$rc"; tail -3 gpurun_out/gpu_tests_x6.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for m in fp32 fwd_x6 bf16x6; do
  FLOODGAN_CONV_MATH=$m timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$m.log 2>&1 || exit 1
  echo "$m: $(grep -o '"value": [0-9.]*' gpurun_out/bench_$m.log) $(grep -o '"achieved": [0-9.]*' gpurun_out/bench_$m.log)"
done
