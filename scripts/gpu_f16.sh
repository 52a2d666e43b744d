#!/bin/bash
# f16x3 evaluation: accuracy + tile sweep, GPU tests and bench under FLOODGAN_CONV_MATH=$MATH.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
MATH=${MATH:-f16x3}
MODES=${MODES:-bf16x6,f16x3} TILES=${TILES:-0,1,2,3,4,5} WTILES=${WTILES:-0,1,2,3} \
  timeout -k 10 600 python scripts/bench_conv.py > gpurun_out/bench_conv.log 2>&1
rc=$?; echo "bench_conv rc=$rc"; grep accuracy gpurun_out/bench_conv.log
[ $rc -eq 0 ] || { tail -20 gpurun_out/bench_conv.log; exit $rc; }
FLOODGAN_CONV_MATH=$MATH timeout -k 10 600 python -m pytest tests -m gpu -q -rf --timeout=500 > gpurun_out/gpu_tests_$MATH.log 2>&1
rc=$?; echo "pytest($MATH) rc=$rc"; tail -25 gpurun_out/gpu_tests_$MATH.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
FLOODGAN_CONV_MATH=$MATH timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$MATH.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/bench_$MATH.log
exit $rc
