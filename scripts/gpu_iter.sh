#!/bin/bash
# One optimisation iteration on the GPU box: conv micro-bench (tile sweep), GPU parity tests in
# the default math, one full bench.  Each GPU step has its own time limit; stop at the first failure.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
ACCURACY=${ACCURACY:-1} timeout -k 10 420 python scripts/bench_conv.py > gpurun_out/bench_conv.log 2>&1
rc=$?; echo "bench_conv rc=$rc"; tail -4 gpurun_out/bench_conv.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -x -q --timeout=500 > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*\|"achieved": [0-9.]*\|"frac": [0-9.]*' gpurun_out/bench.log
exit $rc
