#!/bin/bash
# f3 kernel iteration: its parity tests, the micro-benchmark, the full GPU suite, one bench.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "f3_tiles or window or wgrad_f3 or wgrad_window" -x -q --timeout 120 --timeout-method thread > gpurun_out/f3_tests.log 2>&1
rc=$?; echo "f3 tests rc=$rc"; tail -5 gpurun_out/f3_tests.log; [ $rc -eq 0 ] || exit $rc
(cd scripts && timeout -k 10 300 python -u bench_f3.py) > gpurun_out/bench_f3.log 2>&1
rc=$?; echo "bench_f3 rc=$rc"; cat gpurun_out/bench_f3.log; [ $rc -eq 0 ] || exit $rc
[ -n "$QUICK" ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
exit $rc
