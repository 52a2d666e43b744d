#!/bin/bash
# round 5: the DP U-criterion tests, the 512^2 update test, the determinism test, then the default bench line
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_dp.py \
    tests/test_gpu_northstar.py -k "two_rank or update_teacher or deterministic" > gpurun_out/r5b_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r5b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r5b_bench.log 2>&1
rc=$?; tail -c 600 gpurun_out/r5b_bench.log; exit $rc
