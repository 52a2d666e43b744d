#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_northstar.py tests/test_gpu_cycle.py -x -q --timeout 300 --timeout-method thread \
    -k "step or northstar or bs8 or cycle or gen or input_grad" > gpurun_out/r3af_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3af_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ab_step.py stem_pad4 4 5 > gpurun_out/r3af_ab_stem_pad4.log 2>&1; rc=$?; tail -2 gpurun_out/r3af_ab_stem_pad4.log; exit $rc
