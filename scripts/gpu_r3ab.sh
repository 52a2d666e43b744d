#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_northstar.py tests/test_gpu_cycle.py -x -q --timeout 300 --timeout-method thread \
    -k "dual or presplit or instnorm or block or step or northstar or bs8 or cycle or gen" > gpurun_out/r3ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3ab_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ab_step.py ps_resid 4 5 > gpurun_out/r3ab_ab_ps_resid.log 2>&1; rc=$?; tail -2 gpurun_out/r3ab_ab_ps_resid.log; exit $rc
