#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "wgrad or conv_fwd_wgrad" > gpurun_out/r3ad_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3ad_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ab_step.py wgrad_f3 3 5 0,2 > gpurun_out/r3ad_ab.log 2>&1; rc=$?; tail -2 gpurun_out/r3ad_ab.log; [ $rc -ne 0 ] && exit $rc
TAG=r3ad scripts/gpu_r3.sh
