#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bench_f3_presplit.py 4,5,10 > gpurun_out/r3v_f3_presplit_cfg.log 2>&1; rc=$?; cat gpurun_out/r3v_f3_presplit_cfg.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_northstar.py -x -q --timeout 300 --timeout-method thread \
    -k "presplit or f3_tiles or fused or step or bs8 or block" > gpurun_out/r3v_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3v_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ab_step.py ps_wide 3 5 4,5,10 > gpurun_out/r3v_ab_ps_wide.log 2>&1; rc=$?; tail -3 gpurun_out/r3v_ab_ps_wide.log; exit $rc
