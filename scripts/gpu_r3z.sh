#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "phase_stream or convT or fused or f3_tiles or presplit" > gpurun_out/r3z_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3z_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_narrow_cfg.py > gpurun_out/r3z_narrow.log 2>&1; rc=$?; cat gpurun_out/r3z_narrow.log | head -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ab_step.py phase 3 5 > gpurun_out/r3z_ab_phase.log 2>&1; rc=$?; tail -2 gpurun_out/r3z_ab_phase.log; exit $rc
