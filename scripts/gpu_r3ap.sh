#!/bin/bash
# conv_win strip-fragment prefetch: window parity tests, then the A/B on the content head
set -o pipefail
mkdir -p gpurun_out
FLOODGAN_WIN_APF=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "conv_window" > gpurun_out/r3ap_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/diag_win_waves.py > gpurun_out/r3ap_win_apf.log 2>&1
