#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_northstar.py -x -q --timeout 300 --timeout-method thread \
    -k "wgrad or conv_fwd_wgrad or step or disc" > gpurun_out/r3ae_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3ae_tests.log; [ $rc -ne 0 ] && exit $rc
scripts/gpu_profile.sh r3ae > gpurun_out/r3ae_prof.log 2>&1 || exit 1
python scripts/kstats.py $(find gpurun_out/prof_r3ae -name "*kernel_stats.csv" | head -1) 4 60 | grep -i "total\|wgrad\|x6"
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/prof_r3ae/bench.log
