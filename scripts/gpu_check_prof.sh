#!/bin/bash
# conv-engine tests (pipelined kernel tiles / streams / pre-split / the step parity), then one kernel-trace profile
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
TAG=${TAG:-chk}
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_northstar.py -x -q --timeout 300 --timeout-method thread \
    -k "${TESTK:-conv or presplit or instnorm or block or step or northstar or bs8 or convT or fused}" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
scripts/gpu_profile.sh $TAG > gpurun_out/${TAG}_prof.log 2>&1 || { echo "profile failed"; exit 1; }
python scripts/kstats.py $(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1) 4 24
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/prof_$TAG/bench.log
