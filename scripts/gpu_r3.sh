#!/bin/bash
# Round-3 GPU session: the whole -m gpu suite, smoke, a short bench and a kernel-trace profile, each step under
# its own limit; stops at the first abnormal exit.  TAG names the outputs (gpurun_out/<TAG>_*).
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-r3}
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q -rf --timeout 600 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: abnormal pytest exit"; exit $rc; fi
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/${TAG}_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps ${BENCH_STEPS:-10} --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*' gpurun_out/${TAG}_bench.log; [ $rc -ne 0 ] && exit $rc
scripts/gpu_profile.sh $TAG > gpurun_out/${TAG}_prof.log 2>&1 || { echo "profile failed"; exit 1; }
python scripts/kstats.py $(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1) 4 16
