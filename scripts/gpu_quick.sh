#!/bin/bash
# A short GPU session for a change under test: the targeted parity tests (TESTS, pytest -k expression), then the
# bench and its kernel profile, then (AB=1) the A/B switches; every step under its own limit, stop at the first
# failure.   TESTS="stem or window" TAG=r4b AB=1 SWITCHES="stem_wgrad" scripts/gpu_quick.sh
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-quick}
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "$TESTS" --timeout 300 --timeout-method thread \
      > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; tail -5 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
fi
timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-10} --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 \
  || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/${TAG}_bench.log
if [ -n "$PROF" ]; then
  scripts/gpu_profile.sh $TAG > /dev/null 2>&1 || { echo "profile failed"; exit 1; }
fi
if [ -n "$AB" ]; then
  scripts/gpu_ab_step.sh $TAG || exit 1
fi
echo "quick done"
