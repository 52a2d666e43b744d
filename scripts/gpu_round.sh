#!/bin/bash
# One GPU session: tile micro-bench, parity tests + smoke + bench, a 2-rank gloo bench on the one GPU
# (DP2=1), kernel profile, counter passes on the resblock conv.  Every GPU step has its own limit;
# stop at the first failure.
cd "$(dirname "$0")/.." || exit 1
TAG=${TAG:-run}
mkdir -p gpurun_out
if [ -n "$TILES" ]; then
  ACCURACY=${ACCURACY:-0} MODES=${MODES:-f16x3} timeout -k 10 600 python scripts/bench_conv.py > gpurun_out/bench_conv.log 2>&1 \
    || { echo "bench_conv failed"; tail -20 gpurun_out/bench_conv.log; exit 1; }
fi
BENCH_ARGS=--no-cpu-baseline scripts/gpu_check.sh > gpurun_out/check.log 2>&1
rc=$?; grep -a "passed\|failed\|smoke:\|rc=" gpurun_out/check.log; [ $rc -eq 0 ] || exit $rc
grep -o '"value": [0-9.]*' gpurun_out/bench.log
if [ -n "$DP2" ]; then
  timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/bench_dp2_gloo.log 2>&1 \
    || { echo "dp2 bench failed"; tail -20 gpurun_out/bench_dp2_gloo.log; exit 1; }
  grep -o '"value": [0-9.]*\|"n_gpus": [0-9]*\|"parallelism": "[a-z0-9]*"' gpurun_out/bench_dp2_gloo.log
fi
scripts/gpu_profile.sh $TAG > /dev/null 2>&1 || { echo "profile failed"; exit 1; }
if [ -n "$PMC" ]; then
  for k in fwd_stats_ps dgrad_ps wgrad_ps; do
    KIND=$k scripts/gpu_pmc.sh ${TAG}_$k > /dev/null || { echo "pmc $k failed"; exit 1; }
  done
fi
echo "round done"
