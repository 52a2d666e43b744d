#!/bin/bash
# Interleaved in-process A/B runs of engine switches on the full bs-8 512^2 step (scripts/ab_step.py), each under
# its own time limit, plus optional micro-benchmarks (MICRO="script1.py script2.py").
#   SWITCHES="stem_wgrad win_rs" ROUNDS=3 STEPS=5 scripts/gpu_ab_step.sh <tag>
cd "$(dirname "$0")/.." || exit 1
TAG=${1:-ab}
mkdir -p gpurun_out
for s in $MICRO; do
  timeout -k 10 300 python "scripts/$s" > "gpurun_out/${TAG}_$(basename "$s" .py).log" 2>&1 \
    || { echo "$s failed"; tail -20 "gpurun_out/${TAG}_$(basename "$s" .py).log"; exit 1; }
  cat "gpurun_out/${TAG}_$(basename "$s" .py).log"
done
for s in $SWITCHES; do
  timeout -k 10 400 python scripts/ab_step.py "$s" "${ROUNDS:-3}" "${STEPS:-5}" > "gpurun_out/${TAG}_ab_$s.log" 2>&1 \
    || { echo "ab $s failed"; tail -20 "gpurun_out/${TAG}_ab_$s.log"; exit 1; }
  cat "gpurun_out/${TAG}_ab_$s.log"
done
