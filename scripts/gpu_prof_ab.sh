#!/bin/bash
# kernel-trace profiles of the same short bench under an environment switch (VAR=0 / VAR=1): per-kernel A/B
cd "$(dirname "$0")/.." || exit 1
VAR=${VAR:-FLOODGAN_PRESPLIT}
TAG=${TAG:-ab}
for v in 0 1; do
  export $VAR=$v
  scripts/gpu_profile.sh ${TAG}_$v > gpurun_out/${TAG}_$v.log 2>&1 || { echo "profile $v failed"; exit 1; }
done
for v in 0 1; do
  echo "== $VAR=$v"; python scripts/kstats.py $(find gpurun_out/prof_${TAG}_$v -name "*kernel_stats.csv" | head -1) 4 16
done
