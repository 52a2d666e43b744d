#!/bin/bash
# Kernel-trace profile of a short bench run (rocprofv3 --kernel-trace --stats, CSV).
REPO="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$REPO/gpurun_out/prof_${1:-run}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT" -o prof --output-format csv -- \
    python3 "$REPO/bench.py" --workload ${WORKLOAD:-paired} --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-fp32-math > "$OUT/bench.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
find "$OUT" -name "*kernel_stats.csv" | head -3
exit $rc
