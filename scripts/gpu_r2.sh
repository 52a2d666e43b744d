#!/bin/bash
# One GPU session (round 2): GPU parity tests, smoke, bench, and (PROF=1) a rocprofv3 kernel trace of
# the bench.  Each GPU step has its own time limit; a test failure (rc 1) does not stop the session,
# anything else (fault, abort, time limit) does.
#   TAG=r2a scripts/gpu_r2.sh [pytest selection args...]
cd "$(dirname "$0")/.." || exit 1
REPO=$(pwd)
TAG=${TAG:-r2}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {   # name limit cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -4 "$OUT/${TAG}_$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
if [ "${TESTS:-1}" = 1 ]; then
  # pytest selection: the arguments, else the whole GPU suite
  SEL=("$@"); [ ${#SEL[@]} -eq 0 ] && SEL=(tests)
  run tests ${TEST_LIMIT:-1200} python -u -m pytest -m gpu -v -rf --timeout 300 --timeout-method thread "${SEL[@]}"
fi
if [ "${SMOKE:-1}" = 1 ]; then run smoke 300 python -u __graft_entry__.py smoke; fi
if [ "${BENCH:-1}" = 1 ]; then run bench 600 python -u bench.py --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS}; fi
if [ "${PROF:-0}" = 1 ]; then
  P="$OUT/prof_${TAG}"
  mkdir -p "$P"
  cd /tmp
  run prof 600 rocprofv3 --kernel-trace --stats -d "$P" -o prof --output-format csv -- \
      python3 "$REPO/bench.py" --steps ${PSTEPS:-4} --warmup 2 --no-cpu-baseline ${BENCH_ARGS}
fi
echo "session done"
