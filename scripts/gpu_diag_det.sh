#!/bin/bash
# Run-to-run determinism of the step under several switch settings (scripts/diag_determinism.py), each its own
# process under its own limit; stops at the first failing run.
cd "$(dirname "$0")/.." || exit 1
TAG=${1:-det}; REPS=${REPS:-30}; RES=${RES:-128}; BS=${BS:-8}
mkdir -p gpurun_out
run() {
  timeout -k 10 240 env "$@" >> gpurun_out/${TAG}_det.log 2>&1 || { echo "run $* failed"; tail -5 gpurun_out/${TAG}_det.log; exit 1; }
}
: > gpurun_out/${TAG}_det.log
run python scripts/diag_determinism.py $REPS $RES $BS
run FLOODGAN_F3_NARROW=0 python scripts/diag_determinism.py $REPS $RES $BS
run FLOODGAN_STEM_FWD=0 python scripts/diag_determinism.py $REPS $RES $BS
run python scripts/diag_determinism.py $REPS $RES $BS head_1x1=0
run python scripts/diag_determinism.py $REPS $RES $BS splitpix=0
run python scripts/diag_determinism.py $REPS $RES $BS use_win=0
grep "repeats differ" gpurun_out/${TAG}_det.log
