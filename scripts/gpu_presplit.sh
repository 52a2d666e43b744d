#!/bin/bash
# pre-split operand checks: the new unit tests, the norm / conv / block / step parity tests, then an interleaved A/B
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r3n}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_northstar.py -x -q --timeout 300 --timeout-method thread \
    -k "presplit or instnorm or block or step or northstar or gen or bs8 or smoke" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ab_step.py presplit 4 5 > gpurun_out/${TAG}_ab_presplit.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_ab_presplit.log; exit $rc
