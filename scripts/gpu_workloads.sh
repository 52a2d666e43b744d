#!/bin/bash
# The other workloads' bench lines (BASELINE configs 3/4 and Pix2Pix), one GPU, each step under its own limit.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
TAG=${TAG:-wl}
run() {   # name args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -o '"value": [0-9.]*, "unit": "[^"]*"\|"ms_per_step": [0-9.]*' "gpurun_out/${TAG}_$name.log" | tr '\n' ' '; echo
  [ $rc -ne 0 ] && exit $rc
  return 0
}
run attentiongan_512 --workload attentiongan
run cyclegan_512 --workload cyclegan
run attentiongan_256 --workload attentiongan --res 256
run attentiongan_tiles_crop4 --workload attentiongan --data tiles --crop 4 --res 512
run pix2pix_512 --workload pix2pix
echo "workloads done"
