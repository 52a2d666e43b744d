#!/bin/bash
# Counter passes (rocprofv3 --pmc, kernel trace only) over scripts/conv_one.py.
REPO="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$REPO/gpurun_out/pmc_${1:-run}"
KIND=${KIND:-fwd}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/avail.txt" 2>&1
i=0
while read -r pass; do
  [ -z "$pass" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace -d "$OUT/p$i" -o pmc --output-format csv -- \
      python3 "$REPO/scripts/conv_one.py" $KIND 10 > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($pass) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done <<PASSES
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS
GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
PASSES
exit 0
