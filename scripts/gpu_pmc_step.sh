#!/bin/bash
# Counter passes (rocprofv3 --pmc, kernel trace only) over ONE bench step (bs 8, 512^2) after one warm-up,
# so that every kernel of the step gets its counters from the binary the bench runs.  Summarise with
#   python scripts/pmc_step_summary.py gpurun_out/pmcstep_<tag> > profiles/.../<tag>_pmc_step.json
REPO="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$REPO/gpurun_out/pmcstep_${1:-run}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CMD=(python3 "$REPO/bench.py" --workload "${WORKLOAD:-paired}" --steps 1 --warmup 1 --no-cpu-baseline --no-fp32-math)
[ -f "$OUT/avail.txt" ] || timeout -k 10 120 rocprofv3 -L > "$OUT/avail.txt" 2>&1
i=0
while read -r pass; do
  [ -z "$pass" ] && continue
  i=$((i+1))
  [ -n "$MAXPASS" ] && [ $i -gt $MAXPASS ] && break
  timeout -s KILL ${PASS_TIMEOUT:-240} rocprofv3 --pmc $pass --kernel-trace -d "$OUT/p$i" -o pmc --output-format csv -- \
      "${CMD[@]}" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($pass) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done <<PASSES
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
PASSES
exit 0
