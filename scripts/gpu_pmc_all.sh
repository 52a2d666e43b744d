#!/bin/bash
# Counter passes for the kernels bench.py's roofline names (the three resblock conv kinds) and the stem strip
# kernels, each summarised into gpurun_out/<tag>_pmc_*.json (copy into profiles/<round>/); stops at the first failing pass.
#   scripts/gpu_pmc_all.sh r4 round4 ["fwd_stats_ps dgrad_ps wgrad_ps stem_wgrad stem_fwd"]
cd "$(dirname "$0")/.." || exit 1
TAG=${1:-r4}; RD=${2:-round4}; KINDS=${3:-"fwd_stats_ps dgrad_ps wgrad_ps stem_wgrad stem_fwd"}
mkdir -p "profiles/$RD"
for k in $KINDS; do
  case $k in
    fwd_stats_ps) key=conv_fwd_f3; ktag="conv_fwd_f3_kernel<256,256,...,STATS>"; name=resblock_fwd_stats_ps;;
    dgrad_ps) key=conv_fwd_f3; ktag="conv_fwd_f3_kernel<256,256,...> (input-gradient interior)"; name=resblock_dgrad_ps;;
    wgrad_ps) key=conv_wgrad_f3; ktag="conv_wgrad_f3_kernel<256,0,3>"; name=resblock_wgrad_ps;;
    stem_wgrad) key=stem_wgrad_kernel; ktag="stem_wgrad_kernel"; name=stem_wgrad;;
    stem_fwd) key=stem_fwd_kernel; ktag="stem_fwd_kernel"; name=stem_fwd;;
    win_fwd) key=conv_win2_kernel; ktag="conv_win2_kernel<7>"; name=win_fwd;;
    quad_stats) key="true, true, true>"; ktag="conv_fwd_f3_kernel<256,256,...,STATS,PS,QUAD> (deconv2)"; name=deconv2_quad;;
    convT4_stats) key="512, 64, 64, 64, 2, 3, true, true, false>"; ktag="conv_fwd_f3_kernel<512,64,...> (deconv2 4 phases)"; name=deconv2_4phase;;
    *) echo "unknown kind $k"; exit 1;;
  esac
  KIND=$k scripts/gpu_pmc.sh "${TAG}_$k" || { echo "pmc $k failed"; exit 1; }
  python scripts/pmc_summary.py "gpurun_out/pmc_${TAG}_$k" "$key" "$ktag" "$k" > "gpurun_out/${TAG}_pmc_$name.json" \
    || { echo "summary $k failed"; exit 1; }
  cat "gpurun_out/${TAG}_pmc_$name.json"
done
