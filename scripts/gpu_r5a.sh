set -o pipefail
cd $GRAFT_REPO_ROOT
STEPS=3 timeout -k 10 400 bash scripts/gpu_profile.sh r5a > gpurun_out/r5a_prof.log 2>&1 || { echo prof failed; exit 1; }
python scripts/kstats_timed.py $(find gpurun_out/prof_r5a -name "*kernel_trace.csv" | head -1) 1 3 gpurun_out/r5a_kernel_stats_timed.csv > gpurun_out/r5a_kstats.txt 2>&1
PASS_TIMEOUT=200 bash scripts/gpu_pmc_step.sh r5a > gpurun_out/r5a_pmcstep.log 2>&1 || { echo pmc failed; cat gpurun_out/r5a_pmcstep.log; exit 1; }
python scripts/pmc_step_summary.py gpurun_out/pmcstep_r5a 80 > gpurun_out/r5a_pmc_step.json
echo done
