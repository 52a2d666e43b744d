cd /root/repo
FLOODGAN_LIB=$PWD/flood-prediction-gan_amd/build/diag/libfloodgan.so timeout -k 10 400 python -u scripts/diag_f3_narrow.py > gpurun_out/r3q_diag_narrow.log 2>&1; rc=$?; cat gpurun_out/r3q_diag_narrow.log; [ $rc -ne 0 ] && exit $rc
TAG=r3r TESTK="presplit or instnorm or block or step or northstar or bs8 or convT or fused or disc or cycle or dp or tail or decisions" bash scripts/gpu_check_prof.sh
