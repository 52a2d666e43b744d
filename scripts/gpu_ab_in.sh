cd /root/repo && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "instnorm or fused_in_stats" > gpurun_out/r3m_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3m_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/ab_step.py in_rows 4 5 > gpurun_out/r3m_ab_in_rows.log 2>&1; rc=$?; cat gpurun_out/r3m_ab_in_rows.log | tail -3; exit $rc
