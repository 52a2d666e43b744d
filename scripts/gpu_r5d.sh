cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_pix2pix.py -k "torch_stream or host_dropout" > gpurun_out/r5d_tests.log 2>&1
tail -40 gpurun_out/r5d_tests.log
