cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/x6d_t.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/x6d_t.log; exit 1; }
echo TESTS_OK; tail -2 gpurun_out/x6d_t.log
AB_CMD="python tools/x6f_check.py" bash tools/ab_swap.sh
grep -h "ms\|err" gpurun_out/ab_new1.log | tail -25
echo ---- old; grep -h "ms\|err" gpurun_out/ab_old1.log | tail -25
