#!/bin/bash
# Round-4: dropout keep-bitmask — kernel tests, the attention parity tests, full-size step parity, attention timing
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" > gpurun_out/r04_attn_test.log 2>&1 || { echo ATTN_TEST_FAILED; tail -30 gpurun_out/r04_attn_test.log; exit 1; }
echo ATTN_TEST_OK
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fullsize_gpu.py tests/test_layers_gpu.py tests/test_fusion_gpu.py tests/test_trainer_gpu.py > gpurun_out/r04_step_test.log 2>&1 || { echo STEP_TEST_FAILED; tail -30 gpurun_out/r04_step_test.log; exit 1; }
echo STEP_TEST_OK
timeout -k 10 300 python tools/attn_bench.py > gpurun_out/r04_attn_bench.log 2>&1 || { echo ATTN_BENCH_FAILED; tail -20 gpurun_out/r04_attn_bench.log; exit 1; }
echo ATTN_BENCH_OK
