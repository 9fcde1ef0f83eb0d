#!/bin/bash
# Round-4: bf16 attention fixed modes (tests + A/B against the generic mode), then the bf16 GEMM diagnosis
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04e
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" > gpurun_out/r04f_attn_test.log 2>&1 || { echo ATTN_TEST_FAILED; tail -30 gpurun_out/r04f_attn_test.log; exit 1; }
echo ATTN_TEST_OK
timeout -k 10 300 python tools/attn_bench.py --dtype bf16 --ab-generic > gpurun_out/r04f_attn_bench.log 2>&1 || { echo ATTN_BENCH_FAILED; tail -20 gpurun_out/r04f_attn_bench.log; exit 1; }
echo ATTN_BENCH_OK
bash tools/r04e.sh && echo GEMM_DIAG_OK
