#!/bin/bash
# Round-4: four-wave AGPR split-operand GEMM — bitwise check against x6f, then the A/B timing
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "x6w" > gpurun_out/r04_x6w_test.log 2>&1 || { echo X6W_TEST_FAILED; tail -30 gpurun_out/r04_x6w_test.log; exit 1; }
echo X6W_TEST_OK
timeout -k 10 300 python tools/x6w_ab.py 3 > gpurun_out/r04_x6w_ab.log 2>&1 || { echo X6W_AB_FAILED; tail -20 gpurun_out/r04_x6w_ab.log; exit 1; }
echo X6W_AB_OK
cat gpurun_out/r04_x6w_ab.log
