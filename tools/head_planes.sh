#!/bin/bash
# Fusion head GPU tests (+ predictor, full-size) and the default bench line.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fusion_gpu.py tests/test_predict_gpu.py tests/test_fullsize_gpu.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/hp_t.log 2>&1 || { echo TESTS_FAILED; exit 1; }; echo TESTS_OK
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/hp_b.log 2>&1
echo BENCH_OK
