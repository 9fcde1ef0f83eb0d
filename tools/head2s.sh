#!/bin/bash
# Two-stream fusion head: fusion GPU tests, then the bench with MMFD_SERIAL_HEAD=1 vs the default.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fusion_gpu.py tests/test_predict_gpu.py -m gpu -x -v --timeout 200 \
  --timeout-method thread > gpurun_out/h_t.log 2>&1 || { echo TESTS_FAILED; exit 1; }; echo TESTS_OK
MMFD_SERIAL_HEAD=1 timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/h_serial.log 2>&1
echo SERIAL_OK
timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/h_two.log 2>&1
echo TWO_OK
