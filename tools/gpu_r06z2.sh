#!/bin/bash
# the extended activations' full epilogue through the reduce (new test)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "ext_acts or gelu_deriv or mul_aux" > gpurun_out/r06z2_tests.log 2>&1 || { tail -40 gpurun_out/r06z2_tests.log; exit 1; }
tail -1 gpurun_out/r06z2_tests.log
