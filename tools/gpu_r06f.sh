#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "g4 or dx_forward" \
  > gpurun_out/r06f_tests.log 2>&1 || { tail -30 gpurun_out/r06f_tests.log; exit 1; }
tail -2 gpurun_out/r06f_tests.log
timeout -k 10 300 python3 tools/dx_ab.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 400 python3 tools/g4_time.py 2>&1 | grep -v amdgpu.ids | tail -30
