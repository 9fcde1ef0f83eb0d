#!/bin/bash
# round 6: targeted GPU tests for the hygiene changes, then the config-5 extract profile
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "g4 or embed" > gpurun_out/r06a_tests.log 2>&1 || { tail -30 gpurun_out/r06a_tests.log; exit 1; }
tail -3 gpurun_out/r06a_tests.log
bash tools/prof_extract.sh
