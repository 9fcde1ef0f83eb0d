#!/bin/bash
# LayerNorm two-rows-per-wave bf16 kernels + prefetching backward: LN tests, then old/new LN timings
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "layernorm" > gpurun_out/r06h_tests.log 2>&1 || { tail -40 gpurun_out/r06h_tests.log; exit 1; }
tail -2 gpurun_out/r06h_tests.log
for r in 1 2; do
  MMFD_LIB_PATH=tools/_ab/ln_old/libmmfd_hip.so timeout -k 10 200 python tools/ln_bench.py 2>&1 | grep RESULT | sed "s/^RESULT/old$r/"
  timeout -k 10 200 python tools/ln_bench.py 2>&1 | grep RESULT | sed "s/^RESULT/new$r/"
done
