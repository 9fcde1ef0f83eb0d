#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_layers_gpu.py \
  tests/test_fusion_gpu.py -k "attn or attention or head or fusion or mha or layer" > gpurun_out/r06e_tests.log 2>&1 || { tail -30 gpurun_out/r06e_tests.log; exit 1; }
tail -2 gpurun_out/r06e_tests.log
for arm in 0; do
  timeout -k 10 600 python tools/attn_bench.py --ab-generic --dtype bf16 > gpurun_out/r06e_attn_$arm.log 2>&1 || { tail gpurun_out/r06e_attn_$arm.log; exit 1; }
done
cat gpurun_out/r06e_attn_0.log
