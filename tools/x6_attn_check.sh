#!/bin/bash
# split-operand fp32 attention: kernel tests vs fp64, then per-call times (split vs native fp32, bf16)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "attention or attn" > gpurun_out/x6a_t.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/x6a_t.log; exit 1; }
echo TESTS_OK; tail -3 gpurun_out/x6a_t.log
timeout -k 10 200 python -u tools/attn_bench.py --dtype fp32 --fp32-mode split > gpurun_out/x6a_b.log 2>&1 &&
timeout -k 10 200 python -u tools/attn_bench.py --dtype fp32,bf16 --fp32-mode native >> gpurun_out/x6a_b.log 2>&1
cat gpurun_out/x6a_b.log
if [ -f tools/_stamps/libmmfd_hip_x6astamps.so ] && [ "${STAMPS:-0}" = 1 ]; then
  timeout -k 10 120 python tools/x6a_stamps.py vit && timeout -k 10 120 python tools/x6a_stamps.py bert
fi
