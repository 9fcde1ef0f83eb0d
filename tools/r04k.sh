#!/bin/bash
# Round-4: single-launch LayerNorm gamma/beta reduction — LayerNorm GPU tests, then same-box A/B of the bf16
# and fp32 bench steps against the previous build (tools/_ab/prev)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "layernorm or ln_" > gpurun_out/r04k_ln_test.log 2>&1 || { echo LN_TEST_FAILED; tail -20 gpurun_out/r04k_ln_test.log; exit 1; }
echo LN_TEST_OK
rm -rf gpurun_out/lib_ab
AB_WHAT=bench AB_LIB=tools/_ab/prev/libmmfd_hip.so bash tools/lib_ab.sh
mv gpurun_out/lib_ab gpurun_out/lib_ab_bf16
AB_WHAT=bench AB_DTYPE=fp32 AB_LIB=tools/_ab/prev/libmmfd_hip.so bash tools/lib_ab.sh
