#!/bin/bash
# Round-4: compiler scheduling strategies (max-memory-clause, max-ilp) on the whole library — GEMM GPU
# tests on each variant, then same-box GEMM A/B (fp32 split-operand and bf16) against the in-tree build
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in smc silp; do
  MMFD_LIB_PATH=tools/_ab/$v/libmmfd_hip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > gpurun_out/r04o_${v}_test.log 2>&1 || { echo ${v}_TEST_FAILED; tail -20 gpurun_out/r04o_${v}_test.log; exit 1; }
  echo ${v}_TEST_OK; tail -1 gpurun_out/r04o_${v}_test.log
done
for v in smc silp; do
  for dt in fp32 bf16; do
    rm -rf gpurun_out/lib_ab
    AB_WHAT=gemm AB_DTYPE=$dt AB_LIB=tools/_ab/$v/libmmfd_hip.so bash tools/lib_ab.sh
    mv gpurun_out/lib_ab gpurun_out/lib_ab_${v}_$dt
  done
done
