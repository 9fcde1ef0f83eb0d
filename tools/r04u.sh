#!/bin/bash
# Round-4: gemm.hip with max-ilp and without SLP vectorisation (no register spills in any GEMM
# instantiation) — GEMM tests, same-box bf16 GEMM and bench-step A/B against the in-tree build (max-ilp)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MMFD_LIB_PATH=tools/_ab/ilpnoslp/libmmfd_hip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > gpurun_out/r04u_test.log 2>&1 || { echo TEST_FAILED; tail -20 gpurun_out/r04u_test.log; exit 1; }
echo TEST_OK
rm -rf gpurun_out/lib_ab
AB_WHAT="gemm bench" AB_LIB=tools/_ab/ilpnoslp/libmmfd_hip.so bash tools/lib_ab.sh
mv gpurun_out/lib_ab gpurun_out/lib_ab_ilpnoslp
