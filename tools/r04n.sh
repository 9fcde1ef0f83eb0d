#!/bin/bash
# Round-4: bf16 LayerNorm backward with the next row prefetched — LayerNorm GPU tests on the variant
# library, then same-box A/B of the bf16 bench step against the in-tree build
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MMFD_LIB_PATH=tools/_ab/lnpf/libmmfd_hip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "layernorm or ln_" > gpurun_out/r04n_ln_test.log 2>&1 || { echo LN_TEST_FAILED; tail -20 gpurun_out/r04n_ln_test.log; exit 1; }
echo LN_TEST_OK
tail -2 gpurun_out/r04n_ln_test.log
rm -rf gpurun_out/lib_ab
AB_WHAT=bench AB_LIB=tools/_ab/lnpf/libmmfd_hip.so bash tools/lib_ab.sh
