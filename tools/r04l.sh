#!/bin/bash
# Round-4: batched head staging (all loads of a batch before the LDS writes) and one-block-ahead row
# prefetch in the bf16 attention kernels — attention GPU tests on the variant library, then same-box A/B
# of the attention kernels and the bf16 bench step against the in-tree build
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MMFD_LIB_PATH=tools/_ab/stage/libmmfd_hip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" > gpurun_out/r04l_attn_test.log 2>&1 || { echo ATTN_TEST_FAILED; tail -20 gpurun_out/r04l_attn_test.log; exit 1; }
echo ATTN_TEST_OK
tail -3 gpurun_out/r04l_attn_test.log
rm -rf gpurun_out/lib_ab
AB_WHAT="attn bench" AB_LIB=tools/_ab/stage/libmmfd_hip.so bash tools/lib_ab.sh
