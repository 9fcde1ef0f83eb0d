#!/bin/bash
# Round-4: scheduler strategies for the attention kernels — attention tests per variant, then same-box
# attention A/B (bf16 and fp32 split-operand) against the in-tree build
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ailp amc; do
  MMFD_LIB_PATH=tools/_ab/$v/libmmfd_hip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" > gpurun_out/r04t_${v}_test.log 2>&1 || { echo ${v}_TEST_FAILED; tail -20 gpurun_out/r04t_${v}_test.log; exit 1; }
  echo ${v}_TEST_OK
  rm -rf gpurun_out/lib_ab
  AB_WHAT=attn AB_DTYPE=bf16,fp32 AB_LIB=tools/_ab/$v/libmmfd_hip.so bash tools/lib_ab.sh
  mv gpurun_out/lib_ab gpurun_out/lib_ab_${v}_attn
done
