#!/bin/bash
# split-operand fp32 attention phase experiment: full / staging without HBM loads / staging only
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for d in 0 1 2; do
  echo "MMFD_X6A_DBG=$d"
  MMFD_X6A_DBG=$d timeout -k 10 200 python -u tools/attn_bench.py --dtype fp32 --fp32-mode split 2>&1 | grep fp32 || exit 1
done
