#!/bin/bash
# GPU box A/B of two builds on one box: tools/_ab/libmmfd_old.so (a previous commit's csrc, built
# by hand) vs the in-tree library, interleaved (old, new, old, new) so clock drift hits both.
#   AB_WHAT="bench attn" bash tools/ab.sh
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OLD=tools/_ab/libmmfd_old.so
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export MMFD_LIB_PATH=$OLD; else unset MMFD_LIB_PATH; fi
    for w in ${AB_WHAT:-bench attn}; do
      if [ $w = bench ]; then
        timeout -k 10 240 python bench.py --steps ${AB_STEPS:-8} --warmup 2 --no-cpu-baseline > gpurun_out/ab_b.log 2>&1
        python -c "import json,sys; d=json.loads(open('gpurun_out/ab_b.log').read().strip().splitlines()[-1]); print('$v bench', d['value'], 'pairs/s', d['roofline']['achieved'], 'TF/s')"
      elif [ $w = attn ]; then
        timeout -k 10 120 python tools/attn_bench.py --iters 20 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /"
      elif [ $w = gemm ]; then
        timeout -k 10 200 python tools/gemm_epi_bench.py 2>&1 | grep "^RESULT" | sed "s/^RESULT/$v/"
      fi
    done
  done
done
