#!/bin/bash
# A/B of an alternative build (AB_LIB, e.g. tools/_ab/libmmfd_nt.so) against the in-tree library on
# one box, interleaved (new, alt, new, alt): the encoder GEMM shapes and the bench step of AB_DTYPE
# (bf16 default, or fp32).
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/lib_ab
mkdir -p $O
for r in 1 2; do
  for v in base alt; do
    if [ $v = alt ]; then export MMFD_LIB_PATH=$AB_LIB; else unset MMFD_LIB_PATH; fi
    timeout -k 10 300 python3 tools/gemm_bench.py --dtype ${AB_DTYPE:-bf16} --iters 10 > $O/gemm_${v}_$r.log 2>&1
    timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --precision ${AB_DTYPE:-bf16} --no-bf16 > $O/bench_${v}_$r.log 2>&1
    echo "$v $r done"
  done
done
