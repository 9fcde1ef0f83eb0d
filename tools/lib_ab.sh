#!/bin/bash
# A/B of an alternative build (AB_LIB, e.g. tools/_ab/prev/libmmfd_hip.so from tools/build_variant.sh)
# against the in-tree library on one box, interleaved (base, alt, base, alt). AB_WHAT picks the
# measurements (default "gemm bench"): gemm = tools/gemm_bench.py, bench = the bench step, attn =
# tools/attn_bench.py; AB_DTYPE = bf16 (default) or fp32. Summary: tools/lib_ab_summary.py.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/lib_ab
mkdir -p $O
DT=${AB_DTYPE:-bf16}
for r in 1 2; do
  for v in base alt; do
    if [ $v = alt ]; then export MMFD_LIB_PATH=$AB_LIB; else unset MMFD_LIB_PATH; fi
    for w in ${AB_WHAT:-gemm bench}; do
      case $w in
        gemm) timeout -k 10 300 python3 tools/gemm_bench.py --dtype $DT --iters 10 > $O/gemm_${v}_$r.log 2>&1 ;;
        bench) timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --precision $DT --no-bf16 > $O/bench_${v}_$r.log 2>&1 ;;
        attn) timeout -k 10 200 python3 tools/attn_bench.py --dtype $DT --iters 20 > $O/attn_${v}_$r.log 2>&1 ;;
      esac
    done
    echo "$v $r done"
  done
done
