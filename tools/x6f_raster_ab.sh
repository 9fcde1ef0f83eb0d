#!/bin/bash
# x6f grouped tile raster (MMFD_X6F_GROUP_M, an option removed after this measurement: profiles/r04_x6f_raster_ab.log): fp32 encoder GEMM times interleaved per setting, then FETCH_SIZE
# per dispatch of the forward instantiation for each setting (one --pmc pass each)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/x6f_raster
mkdir -p $O
for r in 1 2; do
  for g in 1 4 8; do
    MMFD_X6F_GROUP_M=$g timeout -k 10 300 python3 tools/gemm_bench.py --dtype fp32 --iters 5 > $O/gemm_g${g}_$r.log 2>&1
    echo "g$g $r done"
  done
done
for g in 1 4 8; do
  MMFD_X6F_GROUP_M=$g timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_g$g -o run --output-format csv -- python3 tools/gemm_bench.py --dtype fp32 --iters 2 > $O/pmc_g$g.log 2>&1
  echo "pmc g$g done"
done
