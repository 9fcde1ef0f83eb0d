#!/bin/bash
# config-5 extract regression hunt: the tree vs variants with one source file from the session start
# (tools/_ab/vA: gemm_tiles.h, vB: gemm.hip, vC: layernorm.hip) and the whole session-start tree
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
OUT=$GRAFT_REPO_ROOT/gpurun_out
for r in 1 2; do
  for v in new vA vB vC s0; do
    unset MMFD_LIB_PATH; D=.
    case $v in vA|vB|vC) export MMFD_LIB_PATH=tools/_ab/$v/libmmfd_hip.so;; s0) D=tools/_ab/s0tree;; esac
    (cd $D && timeout -k 10 400 python3 bench.py --workload extract --steps 5 --warmup 2 --no-cpu-baseline > $OUT/r06t_$v$r.json 2>$OUT/r06t_$v$r.err) || { tail -5 $OUT/r06t_$v$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/r06t_$v$r.json').read().strip().splitlines()[-1]); print('$v$r', d['value'], d['images_per_s_per_gpu'], d['texts_per_s_per_gpu'], d['bf16']['images_per_s_per_gpu'], d['bf16'].get('texts_per_s_per_gpu'))"
  done
done
