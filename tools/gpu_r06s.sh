#!/bin/bash
# config-5 extract: same-box A/B of the session-start tree (tools/_ab/s0tree: cc43c45's package and
# library) against the current tree
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
OUT=$GRAFT_REPO_ROOT/gpurun_out
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then D=tools/_ab/s0tree; else D=.; fi
    (cd $D && timeout -k 10 400 python3 bench.py --workload extract --steps 5 --warmup 2 --no-cpu-baseline > $OUT/r06s_$v$r.json 2>$OUT/r06s_$v$r.err) || { tail -5 $OUT/r06s_$v$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/r06s_$v$r.json').read().strip().splitlines()[-1]); print('$v$r', d['value'], d['images_per_s_per_gpu'], d['texts_per_s_per_gpu'], d['bf16']['images_per_s_per_gpu'], d['bf16'].get('texts_per_s_per_gpu'))"
  done
done
