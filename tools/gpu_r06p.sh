#!/bin/bash
# four-wave GEMM past K = 1024 (FFN2 forward, FFN1 data gradient at K = 3072): step A/B of
# MMFD_G4_KMAX=4096 (+ MMFD_DX_TRANSPOSED=2) against the default limit
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for r in 1 2; do
  for v in 0 1 2; do
    unset MMFD_G4_KMAX MMFD_DX_TRANSPOSED
    if [ $v = 1 ]; then export MMFD_G4_KMAX=4096; fi
    if [ $v = 2 ]; then export MMFD_G4_KMAX=4096 MMFD_DX_TRANSPOSED=2; fi
    timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/r06p_b$v$r.log 2>&1 || { tail -20 gpurun_out/r06p_b$v$r.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/r06p_b$v$r.log'):
    if l.startswith('{'):
        d = json.loads(l); b = d.get('bf16') or {}
        print('kmax_variant=$v run$r', d['value'], d['ms_per_step'], d['roofline']['frac'], b.get('value'), b.get('ms_per_step'))"
  done
done
