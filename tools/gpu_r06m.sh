#!/bin/bash
# LN microbench (fp32 backward without prefetch) + same-box A/B of the FFN1 forward on the four-wave
# kernel (MMFD_G4_GELU=1: EPI 5, GELU with its derivative to aux) against gemm256_kernel
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 200 python tools/ln_bench.py 2>&1 | grep RESULT
for r in 1 2; do
  for v in 0 1; do
    if [ $v = 1 ]; then export MMFD_G4_GELU=1; else unset MMFD_G4_GELU; fi
    timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/r06m_b$v$r.log 2>&1 || { tail -20 gpurun_out/r06m_b$v$r.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/r06m_b$v$r.log'):
    if l.startswith('{'):
        d = json.loads(l); b = d.get('bf16') or {}
        print('g4gelu=$v run$r', d['value'], d['ms_per_step'], d['roofline']['frac'], b.get('value'), b.get('ms_per_step'))"
  done
done
