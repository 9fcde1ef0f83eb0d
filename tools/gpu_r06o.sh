#!/bin/bash
# persistent four-wave GEMM: G4 tests, per-GEMM and step A/B against one workgroup per tile
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "g4 or dx_forward or gelu_deriv" > gpurun_out/r06o_tests.log 2>&1 || { tail -40 gpurun_out/r06o_tests.log; exit 1; }
tail -2 gpurun_out/r06o_tests.log
for r in 1 2; do
  for v in 0 1; do
    export MMFD_G4_PERSIST=$v
    timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/r06o_b$v$r.log 2>&1 || { tail -20 gpurun_out/r06o_b$v$r.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/r06o_b$v$r.log'):
    if l.startswith('{'):
        d = json.loads(l); b = d.get('bf16') or {}
        print('persist=$v run$r', d['value'], d['ms_per_step'], d['roofline']['frac'], b.get('value'), b.get('ms_per_step'))"
  done
done
