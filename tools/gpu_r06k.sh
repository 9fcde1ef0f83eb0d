#!/bin/bash
# partitioned split-K reduce: GEMM / trainer tests, then step A/B against tools/_ab/skr_old (HEAD's reduce)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  tests/test_trainer_gpu.py tests/test_fullsize_gpu.py > gpurun_out/r06k_tests.log 2>&1 || { tail -40 gpurun_out/r06k_tests.log; exit 1; }
tail -2 gpurun_out/r06k_tests.log
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export MMFD_LIB_PATH=tools/_ab/skr_old/libmmfd_hip.so; else unset MMFD_LIB_PATH; fi
    timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/r06k_b$v$r.log 2>&1 || { tail -20 gpurun_out/r06k_b$v$r.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/r06k_b$v$r.log'):
    if l.startswith('{'):
        d = json.loads(l); b = d.get('bf16') or {}
        print('$v run$r', d['value'], d['ms_per_step'], d['roofline']['frac'], b.get('value'), b.get('ms_per_step'))"
  done
done
