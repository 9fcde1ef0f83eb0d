#!/bin/bash
# split-operand ext instantiation (GELU_D / MUL_AUX in x6f): tests, then the fp32 step with the GELU
# derivative saved (MMFD_GELU_DERIV=1, default) vs the pre-activation (=0), same library, interleaved
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
OUT=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  tests/test_trainer_gpu.py tests/test_fullsize_gpu.py > $OUT/r06z3_tests.log 2>&1 || { tail -40 $OUT/r06z3_tests.log; exit 1; }
tail -1 $OUT/r06z3_tests.log
for r in 1 2; do
  for v in 0 1; do
    MMFD_GELU_DERIV=$v timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-bf16 > $OUT/r06z3_t$v$r.log 2>&1 || { tail -20 $OUT/r06z3_t$v$r.log; exit 1; }
    python3 -c "
import json
for l in open('$OUT/r06z3_t$v$r.log'):
    if l.startswith('{'):
        d = json.loads(l)
        print('deriv=$v run$r', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
  done
done
