#!/bin/bash
# GPU tests named by TESTS (optional), then an interleaved new/old A/B of the default bench line
# (tools/_ab/libmmfd_old.so = the previous build, swapped in place)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_t.log 2>&1 \
    || { echo TESTS_FAILED; tail -30 gpurun_out/ab_t.log; exit 1; }
  echo TESTS_OK; tail -1 gpurun_out/ab_t.log
fi
LIB=multimodal-misinformation-detection_amd/libmmfd_hip.so
cp $LIB gpurun_out/_new.so
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then cp tools/_ab/libmmfd_old.so $LIB; else cp gpurun_out/_new.so $LIB; fi
    timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline $BENCH_ARGS > gpurun_out/bab_$v$r.log 2>&1
    python3 -c "
import json
for l in open('gpurun_out/bab_$v$r.log'):
    if l.startswith('{'):
        d = json.loads(l); b = d.get('bf16') or {}
        print('$v$r', d['value'], d['ms_per_step'], d['roofline']['frac'], b.get('value'), b.get('ms_per_step'))"
  done
done
cp gpurun_out/_new.so $LIB
rm -f gpurun_out/_new.so
