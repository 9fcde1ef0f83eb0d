#!/bin/bash
# x6 attention output stores: attention kernel tests, then old/new A/B of tools/attn_bench.py with
# the encoders' plane outputs (tools/_ab/libmmfd_old.so = the previous build)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "attention or attn" > gpurun_out/xs_t.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/xs_t.log; exit 1; }
echo TESTS_OK; tail -2 gpurun_out/xs_t.log
LIB=multimodal-misinformation-detection_amd/libmmfd_hip.so
cp $LIB gpurun_out/_new.so
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then cp tools/_ab/libmmfd_old.so $LIB; else cp gpurun_out/_new.so $LIB; fi
    timeout -k 10 200 python -u tools/attn_bench.py --dtype fp32 --planes --iters 10 > gpurun_out/xs_$v$r.log 2>&1
    echo "== $v$r"; cat gpurun_out/xs_$v$r.log
  done
done
cp gpurun_out/_new.so $LIB
rm -f gpurun_out/_new.so
