#!/bin/bash
# lean 256x256 G8 instantiations (gemm256_kernel lean / gemm256_act_kernel): GEMM, full-size, conv, trainer
# tests, then extract and training A/B against tools/_ab/hd (HEAD's gemm256.h)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
OUT=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_fullsize_gpu.py tests/test_conv_gpu.py \
  tests/test_trainer_gpu.py > $OUT/r06yb_tests.log 2>&1 || { tail -40 $OUT/r06yb_tests.log; exit 1; }
tail -1 $OUT/r06yb_tests.log
for r in 1 2; do
  for v in new hd; do
    unset MMFD_LIB_PATH; [ $v = hd ] && export MMFD_LIB_PATH=tools/_ab/hd/libmmfd_hip.so
    timeout -k 10 400 python3 bench.py --workload extract --steps 5 --warmup 2 --no-cpu-baseline > $OUT/r06yb_x$v$r.json 2>$OUT/r06yb_x$v$r.err || { tail -5 $OUT/r06yb_x$v$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/r06yb_x$v$r.json').read().strip().splitlines()[-1]); print('extract $v$r', d['value'], d['images_per_s_per_gpu'], d['texts_per_s_per_gpu'], d['bf16']['images_per_s_per_gpu'], d['bf16'].get('texts_per_s_per_gpu'))"
  done
done
for r in 1 2; do
  for v in new hd; do
    unset MMFD_LIB_PATH; [ $v = hd ] && export MMFD_LIB_PATH=tools/_ab/hd/libmmfd_hip.so
    timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline > $OUT/r06yb_t$v$r.log 2>&1 || { tail -20 $OUT/r06yb_t$v$r.log; exit 1; }
    python3 -c "
import json
for l in open('$OUT/r06yb_t$v$r.log'):
    if l.startswith('{'):
        d = json.loads(l); b = d.get('bf16') or {}
        print('train $v$r', d['value'], d['ms_per_step'], d['roofline']['frac'], b.get('value'), b.get('ms_per_step'))"
  done
done
