#!/bin/bash
# G4 data-gradient (transposed weight) tests, the bf16 full-size tests, then a same-box bench A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "transpose or dx_forward or g4" > gpurun_out/r06d_tests.log 2>&1 || { tail -30 gpurun_out/r06d_tests.log; exit 1; }
tail -2 gpurun_out/r06d_tests.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_fullsize_gpu.py tests/test_encoders_gpu.py \
  > gpurun_out/r06d_tests2.log 2>&1 || { tail -30 gpurun_out/r06d_tests2.log; exit 1; }
tail -2 gpurun_out/r06d_tests2.log
for arm in 1 0 2 1 0 2; do
  MMFD_DX_TRANSPOSED=$arm timeout -k 10 600 python bench.py --precision bf16 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06d_bench_$arm.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r06d_bench_$arm.json').read().strip().splitlines()[-1]); print('dxT=$arm', d['value'], d['roofline']['kernel'], d['roofline']['frac'])"
done
