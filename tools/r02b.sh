export TMPDIR=/tmp
mkdir -p gpurun_out/r02c
timeout -k 10 900 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_fullsize_gpu.py tests/test_kernels_gpu.py tests/test_dp_gpu.py > gpurun_out/r02c/t.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -le 1 ]; then
  timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/r02c/bench.json 2> gpurun_out/r02c/bench.err
  echo "bench rc=$?"
fi
