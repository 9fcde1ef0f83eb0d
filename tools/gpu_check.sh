#!/bin/bash
# GPU-box check: full GPU test suite, smoke(), then the bench line (run via gpurun from the repo root).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo TESTS_FAILED; exit 1; }; echo TESTS_OK
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; exit 1; }; echo SMOKE_OK
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/b.log 2>&1 && echo BENCH_OK
fi
