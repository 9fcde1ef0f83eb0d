#!/bin/bash
# Profile the default bench workload on the GPU box (run via gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats          -> per-kernel time summary
#   2. rocprofv3 --pmc FETCH_SIZE  (own pass)     -> HBM read bytes per dispatch
#   3. rocprofv3 --pmc WRITE_SIZE  (own pass)     -> HBM write bytes per dispatch
# then tools/pmc_summary.py folds them into profiles/<tag>_*.{csv,json}.
# BENCH_ARGS (default: fp32 headline leg only) selects the bench line that is profiled.
set -e
TAG=${1:-r01}
STEPS=${STEPS:-5}
BENCH_ARGS=${BENCH_ARGS:---precision fp32 --no-bf16}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 bench.py --steps $STEPS --warmup 2 --no-cpu-baseline $BENCH_ARGS > $OUT/bench_trace.json
if [ "${PMC:-1}" = 0 ]; then exit 0; fi
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $OUT/bench_fetch.json
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $OUT/bench_write.json
python3 tools/pmc_summary.py $OUT $TAG
