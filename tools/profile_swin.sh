#!/bin/bash
# GPU box: bench line + kernel trace of the Swinv2 image pre-embedding workload.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_swin
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --workload preembed_image --steps 10 --warmup 3 ${SWIN_ARGS:-} > $OUT/bench.json
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 bench.py --workload preembed_image --steps 3 --warmup 1 ${SWIN_ARGS:-} > $OUT/bench_prof.json
