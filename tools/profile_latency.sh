#!/bin/bash
# GPU box: kernel trace of the single-pair latency workload (graph replay + eager).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_lat
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 bench.py --workload latency --steps 10 --warmup 2 > $OUT/bench.json
