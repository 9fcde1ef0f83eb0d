#!/bin/bash
# GPU box: kernel trace of the DeBERTa pre-embedding workload.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_pe
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 bench.py --workload preembed --steps 3 --warmup 1 > $OUT/bench.json
