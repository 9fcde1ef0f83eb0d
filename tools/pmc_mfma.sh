#!/bin/bash
# MFMA-utilisation counters of the bench step (one rocprofv3 --pmc pass, kernel-trace only):
#   SQ_INSTS_VALU_MFMA_MOPS_F32 / _BF16 (x512 = MFMA FLOPs), SQ_VALU_MFMA_BUSY_CYCLES (MFMA-busy
#   SIMD cycles), SQ_INSTS_MFMA, SQ_INSTS_VALU, SQ_WAIT_ANY, SQ_WAVE_CYCLES, GRBM_GUI_ACTIVE
# then tools/pmc_mfma_summary.py writes profiles/<tag>_mfma.json.
set -e
TAG=${1:-r02}
BENCH_ARGS=${BENCH_ARGS:---precision fp32 --no-bf16}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES \
  SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $OUT/mfma -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $OUT/bench_mfma.json
