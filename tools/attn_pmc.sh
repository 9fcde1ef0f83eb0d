#!/bin/bash
# PMC passes over tools/attn_bench.py (run via gpurun from the repo root); counters per pass fit one
# SQ block (8 slots).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/attn_pmc
mkdir -p $OUT
timeout -k 10 300 python3 tools/attn_bench.py > $OUT/bench.txt
timeout -k 10 300 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  -d $OUT/p1 -o run --output-format csv -- python3 tools/attn_bench.py --iters 2 > /dev/null
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM \
  -d $OUT/p2 -o run --output-format csv -- python3 tools/attn_bench.py --iters 2 > /dev/null
