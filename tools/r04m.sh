#!/bin/bash
# Round-4: bf16 attention counters (two SQ passes) and a kernel trace over tools/attn_bench.py
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04m
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 200 python3 tools/attn_bench.py --dtype bf16 > $OUT/bench.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  -d $OUT/p1 -o run --output-format csv -- python3 tools/attn_bench.py --dtype bf16 --iters 2 > $OUT/p1.log 2>&1
echo P1_OK
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM \
  -d $OUT/p2 -o run --output-format csv -- python3 tools/attn_bench.py --dtype bf16 --iters 2 > $OUT/p2.log 2>&1
echo P2_OK
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_VMEM SQ_WAIT_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_BRANCH SQ_CYCLES \
  -d $OUT/p3 -o run --output-format csv -- python3 tools/attn_bench.py --dtype bf16 --iters 2 > $OUT/p3.log 2>&1 || echo P3_FAILED
python3 tools/pmc_kernels.py $OUT attn > $OUT/summary.txt
echo DONE
