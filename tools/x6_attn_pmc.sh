#!/bin/bash
# PMC passes over the fp32 split-operand attention kernels (tools/attn_bench.py --dtype fp32),
# summarised per kernel by tools/pmc_kernels.py
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/x6a_pmc${DBG:-0}
mkdir -p $OUT
export MMFD_X6A_DBG=${DBG:-0}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  -d $OUT/p1 -o run --output-format csv -- python3 tools/attn_bench.py --dtype fp32 --iters 2 > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES \
  -d $OUT/p2 -o run --output-format csv -- python3 tools/attn_bench.py --dtype fp32 --iters 2 > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_ACTIVE_INST_MISC SQ_WAIT_INST_VALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE \
  -d $OUT/p3 -o run --output-format csv -- python3 tools/attn_bench.py --dtype fp32 --iters 2 > /dev/null || exit 1
python3 tools/pmc_kernels.py $OUT attn > $OUT/summary.txt; cat $OUT/summary.txt
