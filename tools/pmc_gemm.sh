#!/bin/bash
# Counter passes over one bf16 GEMM shape, full epilogue vs. epilogue skipped (alpha = 12345):
#   bash tools/pmc_gemm.sh [M N K]   (run via gpurun; outputs under gpurun_out/pmc_gemm/)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
M=${1:-65536}; N=${2:-3072}; K=${3:-768}
OUT=gpurun_out/pmc_gemm; mkdir -p $OUT
for a in 1.0 12345.0; do
  ALPHA=$a timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU -d $OUT/a$a -o run --output-format csv -- python3 tools/gemm_one.py $M $N $K nt 5 > /dev/null
  ALPHA=$a timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/b$a -o run --output-format csv -- python3 tools/gemm_one.py $M $N $K nt 5 > /dev/null
done
echo done
