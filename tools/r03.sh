#!/bin/bash
# Round-3 profile set (fused-plane split-operand fp32 GEMMs), run via gpurun from the repo root:
# the fp32 headline step with the encoders and the head halves serialized (per-kernel figures that match the bench's
# GEMM probe): kernel trace + FETCH_SIZE + WRITE_SIZE + MFMA counters; the step as benched (two
# streams, graph) kernel trace only; the bf16 leg's kernel trace + HBM passes.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${TAG:-r03a}
MMFD_SERIAL_ENCODERS=1 MMFD_SERIAL_HEAD=1 STEPS=4 BENCH_ARGS="--precision fp32 --no-bf16" bash tools/profile.sh ${T}_fp32
MMFD_SERIAL_ENCODERS=1 MMFD_SERIAL_HEAD=1 BENCH_ARGS="--precision fp32 --no-bf16" bash tools/pmc_mfma.sh ${T}_fp32
PMC=0 STEPS=4 BENCH_ARGS="--precision fp32 --no-bf16" bash tools/profile.sh ${T}_fp32_step
MMFD_SERIAL_ENCODERS=1 MMFD_SERIAL_HEAD=1 STEPS=4 BENCH_ARGS="--precision bf16 --no-bf16" bash tools/profile.sh ${T}_bf16
python3 tools/pmc_mfma_summary.py gpurun_out/prof_${T}_fp32 ${T}_fp32
MMFD_SERIAL_ENCODERS=1 MMFD_SERIAL_HEAD=1 BENCH_ARGS="--precision bf16 --no-bf16" bash tools/pmc_mfma.sh ${T}_bf16
