#!/bin/bash
# Round-2 profile set (run via gpurun from the repo root): the fp32 headline step as the bench runs
# it (graph replay, two encoder streams) and, for per-kernel figures that match the bench's
# serialized GEMM probe, the same command with the encoders on one stream (MMFD_SERIAL_ENCODERS=1):
# kernel trace + FETCH_SIZE + WRITE_SIZE + MFMA counters; the bf16 leg likewise.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PMC=0 STEPS=5 BENCH_ARGS="--precision fp32 --no-bf16" bash tools/profile.sh r02e_fp32_step
MMFD_SERIAL_ENCODERS=1 STEPS=5 BENCH_ARGS="--precision fp32 --no-bf16" bash tools/profile.sh r02e_fp32
MMFD_SERIAL_ENCODERS=1 BENCH_ARGS="--precision fp32 --no-bf16" bash tools/pmc_mfma.sh r02e_fp32
MMFD_SERIAL_ENCODERS=1 STEPS=5 BENCH_ARGS="--precision bf16 --no-bf16" bash tools/profile.sh r02e_bf16
MMFD_SERIAL_ENCODERS=1 BENCH_ARGS="--precision bf16 --no-bf16" bash tools/pmc_mfma.sh r02e_bf16
