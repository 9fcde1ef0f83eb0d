#!/bin/bash
# Round-4: max-ilp scheduling variant — same-box bench-step A/B (bf16, then fp32) against the in-tree build
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/lib_ab
AB_WHAT=bench AB_LIB=tools/_ab/silp/libmmfd_hip.so bash tools/lib_ab.sh
mv gpurun_out/lib_ab gpurun_out/lib_ab_silp_bench_bf16
AB_WHAT=bench AB_DTYPE=fp32 AB_LIB=tools/_ab/silp/libmmfd_hip.so bash tools/lib_ab.sh
mv gpurun_out/lib_ab gpurun_out/lib_ab_silp_bench_fp32
