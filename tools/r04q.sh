#!/bin/bash
# Round-4: the max-ilp scheduler on gemm.hip only (in-tree build) — full GPU check (tests, smoke, bench),
# then a same-box bench A/B against the default-scheduler build (tools/_ab/noilp: here "alt" is the OLD build)
set -e
cd "$GRAFT_REPO_ROOT"
BENCH_ARGS=" " bash tools/gpu_check.sh
rm -rf gpurun_out/lib_ab
AB_WHAT=bench AB_LIB=tools/_ab/noilp/libmmfd_hip.so bash tools/lib_ab.sh
mv gpurun_out/lib_ab gpurun_out/lib_ab_noilp_bf16
