#!/bin/bash
# Round-4: AMDGPU register-pressure trackers + no unclustered high-RP reschedule (whole library) — GEMM
# tests, then same-box bench-step A/B (fp32, bf16) against the in-tree build
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MMFD_LIB_PATH=tools/_ab/fboth/libmmfd_hip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or attention or layernorm" > gpurun_out/r04s_test.log 2>&1 || { echo TEST_FAILED; tail -20 gpurun_out/r04s_test.log; exit 1; }
echo TEST_OK
rm -rf gpurun_out/lib_ab
AB_WHAT=bench AB_DTYPE=fp32 AB_LIB=tools/_ab/fboth/libmmfd_hip.so bash tools/lib_ab.sh
mv gpurun_out/lib_ab gpurun_out/lib_ab_fboth_fp32
AB_WHAT=bench AB_LIB=tools/_ab/fboth/libmmfd_hip.so bash tools/lib_ab.sh
mv gpurun_out/lib_ab gpurun_out/lib_ab_fboth_bf16
