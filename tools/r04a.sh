#!/bin/bash
# Round-4 first GPU pass: the new parity tests (config 2 at bs=64, config 3 at bs=256, split-operand
# GEMMs at the bench shapes), the graph-captured DP step on world-1 RCCL, memory accounting, DP overhead.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fullsize_gpu.py tests/test_kernels_gpu.py tests/test_dp_gpu.py -k "bs256 or bs64 or bench_shapes or graph_captured" > gpurun_out/r04_parity.log 2>&1 || { echo TESTS_FAILED; exit 1; }
echo TESTS_OK
timeout -k 10 300 python tools/mem_account.py --out gpurun_out/r04_memory.json > gpurun_out/r04_mem.log 2>&1 || { echo MEM_FAILED; exit 1; }
echo MEM_OK
timeout -k 10 300 python tools/dp_overhead.py 5 > gpurun_out/r04_dp_overhead.log 2>&1 || { echo DPO_FAILED; exit 1; }
echo DPO_OK
timeout -k 10 400 python bench.py --workload extract --steps 5 --warmup 2 > gpurun_out/r04_extract.log 2>&1 || { echo EXTRACT_FAILED; exit 1; }
echo EXTRACT_OK
