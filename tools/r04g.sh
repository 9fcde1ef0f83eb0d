#!/bin/bash
# Round-4: full GPU suite on the attention fixed modes, then the names of the hipBLASLt kernels torch.matmul picks
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
BENCH=0 bash tools/gpu_check.sh
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/blaslt -o run --output-format csv -- python3 tools/blaslt_names.py > gpurun_out/blaslt.log 2>&1 && echo BLASLT_OK
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b.log 2>&1 && echo BENCH_OK
