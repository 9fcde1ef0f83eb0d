#!/bin/bash
# Round-4: bf16 K-tile segments split into fragment reads / refill issue / vmcnt wait (G8_PSTAMP 17-20)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04i
timeout -k 10 120 python3 tools/g8_stamps.py 100864 3072 768 gelu bf16 1 > gpurun_out/r04i/stamps_ffn1.log 2>&1
timeout -k 10 120 python3 tools/g8_stamps.py 100864 768 3072 plain bf16 1 > gpurun_out/r04i/stamps_ffn2.log 2>&1
echo STAMPS_OK
