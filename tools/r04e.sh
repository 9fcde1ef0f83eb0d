#!/bin/bash
# bf16 GEMM diagnosis (round 4): our 256x256 kernel vs hipBLASLt on the encoder shapes, and s_memtime
# phase stamps of the bf16 forward GEMMs (tools/g8_stamps.py on the prebuilt tools/_stamps library)
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 300 python3 tools/gemm_bench.py --dtype bf16 --lib --iters 10 > $O/gemm_bench_bf16.log 2>&1
timeout -k 10 120 python3 tools/g8_stamps.py 100864 3072 768 gelu bf16 > $O/stamps_ffn1.log 2>&1
timeout -k 10 120 python3 tools/g8_stamps.py 100864 2304 768 plain bf16 > $O/stamps_qkv.log 2>&1
timeout -k 10 120 python3 tools/g8_stamps.py 100864 768 3072 plain bf16 > $O/stamps_ffn2.log 2>&1
timeout -k 10 120 python3 tools/g8_stamps.py 100864 768 3072 gelubwd bf16 > $O/stamps_dx_gelubwd.log 2>&1
