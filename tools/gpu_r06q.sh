#!/bin/bash
# LayerNorm backward grid size (gamma/beta partial rows): ln_bench at 2048 / 1024 / 512 / 256 blocks
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
  -k "layernorm" > gpurun_out/r06q_tests.log 2>&1 || { tail -40 gpurun_out/r06q_tests.log; exit 1; }
tail -1 gpurun_out/r06q_tests.log
for nb in 2048 1024 512 256; do
  MMFD_LN_BWD_BLOCKS=$nb timeout -k 10 200 python tools/ln_bench.py 2>&1 | grep RESULT | sed "s/^RESULT/blocks=$nb/"
done
timeout -k 10 300 python tools/x6f_epi_probe.py 2>&1 | grep RESULT
