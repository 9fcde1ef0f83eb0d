#!/bin/bash
# round 6: implicit-GEMM conv tests + the evidence tests, then the extract bench (fp32 + bf16)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_conv_gpu.py tests/test_kernels_gpu.py \
  tests/test_evidence_gpu.py -k "conv or narrow or resnet or im2col or corpus or gemm or image" > gpurun_out/r06b_tests.log 2>&1 || { tail -40 gpurun_out/r06b_tests.log; exit 1; }
tail -3 gpurun_out/r06b_tests.log
timeout -k 10 400 python3 bench.py --workload extract --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r06b_extract.json 2> gpurun_out/r06b_extract.err || { tail -20 gpurun_out/r06b_extract.err; exit 1; }
MMFD_CONV_IM2COL=1 timeout -k 10 400 python3 bench.py --workload extract --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r06b_extract_im2col.json 2> gpurun_out/r06b_extract_im2col.err
python3 - <<'P'
import json
for f in ("gpurun_out/r06b_extract.json", "gpurun_out/r06b_extract_im2col.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["images_per_s_per_gpu"], d.get("bf16", {}).get("images_per_s_per_gpu"), d["roofline"]["kernel"], d["roofline"]["frac"])
P
