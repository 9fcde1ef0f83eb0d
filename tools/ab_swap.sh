#!/bin/bash
# GPU-box A/B of two builds of libmmfd_hip.so in one call: the in-tree library ("new") and
# tools/_ab/libmmfd_old.so ("old") swapped in place between runs (the torch custom-op library
# resolves libmmfd_hip.so next to itself), interleaved new, old, new, old.
#   AB_CMD="python tools/gemm_bench.py --dtype fp32 --iters 5" bash tools/ab_swap.sh
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
LIB=multimodal-misinformation-detection_amd/libmmfd_hip.so
cp $LIB gpurun_out/_new.so
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then cp tools/_ab/libmmfd_old.so $LIB; else cp gpurun_out/_new.so $LIB; fi
    timeout -k 10 200 $AB_CMD > gpurun_out/ab_$v$r.log 2>&1
    echo "$v$r: $(tail -1 gpurun_out/ab_$v$r.log)"
  done
done
cp gpurun_out/_new.so $LIB
rm -f gpurun_out/_new.so
