#!/bin/bash
# Build an A/B variant of libmmfd_hip.so (+ a copy of the in-tree libmmfd_torch.so beside it) into
# tools/_ab/<name>/:   bash tools/build_variant.sh <name> [git-rev|-] [extra hipcc flags...]
# VARIANT_SCHED overrides the Makefile's gemm.hip scheduler flag (VARIANT_SCHED= for the default scheduler).
# With a git rev, the csrc sources and include/mmfd.h come from that revision, else the working tree.
set -e
NAME=$1; REV=${2:--}; shift 2 || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/multimodal-misinformation-detection_amd/csrc
OUT=$ROOT/tools/_ab/$NAME
rm -rf $OUT && mkdir -p $OUT/pkg/csrc $OUT/include $OUT/o
for f in $(cd $SRC && ls *.hip *.h); do
  if [ "$REV" = "-" ]; then cp $SRC/$f $OUT/pkg/csrc/$f
  else git -C $ROOT show $REV:multimodal-misinformation-detection_amd/csrc/$f > $OUT/pkg/csrc/$f; fi
done
if [ "$REV" = "-" ]; then cp $ROOT/include/mmfd.h $OUT/include/; else git -C $ROOT show $REV:include/mmfd.h > $OUT/include/mmfd.h; fi
for f in $(cd $OUT/pkg/csrc && ls *.hip); do
  extra=""; [ $f = gemm_x6f.hip ] && extra="-fno-slp-vectorize"; [ $f = gemm.hip ] && extra="${VARIANT_SCHED--mllvm -amdgpu-sched-strategy=max-ilp}"
  (/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form $extra "$@" -c $OUT/pkg/csrc/$f -o $OUT/o/$f.o || echo FAIL $f) &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/libmmfd_hip.so $OUT/o/*.o
cp $ROOT/multimodal-misinformation-detection_amd/libmmfd_torch.so $OUT/
rm -rf $OUT/o $OUT/pkg $OUT/include
ls -la $OUT
