#!/bin/bash
# Quick A/B variant of libmmfd_hip.so that recompiles only the GEMM translation units (gemm.hip,
# gemm_f32out.hip, gemm_x6f.hip) with extra flags and links them with the in-tree objects of every
# other file: bash tools/build_gemm_variant.sh <name> [extra hipcc flags...]  -> tools/_ab/<name>/
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/multimodal-misinformation-detection_amd/csrc
OUT=$ROOT/tools/_ab/$NAME
make -C $SRC -s >/dev/null
rm -rf $OUT && mkdir -p $OUT/o
BASE="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form"
ILP="-mllvm -amdgpu-sched-strategy=max-ilp"
/opt/rocm/bin/hipcc $BASE $ILP "$@" -c $SRC/gemm.hip -o $OUT/o/gemm.o &
/opt/rocm/bin/hipcc $BASE $ILP -fno-slp-vectorize "$@" -c $SRC/gemm_f32out.hip -o $OUT/o/gemm_f32out.o &
/opt/rocm/bin/hipcc $BASE -fno-slp-vectorize "$@" -c $SRC/gemm_x6f.hip -o $OUT/o/gemm_x6f.o &
wait
for o in $SRC/build/*.o; do
  b=$(basename $o); case $b in gemm.o|gemm_f32out.o|gemm_x6f.o|torch_ops.o) ;; *) cp $o $OUT/o/ ;; esac
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/libmmfd_hip.so $OUT/o/*.o
cp $ROOT/multimodal-misinformation-detection_amd/libmmfd_torch.so $OUT/
rm -rf $OUT/o
ls -la $OUT/libmmfd_hip.so
