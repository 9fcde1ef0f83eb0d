#!/bin/bash
# A/B build of the four-wave GEMM's schedule: regenerates gemm_g4.hip with G4_READ_AT / G4_DMA_AT
# (positions of the fragment reads / DMA pieces among each part's MFMAs) into tools/_ab/<name>/ and
# links it with the in-tree objects of everything else:  bash tools/g4_variant.sh <name> <read_at> <dma_at>
set -e
NAME=$1; RA=$2; DA=$3
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CSRC=$ROOT/multimodal-misinformation-detection_amd/csrc
OUT=$ROOT/tools/_ab/$NAME
rm -rf $OUT && mkdir -p $OUT
G4_READ_AT=$RA G4_DMA_AT=$DA G4_OUT=$CSRC/gemm_g4_v_$NAME.hip python3 $ROOT/tools/gen_gemm_g4.py > /dev/null
(cd $CSRC && /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form \
   -c gemm_g4_v_$NAME.hip -o $OUT/gemm_g4.o)
rm -f $CSRC/gemm_g4_v_$NAME.hip
objs=$(ls $CSRC/build/*.o | grep -v '/gemm_g4.o$' | grep -v torch_ops)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/libmmfd_hip.so $objs $OUT/gemm_g4.o
cp $ROOT/multimodal-misinformation-detection_amd/libmmfd_torch.so $OUT/
rm -f $OUT/gemm_g4.o
echo built $OUT
