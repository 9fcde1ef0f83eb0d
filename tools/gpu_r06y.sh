#!/bin/bash
# diagnostic: x6f epilogue cost with the act / dropout code compiled out of the tile epilogue
# (tools/_ab/lean, results of act products wrong by design) against the tree, x6f_epi_probe shapes
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for r in 1 2; do
  for v in tree lean; do
    unset MMFD_LIB_PATH; [ $v = lean ] && export MMFD_LIB_PATH=tools/_ab/lean/libmmfd_hip.so
    timeout -k 10 300 python tools/x6f_epi_probe.py 2>&1 | grep RESULT | sed "s/^RESULT/$v$r/"
  done
done
