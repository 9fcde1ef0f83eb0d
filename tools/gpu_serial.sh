#!/bin/bash
# serialized-step kernel traces of both legs (tools/serial_step.py), summarized by tools/step_breakdown.py
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=${1:-r06}
for prec in ${PRECS:-bf16 fp32}; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/serial_$prec -o run --output-format csv -- \
    python3 tools/serial_step.py $prec 4 > gpurun_out/${TAG}_serial_$prec.log 2>&1 || { tail -20 gpurun_out/${TAG}_serial_$prec.log; exit 1; }
  grep serialized gpurun_out/${TAG}_serial_$prec.log
  python3 tools/step_breakdown.py gpurun_out/serial_$prec/run_kernel_stats.csv | tail -12
done
