#!/bin/bash
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_evidence_gpu.py -k "stem or resnet50_full" > gpurun_out/r06c_tests.log 2>&1 || { tail -30 gpurun_out/r06c_tests.log; exit 1; }
tail -2 gpurun_out/r06c_tests.log
bash tools/prof_extract.sh
