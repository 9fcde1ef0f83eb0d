#!/bin/bash
# full GPU suite + smoke + default bench on the current tree (round 6); logs under gpurun_out/
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
TAG=${1:-r06}
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputests.log 2>&1 || { tail -40 gpurun_out/${TAG}_gputests.log; exit 1; }
tail -3 gpurun_out/${TAG}_gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1])
print('fp32', d['value'], 'frac', d['roofline']['frac'], 'bf16', d.get('bf16', {}).get('value'), 'cpu', d.get('cpu_baseline', {}).get('value'))"
