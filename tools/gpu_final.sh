#!/bin/bash
# round-6 closing profile set: fp32 and bf16 kernel traces + HBM passes (tools/profile.sh), MFMA
# counters (tools/pmc_mfma.sh), config-5 extract A/B (implicit conv vs MMFD_CONV_IM2COL=1) on one box
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
T=${1:-r06}
STEPS=5 BENCH_ARGS="--precision fp32 --no-bf16" bash tools/profile.sh ${T}_fp32 || exit 1
echo fp32 profile done
STEPS=5 BENCH_ARGS="--precision bf16" bash tools/profile.sh ${T}_bf16 || exit 1
echo bf16 profile done
BENCH_ARGS="--precision fp32 --no-bf16" bash tools/pmc_mfma.sh ${T}_fp32 || exit 1
BENCH_ARGS="--precision bf16" bash tools/pmc_mfma.sh ${T}_bf16 || exit 1
python3 tools/pmc_mfma_summary.py gpurun_out/prof_${T}_fp32 ${T}_fp32 && python3 tools/pmc_mfma_summary.py gpurun_out/prof_${T}_bf16 ${T}_bf16 || exit 1
echo mfma done
for arm in 0 1 0 1; do
  MMFD_CONV_IM2COL=$arm timeout -k 10 400 python3 bench.py --workload extract --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/${T}_extract_im2col$arm.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/${T}_extract_im2col$arm.json').read().strip().splitlines()[-1]); print('im2col=$arm', d['value'], d['images_per_s_per_gpu'], d['texts_per_s_per_gpu'], d['bf16']['images_per_s_per_gpu'])"
done
