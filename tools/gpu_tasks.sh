#!/bin/bash
# The one GPU-box runner (run through gpurun from the repo root). Each argument is one named task;
# tasks run in order, each under its own time limit (stop at the first
# fault / abort / time limit, keep going after a plain failure such as a red test).
#
#   bash tools/gpu_tasks.sh "<task> [args...]" ["<task> [args...]" ...]
#
# Tasks (LIB=<dir under tools/_ab> runs a task on a variant library built by tools/build_variant.sh):
#   tests [-k EXPR] [FILES...]    pytest -m gpu (default: the whole GPU suite)      -> gpurun_out/tests[_LIB].log
#   smoke                         __graft_entry__.smoke()                           -> gpurun_out/smoke.log
#   bench [bench.py args]         the bench line                                    -> gpurun_out/bench.log
#   ab VARIANT WHAT DTYPE         same-box interleaved A/B of tools/_ab/VARIANT against the in-tree
#                                 library (WHAT: gemm, bench, attn, "gemm bench", ...; DTYPE bf16|fp32)
#                                 -> gpurun_out/ab_VARIANT_WHAT_DTYPE/ + summary.txt
#   gemmbench [args]              tools/gemm_bench.py                               -> gpurun_out/gemmbench.log
#   attnbench [args]              tools/attn_bench.py                               -> gpurun_out/attnbench.log
#   profile TAG DTYPE             kernel trace + FETCH/WRITE passes (tools/profile.sh)
#   mfma TAG DTYPE                MFMA-utilisation pass (tools/pmc_mfma.sh)
#   py SCRIPT [args]              any python tool                                   -> gpurun_out/<script>.log
# Example: bash tools/gpu_tasks.sh "tests -k gemm" "ab ilpnoslp 'gemm bench' bf16"
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out

lib_env() { if [ -n "$LIB" ]; then echo "MMFD_LIB_PATH=tools/_ab/$LIB/libmmfd_hip.so"; fi; }

run() {  # run LIMIT LOG CMD...
  local lim=$1 log=$2; shift 2
  echo "[tasks] $(date +%T) $* > $log" >&2
  ( while sleep 60; do echo "[tasks] $(date +%T) ... $log" >&2; done ) &
  local hb=$!
  timeout -k 10 "$lim" bash -c "$*" > "gpurun_out/$log" 2>&1
  local rc=$?
  kill $hb 2>/dev/null; wait $hb 2>/dev/null
  echo "[tasks] $(date +%T) rc=$rc $log" >&2
  tail -n 3 "gpurun_out/$log" >&2
  case $rc in 124|134|137|139) echo "[tasks] stopping after rc=$rc" >&2; exit $rc ;; esac
  return 0
}

for task in "$@"; do
  eval "set -- $task"
  t=$1; shift
  case $t in
    tests) args=$(printf '%q ' "$@"); run 900 "tests${LIB:+_$LIB}.log" "$(lib_env) python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread ${args:-tests}" ;;
    smoke) run 300 smoke.log "$(lib_env) python -c 'import __graft_entry__ as g; g.smoke()'" ;;
    bench) run 400 bench.log "$(lib_env) python bench.py $*" ;;
    ab)
      v=$1; what=$2; dt=${3:-bf16}
      rm -rf gpurun_out/lib_ab
      run 1100 "ab_${v}.log" "AB_WHAT='$what' AB_DTYPE=$dt AB_LIB=tools/_ab/$v/libmmfd_hip.so bash tools/lib_ab.sh"
      d="gpurun_out/ab_${v}_${what// /_}_$dt"
      rm -rf "$d"; mv gpurun_out/lib_ab "$d"
      python3 tools/lib_ab_summary.py "$d" > "$d/summary.txt" 2>&1; cat "$d/summary.txt" >&2 ;;
    gemmbench) run 400 gemmbench.log "$(lib_env) python tools/gemm_bench.py $*" ;;
    attnbench) run 300 attnbench.log "$(lib_env) python tools/attn_bench.py $*" ;;
    profile) run 1100 "profile_$1.log" "BENCH_ARGS='--precision $2 --no-bf16' bash tools/profile.sh $1_$2" ;;
    mfma) run 400 "mfma_$1.log" "BENCH_ARGS='--precision $2 --no-bf16' bash tools/pmc_mfma.sh $1_$2 && python3 tools/pmc_mfma_summary.py gpurun_out/prof_$1_$2 $1_$2" ;;
    py) s=$1; shift; run 600 "$(basename "$s" .py).log" "$(lib_env) python $s $*" ;;
    *) echo "unknown task $t" >&2; exit 2 ;;
  esac
done
exit 0
