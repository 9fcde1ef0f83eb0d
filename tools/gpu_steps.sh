#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step that faulted,
# aborted or timed out (exit 124 / 134 / 137 / 139 or a negative-signal status), keep going after a
# plain failure (a red test). Usage: tools/gpu_steps.sh "<limit_s> <log> <command...>" ...
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for step in "$@"; do
  read -r lim log cmd <<< "$step"
  echo "[steps] $(date +%T) $cmd > $log" >&2
  # heartbeat: a long step (pytest prints only at a test's end) must not look hung
  ( while sleep 60; do echo "[steps] $(date +%T) ... $log" >&2; done ) &
  hb=$!
  timeout -k 10 "$lim" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  kill $hb 2>/dev/null; wait $hb 2>/dev/null
  echo "[steps] $(date +%T) rc=$rc $log" >&2
  case $rc in 124|134|137|139) echo "[steps] stopping after rc=$rc" >&2; exit $rc ;; esac
done
exit 0
