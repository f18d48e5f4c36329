#!/usr/bin/env bash
# One gpurun session: each GPU step under its own time limit; stop at the first crash/timeout
# (exit 124/134/137/139 or signal) but continue past ordinary test failures (pytest exit 1).
# usage: tools/gpu_session.sh TAG "step1 cmd" "step2 cmd" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
mkdir -p gpurun_out
i=0
for cmd in "$@"; do
  i=$((i+1))
  log="gpurun_out/${tag}_step${i}.log"
  echo "== step $i: $cmd" | tee -a "gpurun_out/${tag}_summary.txt"
  start=$(date +%s)
  bash -c "$cmd" > "$log" 2>&1
  rc=$?
  echo "   rc=$rc $(( $(date +%s) - start ))s log=$log" | tee -a "gpurun_out/${tag}_summary.txt"
  tail -n 5 "$log"
  case $rc in
    0|1|2|5) ;;                 # pass / test failures / usage / no tests
    *) echo "stopping after rc=$rc"; exit $rc ;;
  esac
done
