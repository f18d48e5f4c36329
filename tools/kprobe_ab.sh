#!/usr/bin/env bash
# k_match A/B: kernel_probe per library
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${TAG}; mkdir -p $out
for lib in "" ${LIBS:-}; do
  if [ -n "$lib" ]; then export TSLAM_LIBRARY=$PWD/$lib; else unset TSLAM_LIBRARY; fi
  n=$(basename "${lib:-intree}" .so)
  timeout -k 10 120 python3 -u tools/kernel_probe.py --batch 1024 --kernels ${KERNELS:-match,match,match,match_refine,match_refine} > $out/$n.log 2>&1
  rc=$?
  echo "== $n rc=$rc"; grep -E "^[a-z_]+ +[0-9.]+ us" $out/$n.log | tr '\n' ' '; echo
  case $rc in 0) ;; *) exit $rc ;; esac
done
