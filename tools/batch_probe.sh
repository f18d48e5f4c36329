#!/usr/bin/env bash
# kernel_probe of the front kernels at several batch sizes (per-frame cost vs cache residency)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5q
for b in 64 128 256 512 1024; do
  timeout -k 10 120 python3 -u tools/kernel_probe.py --batch $b --kernels rectify_pyramid,detect,detect,select,describe,describe,describe > gpurun_out/r5q/b$b.log 2>&1
  rc=$?
  echo "== batch $b rc=$rc"; grep -E "^(rectify_pyramid|detect|select|describe) " gpurun_out/r5q/b$b.log | tr '\n' ' '; echo
  case $rc in 0) ;; *) exit $rc ;; esac
done
