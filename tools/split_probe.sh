#!/usr/bin/env bash
# C2 bench with the front and back kernels on disjoint CU sets (--back-cu N --split-cu 1)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r5r
args="--steps 20 --warmup 3 --cpu-budget 0 --latency-frames 0 --boundary-frames 0 --default-frames 0"
for n in 0 32 64 96 128; do
  if [ $n = 0 ]; then extra=""; else extra="--back-cu $n --split-cu 1"; fi
  timeout -k 10 200 python3 -u bench.py $args $extra --out gpurun_out/r5r/b$n.json > gpurun_out/r5r/b$n.log 2>&1
  rc=$?
  echo "== back $n rc=$rc $(python3 -c "import json;d=json.load(open('gpurun_out/r5r/b$n.json'));print(round(d['value']), d['ms_per_step'])" 2>/dev/null)"
  case $rc in 0) ;; *) exit $rc ;; esac
done
