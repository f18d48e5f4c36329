#!/usr/bin/env bash
# SQ instruction counters per kernel for each library build (run from the repo root under gpurun).
# usage: tools/pmc_libs.sh TAG KERNEL_SUBSTRING lib1.so [lib2.so ...]   ("" = the in-tree library)
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; kern=$2; shift 2
out=gpurun_out/$tag
mkdir -p "$out"
args=(--steps 2 --warmup 1 --cpu-budget 0 --latency-frames 0 --boundary-frames 0)
i=0
for lib in "$@"; do
  i=$((i + 1))
  if [ -n "$lib" ]; then export TSLAM_LIBRARY=$PWD/$lib; else unset TSLAM_LIBRARY; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    --output-format csv -d "$out/pmc_$i" -o run -- python3 bench.py "${args[@]}" > "$out/pmc_$i.log" 2>&1
  python3 - "$out/pmc_$i/run_counter_collection.csv" "$kern" "$lib" <<'PY'
import csv, sys
from collections import defaultdict
acc, n = defaultdict(float), defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Kernel_Name"]:
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]].add(r["Dispatch_Id"])
print("[%s] %s" % (sys.argv[3] or "in-tree", sys.argv[2]))
for k in sorted(acc):
    print("   %-20s %14.0f per launch" % (k, acc[k] / max(1, len(n[k]))))
PY
done
