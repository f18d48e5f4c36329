#!/usr/bin/env bash
# SQ counters per kernel (per launch) for the default C2 bench (run from the repo root under gpurun).
# usage: tools/sq_all.sh TAG [counters...]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; shift
ctr=${*:-SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU}
out=gpurun_out/$tag
mkdir -p "$out"
timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$out/pmc" -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-budget 0 --latency-frames 0 --boundary-frames 0 > "$out/pmc.log" 2>&1
python3 - "$out/pmc/run_counter_collection.csv" <<'PY'
import csv, sys
from collections import defaultdict
acc, n = defaultdict(lambda: defaultdict(float)), defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0]
    if k.startswith("k_"):
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k].add(r["Dispatch_Id"])
cols = sorted({c for d in acc.values() for c in d})
print("%-20s" % "kernel" + "".join("%16s" % c[3:] for c in cols))
for k in sorted(acc, key=lambda k: -acc[k].get("SQ_WAVE_CYCLES", 0)):
    print("%-20s" % k + "".join("%16.4g" % (acc[k][c] / len(n[k])) for c in cols))
PY
