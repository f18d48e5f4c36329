#!/usr/bin/env bash
# Quick GPU check (run from the repo root under gpurun): the given pytest files, then the default
# C2 bench without the CPU / boundary legs; results under gpurun_out/<tag>/.
# usage: tools/quick_c2.sh TAG [pytest targets...]
set -euo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
if [ $# -gt 0 ]; then
  timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread "$@" > "$out/tests.log" 2>&1
  tail -1 "$out/tests.log"
fi
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --cpu-budget 0 --latency-frames 0 --boundary-frames 0 \
  --out "$out/bench.json" > "$out/bench.log" 2>&1
python3 - "$out/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value %.0f  ms/step %.3f" % (d["value"], d["ms_per_step"]))
for k, v in (d.get("kernel_us_isolated") or d.get("per_kernel_us_isolated") or {}).items():
    print("  %-16s %8.1f us" % (k, v))
PY
