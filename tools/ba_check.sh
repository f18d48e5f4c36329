#!/usr/bin/env bash
# BA kernel timing (rocprofv3 stats over tools/ba_probe.py) + the BA GPU tests (run under gpurun).
set -euo pipefail
tag=${1:-r3ba}
out=gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- python3 tools/ba_probe.py > "$out/probe.log" 2>&1
grep "local BA\|front end" "$out/probe.log"
python3 - "$out/stats/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_ba_" in r["Name"]:
        print("%-18s calls %4s avg %7.2f us" % (r["Name"].split("(")[0], r["Calls"], float(r["AverageNs"]) / 1000))
PY
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ba.py tests/test_gpu_ba_rig.py -x -q --timeout 200 --timeout-method thread > "$out/tests.log" 2>&1
tail -2 "$out/tests.log"
