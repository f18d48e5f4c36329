#!/usr/bin/env bash
# Isolated per-kernel times of the back end (pose stage split into corr / p3p / ransac / refine)
# at B = 1024: rocprofv3 kernel stats over tools/kernel_probe.py (run under gpurun).
set -euo pipefail
tag=${1:-r3ps}
out=gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- python3 tools/kernel_probe.py --batch 1024 --kernels ${KERNELS:-rectify_pyramid,detect,select,describe,match,match_refine,pose,pose,pose} ${PROBE_ARGS:-} > "$out/probe.log" 2>&1
grep " us" "$out/probe.log" || true
python3 - "$out/stats/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if r["Name"].startswith("k_"):
        print("%-22s calls %4s avg %8.1f us" % (r["Name"].split("(")[0], r["Calls"], float(r["AverageNs"]) / 1000))
PY
