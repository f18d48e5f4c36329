#!/usr/bin/env bash
# k_ransac launch times (kernel trace) at several RANSAC split counts, C2 B = 1024 (under gpurun).
set -euo pipefail
tag=${1:-r3rs4}
for s in ${SPLITS:-1 2 4 8 16}; do
    KERNELS=rectify_pyramid,detect,select,describe,match,match_refine,pose,pose PROBE_ARGS="--splits $s" \
        tools/pose_split.sh "$tag/s$s" > /dev/null
    python3 - "gpurun_out/$tag/s$s/stats/run_kernel_trace.csv" "$s" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].startswith(("k_ransac", "k_refine"))]
for k in ("k_ransac", "k_refine"):
    print("splits", sys.argv[2], k, [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000, 1) for r in rows if r["Kernel_Name"].startswith(k)])
PY
done
