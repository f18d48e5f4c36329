#!/usr/bin/env bash
# k_ransac launch times for experiment libraries (TSLAM_LIBRARY), C2 B = 1024 (under gpurun).
set -euo pipefail
tag=$1; shift
for lib in "" "$@"; do
    if [ -n "$lib" ]; then export TSLAM_LIBRARY=$PWD/$lib; else unset TSLAM_LIBRARY; fi
    n=$(basename "${lib:-intree}" .so)
    KERNELS=rectify_pyramid,detect,select,describe,match,match_refine,pose,pose tools/pose_split.sh "$tag/$n" > /dev/null
    python3 - "gpurun_out/$tag/$n/stats/run_kernel_trace.csv" "$n" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kernel_Name"].startswith(("k_ransac", "k_refine"))]
for k in ("k_ransac", "k_refine"): print(sys.argv[2], k, [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000, 1) for r in rows if r["Kernel_Name"].startswith(k)])
PY
done
