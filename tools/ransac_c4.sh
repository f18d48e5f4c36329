#!/usr/bin/env bash
# Pose-stage kernel times at the C4 shape (1280x800, K = 4000, B = 50) over RANSAC split counts.
set -euo pipefail
tag=${1:-r3c4rs}
for s in ${SPLITS:-2 4 8 16}; do
    KERNELS=rectify_pyramid,detect,select,describe,match,match_refine,pose,pose \
        PROBE_ARGS="--splits $s --width 1280 --height 800 --features 4000 --batch 50" tools/pose_split.sh "$tag/s$s" > /dev/null
    python3 - "gpurun_out/$tag/s$s/stats/run_kernel_trace.csv" "$s" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1]))]
for k in ("k_ransac", "k_refine", "k_p3p", "k_corr"):
    print("splits", sys.argv[2], k, [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000, 1) for r in rows if r["Kernel_Name"].startswith(k)][-2:])
PY
done
