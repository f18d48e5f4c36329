#!/usr/bin/env bash
# A/B of library builds on the GPU box (run from the repo root under gpurun): for each library,
# the C2 bench (value, isolated kernel times) and a rocprofv3 kernel-stats pass.
# usage: tools/ab_libs.sh TAG lib1.so [lib2.so ...]   ("" = the in-tree library)
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
args=(--steps 20 --warmup 3 --cpu-budget 0 --latency-frames 0 --boundary-frames 0)
i=0
for lib in "$@"; do
  i=$((i + 1))
  if [ -n "$lib" ]; then export TSLAM_LIBRARY=$PWD/$lib; else unset TSLAM_LIBRARY; fi
  timeout -k 10 200 python3 -u bench.py "${args[@]}" --out "$out/bench_$i.json" > "$out/bench_$i.log" 2>&1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_$i" -o run -- python3 bench.py "${args[@]}" --steps 10 > "$out/prof_$i.log" 2>&1
  python3 - "$out/bench_$i.json" "$out/prof_$i/run_kernel_stats.csv" "$lib" <<'PY'
import csv, json, sys
d = json.load(open(sys.argv[1]))
print("[%s] value %.0f  ms/step %.3f" % (sys.argv[3] or "in-tree", d["value"], d["ms_per_step"]))
rows = list(csv.DictReader(open(sys.argv[2])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print("   %-28s %9.1f us avg  x%s" % (r["Name"][:28], float(r["AverageNs"]) / 1e3, r["Calls"]))
PY
done
