#!/usr/bin/env bash
# A/B of pipeline schedules (bench flags) on the GPU box, with a kernel trace of each.
# usage: tools/sched_ab.sh TAG "flags A" "flags B" ...
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
args=(--steps 20 --warmup 3 --cpu-budget 0 --latency-frames 0 --boundary-frames 0)
i=0
for flags in "$@"; do
  i=$((i + 1))
  timeout -k 10 200 python3 -u bench.py "${args[@]}" $flags --out "$out/bench_$i.json" > "$out/bench_$i.log" 2>&1
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$out/prof_$i" -o run -- python3 bench.py "${args[@]}" $flags --steps 6 > "$out/prof_$i.log" 2>&1
  python3 - "$out/bench_$i.json" "$flags" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("[%s] value %.0f  ms/step %.3f" % (sys.argv[2], d["value"], d["ms_per_step"]))
PY
done
