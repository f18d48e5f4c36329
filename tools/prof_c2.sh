#!/usr/bin/env bash
# Profile the default C2 bench command on the GPU box (run from the repo root under gpurun):
#   rocprofv3 --kernel-trace --stats, then one PMC pass each for FETCH_SIZE, WRITE_SIZE and the SQ
#   VALU counters (separate runs, MI355X_MICROARCH.md HBM section), summarised into
#   gpurun_out/<tag>/pmc.json, then the bench again reading that summary.
# usage: tools/prof_c2.sh TAG [extra bench args...]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
# the profiled runs skip the B = 1 / B = 64 boundary leg (its small launches would dominate the
# per-kernel averages); the final bench line keeps it
args=(--steps 20 --warmup 3 --cpu-budget 0 --latency-frames 0 --boundary-frames 0 --default-frames 0 "$@")
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- python3 bench.py "${args[@]}" > "$out/stats.log" 2>&1
for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVES"; do
  n=${c%% *}
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$out/pmc_$n" -o run -- python3 bench.py "${args[@]}" --steps 2 --warmup 1 > "$out/pmc_$n.log" 2>&1
done
python3 tools/pmc_summary.py "$out/pmc_FETCH_SIZE" "$out/pmc_WRITE_SIZE" "$out/pmc.json" --batch "${BATCH:-2048}" --sq "$out/pmc_SQ_INSTS_VALU" > /dev/null
timeout -k 10 240 python3 -u bench.py "${args[@]}" --latency-frames 20 --cpu-budget 12 --boundary-frames 1024 --default-frames 1024 --pmc "$out/pmc.json" --out "$out/bench.json"
