#!/usr/bin/env bash
# Profile the C4 bench (1280x800, K=4000, 10-keyframe local BA) on the GPU box:
#   rocprofv3 --kernel-trace --stats, one PMC pass for the FP64 MFMA / VALU counters of the BA
#   Schur kernel, then the bench line itself.   usage: tools/prof_c4.sh TAG [extra bench args...]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
args=(--config c4 --steps 10 --warmup 2 --cpu-budget 0 --latency-frames 0 --boundary-frames 0 "$@")
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o run -- python3 bench.py "${args[@]}" > "$out/stats.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU SQ_WAVES --output-format csv -d "$out/pmc_mfma" -o run -- python3 bench.py "${args[@]}" --steps 2 --warmup 1 > "$out/pmc_mfma.log" 2>&1
timeout -k 10 300 python3 -u bench.py "${args[@]}" --out "$out/bench.json"
