#!/usr/bin/env bash
# Round-3 measurement pass (run from the repo root under gpurun): C2 stats + PMC + bench (with the
# CPU baseline and host boundary), the sharded rehearsal's phases at 2 / 4 / 8 ranks, and the
# C3 / C4 / C5 bench lines.  Every GPU step has its own time limit; stop at the first failure.
set -euo pipefail
tag=${1:-r3q}
out=gpurun_out/$tag
mkdir -p "$out"
tools/prof_c2.sh "$tag" > "$out/prof_c2.log" 2>&1
for w in 2 4 8; do
  timeout -k 10 240 python3 -u tools/shard_probe.py --world $w --out "$out/shard_w$w.json" > "$out/shard_w$w.log" 2>&1
done
for cfg in c3 c4 c5; do
  timeout -k 10 300 python3 -u bench.py --config $cfg --steps 10 --warmup 2 --cpu-budget 0 --boundary-frames 0 \
    --out "$out/bench_$cfg.json" > "$out/bench_$cfg.log" 2>&1
done
echo done
