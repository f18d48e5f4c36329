#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r5az; mkdir -p $out
for rep in 1 2; do
for r in 32 64 96 128; do
  timeout -k 10 200 python3 -u bench.py --config c4 --steps 10 --warmup 3 --cpu-budget 0 --latency-frames 0 --boundary-frames 0 --default-frames 0 --front-cu-reserve $r --out $out/c4_r${r}_$rep.json > $out/c4_r${r}_$rep.log 2>&1 || exit 1
  python3 -c "import json;d=json.load(open('$out/c4_r${r}_$rep.json'));print('reserve $r rep $rep', round(d['value']), round(d['ms_per_step'],3))"
done
done
