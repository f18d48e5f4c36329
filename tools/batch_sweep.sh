#!/usr/bin/env bash
set -euo pipefail
mkdir -p gpurun_out/r3bs
for b in 1024 1536 2048; do
  timeout -k 10 200 python3 -u bench.py --batch $b --steps 10 --warmup 3 --cpu-budget 0 --latency-frames 0 --boundary-frames 0 --out gpurun_out/r3bs/b$b.json > gpurun_out/r3bs/b$b.log 2>&1
  python3 -c "import json;d=json.load(open('gpurun_out/r3bs/b$b.json'));print('B=$b', round(d['value']), round(d['ms_per_step'],3))"
done
