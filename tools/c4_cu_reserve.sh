#!/usr/bin/env bash
set -euo pipefail
out=gpurun_out/r3y; mkdir -p $out
for r in 0 16 32 64; do
  timeout -k 10 200 python3 -u bench.py --config c4 --steps 10 --warmup 2 --cpu-budget 0 --latency-frames 0 --boundary-frames 0 --front-cu-reserve $r --out $out/c4_r$r.json > $out/c4_r$r.log 2>&1
  python3 -c "import json;d=json.load(open('$out/c4_r$r.json'));print('reserve $r', round(d['value']), round(d['ms_per_step'],3), d['per_kernel_us_per_batch'])"
done
