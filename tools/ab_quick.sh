#!/usr/bin/env bash
# Quick A/B of library builds (run from the repo root under gpurun): optional parity file run
# against each library, then the default C2 bench's step and isolated kernel times.
# usage: PARITY=tests/test_gpu_parity.py tools/ab_quick.sh TAG lib1.so [lib2.so ...]
set -euo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
i=0
for lib in "$@"; do
  i=$((i + 1))
  if [ -n "$lib" ]; then export TSLAM_LIBRARY=$PWD/$lib; else unset TSLAM_LIBRARY; fi
  if [ -n "${PARITY:-}" ]; then
    timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread $PARITY > "$out/tests_$i.log" 2>&1 \
      || { echo "[$lib] parity FAILED"; tail -40 "$out/tests_$i.log"; exit 1; }
    echo "[$lib] $(tail -1 "$out/tests_$i.log")"
  fi
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --cpu-budget 0 --latency-frames 0 --boundary-frames 0 \
    ${BENCH_ARGS:-} --out "$out/bench_$i.json" > "$out/bench_$i.log" 2>&1
  python3 - "$out/bench_$i.json" "$lib" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
iso = d.get("per_kernel_us_isolated") or {}
print("[%s] value %.0f  ms/step %.3f  " % (sys.argv[2] or "in-tree", d["value"], d["ms_per_step"])
      + " ".join("%s %.0f" % (k, v) for k, v in iso.items()))
PY
done
