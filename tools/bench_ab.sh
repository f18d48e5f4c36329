#!/usr/bin/env bash
# C2 bench A/B of library builds on the GPU box (run from the repo root under gpurun), each run
# twice, interleaved: tools/bench_ab.sh TAG lib1.so [lib2.so ...]   ("" = the in-tree library)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
args=(--steps 20 --warmup 3 --cpu-budget 0 --latency-frames 0 --boundary-frames 0 --default-frames 0 ${BENCH_ARGS:-})
for rep in 1 2; do
  i=0
  for lib in "$@"; do
    i=$((i + 1))
    if [ -n "$lib" ]; then export TSLAM_LIBRARY=$PWD/$lib; else unset TSLAM_LIBRARY; fi
    timeout -k 10 200 python3 -u bench.py "${args[@]}" --out "$out/bench_${i}_$rep.json" > "$out/bench_${i}_$rep.log" 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "[$lib] rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('[%s] rep %s value %.0f ms/step %.3f' % (sys.argv[2] or 'in-tree', sys.argv[3], d['value'], d['ms_per_step']))" "$out/bench_${i}_$rep.json" "$lib" "$rep"
  done
done
