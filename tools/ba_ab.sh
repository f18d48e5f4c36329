#!/usr/bin/env bash
# BA per-keyframe A/B of library builds (tools/ba_probe.py), each run twice, interleaved:
#   tools/ba_ab.sh TAG lib1.so [lib2.so ...]   ("" = the in-tree library)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
for rep in 1 2; do
  i=0
  for lib in "$@"; do
    i=$((i + 1))
    if [ -n "$lib" ]; then export TSLAM_LIBRARY=$PWD/$lib; else unset TSLAM_LIBRARY; fi
    timeout -k 10 120 python3 -u tools/ba_probe.py > "$out/ba_${i}_$rep.log" 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "[$lib] rc=$rc"; exit $rc; }
    echo "[${lib:-in-tree}] rep $rep $(grep 'local BA' $out/ba_${i}_$rep.log)"
  done
done
