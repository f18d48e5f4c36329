set -euo pipefail
mkdir -p gpurun_out/r3c
for v in v2 v3; do
  TSLAM_LIBRARY=$PWD/variants/$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r3c/tests_$v.log 2>&1 || { echo "$v parity FAILED"; tail -30 gpurun_out/r3c/tests_$v.log; exit 1; }
  tail -1 gpurun_out/r3c/tests_$v.log
done
tools/ab_libs.sh r3c variants/v0.so variants/v1.so variants/v2.so variants/v3.so
