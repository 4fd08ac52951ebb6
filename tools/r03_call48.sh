#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c48
mkdir -p $O
YAVO_LIB=ya_vo_amd/lib/libyavo_nt512.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/pytest_nt512.log 2>&1
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  for v in base nt768 nt512; do
    if [ $v = base ]; then L=ya_vo_amd/lib/libyavo.so; else L=ya_vo_amd/lib/libyavo_$v.so; fi
    YAVO_LIB=$L timeout -k 10 200 $B > $O/ab_${v}_$r.log 2>&1
  done
done
