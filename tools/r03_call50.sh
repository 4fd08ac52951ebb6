#!/bin/bash
# GPU suite at the working tree (RCCL world-1 exchange test included), matcher pipelining forms' parity, then a
# same-box A/B: HEAD's triangulation (libyavo_base.so) vs the copysign rotation, and the FP4 matcher forms
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c50
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -rf --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
for f in fp4p fp4p2 fp4p2w3; do
  YAVO_MATCH_FORM=$f timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "match" > $O/pytest_match_$f.log 2>&1
done
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  YAVO_LIB=ya_vo_amd/lib/libyavo_base.so timeout -k 10 200 $B > $O/ab_base_$r.log 2>&1
  timeout -k 10 200 $B > $O/ab_new_$r.log 2>&1
  for f in fp4p fp4p2 fp4p2w3; do
    YAVO_MATCH_FORM=$f timeout -k 10 200 $B > $O/ab_${f}_$r.log 2>&1
  done
done
