#!/bin/bash
# The LM in 128-thread workgroups under each overlap mode at B = 2048 (same box)
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c62
mkdir -p $O
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  timeout -k 10 200 $B > $O/base_$r.log 2>&1
  YAVO_LM_THREADS=128 timeout -k 10 200 $B --overlap-mode 4 > $O/lm128_ov4_$r.log 2>&1
  YAVO_LM_THREADS=128 timeout -k 10 200 $B --overlap-mode 3 > $O/lm128_ov3_$r.log 2>&1
  YAVO_LM_THREADS=128 YAVO_LM_GRID=1024 timeout -k 10 200 $B > $O/lm128_g1024_$r.log 2>&1
done
