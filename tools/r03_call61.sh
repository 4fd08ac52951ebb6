#!/bin/bash
# Larger steps (B = 3072 / 4096) and 128-thread LM workgroups at B = 2048 (same box)
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c61
mkdir -p $O
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  timeout -k 10 200 $B > $O/b2048_$r.log 2>&1
  timeout -k 10 300 $B --frames 3072 > $O/b3072_$r.log 2>&1
  timeout -k 10 300 $B --frames 4096 > $O/b4096_$r.log 2>&1
  YAVO_LM_THREADS=128 timeout -k 10 200 $B > $O/lm128_$r.log 2>&1
done
