#!/bin/bash
# Workgroup widths at B = 2048: top-K 1024 threads, BRIEF 768 threads (same box)
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c63
mkdir -p $O
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  timeout -k 10 200 $B > $O/base_$r.log 2>&1
  YAVO_LIB=ya_vo_amd/lib/libyavo_tk1024.so timeout -k 10 200 $B > $O/tk1024_$r.log 2>&1
  YAVO_LIB=ya_vo_amd/lib/libyavo_br768.so timeout -k 10 200 $B > $O/br768_$r.log 2>&1
done
