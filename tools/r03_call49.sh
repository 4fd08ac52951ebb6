#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c49
mkdir -p $O
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  for v in base w3 w3pad; do
    L=ya_vo_amd/lib/libyavo.so; P=0
    [ $v != base ] && L=ya_vo_amd/lib/libyavo_w3.so
    [ $v = w3pad ] && P=40000
    YAVO_LM_LDS_PAD=$P YAVO_LIB=$L timeout -k 10 200 $B > $O/ab_${v}_$r.log 2>&1
  done
done
