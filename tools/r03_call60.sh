#!/bin/bash
# Co-residency beside the pose LM at B = 2048: top-K in 256-thread workgroups (one wave per SIMD fits beside two LM
# waves) with the LM's grid at one workgroup per problem / 1024 / 512 (same box)
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c60
mkdir -p $O
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
T=ya_vo_amd/lib/libyavo_tk256.so
for r in 1 2; do
  timeout -k 10 200 $B > $O/base_$r.log 2>&1
  YAVO_LIB=$T timeout -k 10 200 $B > $O/tk256_$r.log 2>&1
  YAVO_LIB=$T YAVO_LM_GRID=1024 timeout -k 10 200 $B > $O/tk256_g1024_$r.log 2>&1
  YAVO_LIB=$T YAVO_LM_GRID=512 timeout -k 10 200 $B > $O/tk256_g512_$r.log 2>&1
done
