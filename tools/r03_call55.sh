#!/bin/bash
# Re-tune at the new default B = 2048: LDS-resident LM form, overlap modes 3 / 4, LM grid 512 / 1024 (same box)
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c55
mkdir -p $O
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  timeout -k 10 200 $B > $O/base_$r.log 2>&1
  YAVO_LM_RESIDENT=1 timeout -k 10 200 $B > $O/resident_$r.log 2>&1
  timeout -k 10 200 $B --overlap-mode 3 > $O/ov3_$r.log 2>&1
  timeout -k 10 200 $B --overlap-mode 4 > $O/ov4_$r.log 2>&1
  YAVO_LM_GRID=1024 timeout -k 10 200 $B > $O/grid1024_$r.log 2>&1
  YAVO_LM_GRID=512 timeout -k 10 200 $B > $O/grid512_$r.log 2>&1
done
for r in 1 2; do
  YAVO_LIB=ya_vo_amd/lib/libyavo_fzu8.so timeout -k 10 200 $B > $O/fzu8_$r.log 2>&1
  YAVO_LIB=ya_vo_amd/lib/libyavo_fzu2.so timeout -k 10 200 $B > $O/fzu2_$r.log 2>&1
done
