#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03c32
mkdir -p $O
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  for v in base t512 t256; do
    if [ $v = base ]; then L=ya_vo_amd/lib/libyavo.so; else L=ya_vo_amd/lib/libyavo_$v.so; fi
    YAVO_LIB=$L timeout -k 10 200 $B > $O/ab_${v}_$r.log 2>&1
  done
done
cd /tmp
for v in base t512; do
  if [ $v = base ]; then L=$GRAFT_REPO_ROOT/ya_vo_amd/lib/libyavo.so; else L=$GRAFT_REPO_ROOT/ya_vo_amd/lib/libyavo_$v.so; fi
  YAVO_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_$v -o out -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0 --steps 20 > $GRAFT_REPO_ROOT/$O/prof_$v.log 2>&1
done
