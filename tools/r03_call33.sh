#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03c33
mkdir -p $O
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  for v in 1024 512 256; do
    YAVO_BUILD_NT=$v timeout -k 10 200 $B > $O/ab_b${v}_$r.log 2>&1
  done
done
