#!/bin/bash
# Edge build placement at B = 2048: workgroup width (its 120 VGPRs x 16 waves leave detect one wave per SIMD on the
# CU), stream priority, and the synchronous build (same box)
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c65
mkdir -p $O
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  timeout -k 10 200 $B > $O/base_$r.log 2>&1
  YAVO_BUILD_NT=512 timeout -k 10 200 $B > $O/nt512_$r.log 2>&1
  YAVO_BUILD_NT=256 timeout -k 10 200 $B > $O/nt256_$r.log 2>&1
  YAVO_BUILD_PRIO=2 timeout -k 10 200 $B > $O/prio_low_$r.log 2>&1
  YAVO_BUILD_ASYNC=0 timeout -k 10 200 $B > $O/sync_$r.log 2>&1
done
