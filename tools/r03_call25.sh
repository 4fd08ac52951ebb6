#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03c25
mkdir -p $O
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  for m in 1 3 4; do
    timeout -k 10 200 $B --overlap-mode $m > $O/mode${m}_$r.log 2>&1
  done
done
