#!/bin/bash
# The full default bench (every leg: CPU baseline, pose check, end-to-end, PNG, LoopHandler) at B = 2048 and at
# B = 1024, with the wall time of each run
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c52
mkdir -p $O
for f in 2048 1024; do
  t0=$SECONDS
  timeout -k 10 900 python bench.py --frames $f > $O/bench_full_$f.log 2> $O/bench_full_$f.err
  echo "frames $f wall_s $((SECONDS - t0))" >> $O/walls.txt
done
