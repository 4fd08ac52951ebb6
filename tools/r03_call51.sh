#!/bin/bash
# Same-box A/B: the headline bench at B = 1024 with / without the 1-rank RCCL exchange, and B = 1536 / 2048
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c51
mkdir -p $O
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  timeout -k 10 200 $B > $O/b1024_$r.log 2>&1
  timeout -k 10 200 $B --collective-world1 > $O/b1024_coll_$r.log 2>&1
done
timeout -k 10 240 $B --frames 1536 > $O/b1536.log 2>&1
timeout -k 10 300 $B --frames 2048 > $O/b2048.log 2>&1
