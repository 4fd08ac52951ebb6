#!/bin/bash
# LK tracking mode at the default B = 2048 and at 1024
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c64
mkdir -p $O
B="python bench.py --tracker lk --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
timeout -k 10 300 $B > $O/lk_2048.log 2>&1
timeout -k 10 300 $B --frames 1024 > $O/lk_1024.log 2>&1
