#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03c24
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o bench -- python3 bench.py --steps 6 --warmup 2 --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0 --no-timing > $O/bench.log 2>&1
