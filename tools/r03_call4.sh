#!/bin/bash
# round 3, call 4: default bench (all legs), LoopHandler with the decode pool
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03c4
mkdir -p $O
timeout -k 10 900 python bench.py > $O/bench_default.log 2>&1
timeout -k 10 400 python tools/bench_loop_handler.py --frames 400 --out $O/loop_handler.json > $O/loop_handler.log 2>&1
