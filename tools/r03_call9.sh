#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03c9
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1
