#!/bin/bash
# round 3, call 6: GPU PNG decoder tests, then the PNG legs of the bench
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03c6
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_png.py > $O/pytest_png.log 2>&1
timeout -k 10 600 python bench.py --cpu-baseline none --loop-handler-frames 0 > $O/bench_png.log 2>&1
