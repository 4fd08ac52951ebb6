#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03c20
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_track.py tests/test_gpu_lk.py > $O/pytest_track.log 2>&1
timeout -k 10 400 python bench.py --tracker lk --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0 > $O/bench_lk.log 2>&1
