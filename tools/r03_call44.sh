#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c44
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_track.py tests/test_gpu_geom.py > $O/pytest.log 2>&1
timeout -k 10 200 python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0 > $O/bench.log 2>&1
