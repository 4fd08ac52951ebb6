#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c36
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_geom.py tests/test_gpu_track.py > $O/pytest.log 2>&1
timeout -k 10 200 python tools/lm_profile.py --frames 1024 > $O/lm_prof_1024.log 2>&1
timeout -k 10 200 python tools/lm_profile.py --frames 1024 --plain > $O/lm_plain_1024.log 2>&1
timeout -k 10 200 python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0 > $O/bench.log 2>&1
