#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c39
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_xlane.py tests/test_gpu_parity.py tests/test_gpu_geom.py tests/test_gpu_map.py tests/test_gpu_shard.py > $O/pytest.log 2>&1
timeout -k 10 200 python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0 > $O/bench.log 2>&1
bash tools/pmc_kernel.sh brief_kernel brief_r03
