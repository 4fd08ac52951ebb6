#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c43
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_geom.py tests/test_gpu_track.py tests/test_gpu_sequence.py tests/test_gpu_lk.py > $O/pytest.log 2>&1
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  for v in 1 0; do
    YAVO_LM_RESIDENT=$v timeout -k 10 100 python tools/lm_profile.py --frames 1024 --plain > $O/lm_res${v}_$r.log 2>&1
    YAVO_LM_RESIDENT=$v timeout -k 10 200 $B > $O/ab_res${v}_$r.log 2>&1
  done
done
bash tools/pmc_traffic.sh --png-steps 0 --loop-handler-frames 0 --e2e-steps 0 > $O/pmc_traffic.log 2>&1
