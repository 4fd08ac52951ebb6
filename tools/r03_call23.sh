#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03c23
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_track.py tests/test_gpu_shard.py tests/test_gpu_map.py > $O/pytest.log 2>&1
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  timeout -k 10 200 $B > $O/new_$r.log 2>&1
  YAVO_LIB=ya_vo_amd/lib/libyavo_p1.so timeout -k 10 200 $B > $O/old_$r.log 2>&1
done
