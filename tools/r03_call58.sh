#!/bin/bash
# detect staging with incremental 32-bit offsets: parity (detect / batch / track), then a same-box A/B
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c58
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_track.py tests/test_gpu_sequence.py > $O/pytest.log 2>&1
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2 3; do
  YAVO_LIB=ya_vo_amd/lib/libyavo_stold.so timeout -k 10 200 $B > $O/ab_old_$r.log 2>&1
  timeout -k 10 200 $B > $O/ab_new_$r.log 2>&1
done
