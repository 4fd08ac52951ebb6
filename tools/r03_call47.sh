#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c47
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_track.py > $O/pytest.log 2>&1
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  for v in base noring bpw3 bpw12; do
    L=ya_vo_amd/lib/libyavo.so; E=1
    [ $v = noring ] && E=0
    [ $v = bpw3 ] && L=ya_vo_amd/lib/libyavo_bpw3.so
    [ $v = bpw12 ] && L=ya_vo_amd/lib/libyavo_bpw12.so
    YAVO_BRIEF_RING=$E YAVO_LIB=$L timeout -k 10 200 $B > $O/ab_${v}_$r.log 2>&1
  done
done
