#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c45
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_geom.py tests/test_gpu_track.py tests/test_gpu_sequence.py > $O/pytest.log 2>&1
timeout -k 10 100 python tools/lm_profile.py --frames 1024 > $O/lm_prof.log 2>&1
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  for v in base l0; do
    if [ $v = base ]; then L=ya_vo_amd/lib/libyavo.so; else L=ya_vo_amd/lib/libyavo_$v.so; fi
    YAVO_LIB=$L timeout -k 10 100 python tools/lm_profile.py --frames 1024 --plain --lib $L > $O/lm_${v}_$r.log 2>&1
    YAVO_LIB=$L timeout -k 10 200 $B > $O/ab_${v}_$r.log 2>&1
  done
done
