#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c41
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_xlane.py tests/test_gpu_parity.py tests/test_gpu_geom.py tests/test_gpu_map.py tests/test_gpu_shard.py > $O/pytest.log 2>&1
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  for v in base ns kpl0; do
    if [ $v = base ]; then L=ya_vo_amd/lib/libyavo.so; else L=ya_vo_amd/lib/libyavo_$v.so; fi
    YAVO_LIB=$L timeout -k 10 200 $B > $O/ab_${v}_$r.log 2>&1
  done
done
bash tools/pmc_kernel.sh brief_kernel brief_sort
