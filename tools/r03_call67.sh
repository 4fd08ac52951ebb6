#!/bin/bash
# map chain through LDS: map / shard / sequence parity, a same-box A/B, and a kernel trace of the new form
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c67
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_map.py tests/test_gpu_shard.py tests/test_gpu_sequence.py > $O/pytest.log 2>&1
B="python bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
for r in 1 2; do
  YAVO_LIB=ya_vo_amd/lib/libyavo_mapold.so timeout -k 10 200 $B > $O/ab_old_$r.log 2>&1
  timeout -k 10 200 $B > $O/ab_new_$r.log 2>&1
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- \
    python3 bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0 > $O/rocprof_bench.log 2>&1
