#!/bin/bash
# round 3, call 1: instruction issue-rate probe, parity of the changed kernels, same-box A/B bench (HEAD kernels vs
# working tree), kernel trace, fresh detect counters
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03
mkdir -p $O
timeout -k 10 180 tools/bin/valu_probe > $O/valu_probe.log 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_lk.py tests/test_gpu_track.py tests/test_loop_handler.py > $O/pytest_sel.log 2>&1
for r in 1 2; do
  YAVO_LIB=$PWD/ya_vo_amd/lib/libyavo_base.so timeout -k 10 300 python bench.py --cpu-baseline none > $O/bench_base_$r.log 2>&1
  timeout -k 10 300 python bench.py --cpu-baseline none > $O/bench_new_$r.log 2>&1
done
timeout -k 10 400 python tools/bench_loop_handler.py --frames 200 --out $O/loop_handler.json > $O/loop_handler.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 bench.py --cpu-baseline none > $O/bench_kt.log 2>&1
bash tools/pmc_kernel.sh detect_kernel det_r03
