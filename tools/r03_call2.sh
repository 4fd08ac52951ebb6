#!/bin/bash
# round 3, call 2: probe (window mode), detect parity, same-box A/B (HEAD~ kernels vs working tree), detect counters
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03c2
mkdir -p $O
timeout -k 10 240 tools/bin/valu_probe > $O/valu_probe.log 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_track.py > $O/pytest_sel.log 2>&1
for r in 1 2; do
  YAVO_LIB=$PWD/ya_vo_amd/lib/libyavo_base.so timeout -k 10 300 python bench.py --cpu-baseline none > $O/bench_base_$r.log 2>&1
  timeout -k 10 300 python bench.py --cpu-baseline none > $O/bench_new_$r.log 2>&1
done
bash tools/pmc_kernel.sh detect_kernel det_c2
python -c "import sys; sys.path.insert(0, 'tools'); import bench_loop_handler as b; print(b.write_sequence('/tmp/lhseq', 60))" > $O/lhseq.log 2>&1
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $O/lhtrace -o lh -- ya_vo_amd/bin/yavo_loop_handler /tmp/lhseq/config.json > $O/lh_trace_run.log 2>&1
timeout -k 10 400 python tools/bench_loop_handler.py --frames 200 --out $O/loop_handler.json > $O/loop_handler.log 2>&1
