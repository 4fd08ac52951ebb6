#!/bin/bash
# LoopHandler throughput (serial / pipelined) + HIP API trace of 60 frames
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03lh}
mkdir -p $O
timeout -k 10 400 python tools/bench_loop_handler.py --frames 200 --out $O/loop_handler.json > $O/loop_handler.log 2>&1
python -c "import sys; sys.path.insert(0, 'tools'); import bench_loop_handler as b; print(b.write_sequence('/tmp/lhseq', 60))" > $O/lhseq.log 2>&1
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $O/lhtrace -o lh -- ya_vo_amd/bin/yavo_loop_handler /tmp/lhseq/config.json > $O/lh_trace_run.log 2>&1
