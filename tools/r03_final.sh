#!/bin/bash
# Round-3 end check at HEAD: the GPU suite, smoke, the full default bench, and a kernel-trace --stats profile of it
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 900 python bench.py > $O/bench_default.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- \
    python3 bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0 > $O/rocprof_bench.log 2>&1
