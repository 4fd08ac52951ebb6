#!/bin/bash
# Round-3 profiles at the new default batch (B = 2048): HBM traffic / FP64 PMC passes (profiles/pmc_traffic.json),
# a kernel-trace --stats summary of the bench, then the full default bench that reads the traffic back
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c53
mkdir -p $O
export TMPDIR=/tmp
bash tools/pmc_traffic.sh --png-steps 0 --loop-handler-frames 0 --e2e-steps 0 > $O/pmc_traffic.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- \
    python3 bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0 > $O/rocprof_bench.log 2>&1
timeout -k 10 900 python bench.py > $O/bench_default.log 2>&1
