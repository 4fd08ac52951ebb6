#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
R=$(pwd)
export TMPDIR=/tmp
O=$R/gpurun_out/r03c34
mkdir -p $O
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o out -- python3 $R/bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0 --steps 20 --no-overlap > $O/serial.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/step -o out -- python3 $R/bench.py --cpu-baseline none --png-steps 0 --loop-handler-frames 0 --e2e-steps 0 --steps 20 > $O/step.log 2>&1
