#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03c27
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_png.py > $O/pytest_png.log 2>&1
timeout -k 10 300 python tools/png_e2e_probe.py > $O/pe2e.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o pe2e -- python3 tools/png_e2e_probe.py > $O/pe2e_tr.log 2>&1
