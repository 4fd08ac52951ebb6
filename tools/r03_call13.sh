#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03c13
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_png.py > $O/pytest_png.log 2>&1
timeout -k 10 300 python tools/png_gpu_probe.py --frames 1024 > $O/png_probe.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pngkt -o png -- python3 tools/png_gpu_probe.py --frames 1024 > $O/png_probe_kt.log 2>&1
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1
