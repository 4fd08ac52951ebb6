#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03c19
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sequence.py tests/test_gpu_ba.py > $O/pytest_seq.log 2>&1
timeout -k 10 300 python tools/bench_sequence.py --out $O/seq_device.json > $O/seq_device.log 2>&1
timeout -k 10 300 python tools/bench_sequence.py --host-window --no-cpu --out $O/seq_host.json > $O/seq_host.log 2>&1
