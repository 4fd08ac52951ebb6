#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c46
mkdir -p $O
timeout -k 10 200 python tools/det_profile.py --frames 1024 > $O/det_prof_1024.log 2>&1
timeout -k 10 200 python tools/brief_profile.py --frames 1024 > $O/brief_prof_1024.log 2>&1 || true
