#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out/r03c35
mkdir -p $O
timeout -k 10 200 python tools/lm_profile.py --frames 1024 > $O/lm_prof_1024.log 2>&1
timeout -k 10 200 python tools/lm_profile.py --frames 128 > $O/lm_prof_128.log 2>&1
timeout -k 10 200 python tools/lm_profile.py --frames 1024 --plain > $O/lm_plain_1024.log 2>&1
