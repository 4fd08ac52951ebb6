#!/bin/bash
# round 3, call 5: SQ counters of brief / match / finalize / top-K at HEAD
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
bash tools/pmc_kernel.sh brief_kernel brief_r03
bash tools/pmc_kernel.sh match_fp4 match_r03
bash tools/pmc_kernel.sh match_finalize fin_r03
bash tools/pmc_kernel.sh topk_kernel topk_r03
