#!/bin/bash
# r03_call56 (matcher epilogue A/B) then r03_call55 (re-tuning at B = 2048) in one box session
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/r03_call56.sh
bash tools/r03_call55.sh
