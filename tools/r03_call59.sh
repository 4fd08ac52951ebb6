#!/bin/bash
# the staging A/B (r03_call58) and then the round-end check (r03_final) in one box session
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/r03_call58.sh
bash tools/r03_final.sh
