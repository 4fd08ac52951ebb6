#!/bin/bash
# the staging A/B (r03_call58), the co-residency A/B (r03_call60), then the round-end check (r03_final), one session
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/r03_call58.sh
bash tools/r03_call60.sh
bash tools/r03_final.sh
