#!/bin/bash
# One GPU-box session: GPU parity tests, smoke, a short bench and a rocprofv3 kernel-trace profile.
# Every GPU step runs under its own timeout; a crash / fault / timeout (anything but exit 0 or a plain
# test failure, 1) ends the script so nothing further touches the GPU.
#   usage (from the repo root on the box): bash tools/gpu_check.sh [bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
: > "$OUT/status.log"
run() {  # run NAME TIMEOUT CMD...
    local name=$1 t=$2
    shift 2
    echo "[$(date +%T)] start $name" | tee -a "$OUT/status.log"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local st=$?
    echo "[$(date +%T)] $name exit=$st" | tee -a "$OUT/status.log"
    tail -5 "$OUT/$name.log"
    return $st
}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

if [ "${SKIP_TESTS:-0}" != "1" ]; then
    run pytest_gpu 900 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread; st=$?; ok $st || exit $st
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; st=$?; ok $st || exit $st
fi
run bench 900 python bench.py "$@"; st=$?; ok $st || exit $st
[ "${PROFILE:-1}" = "1" ] || exit 0
export TMPDIR=/tmp
run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
    python3 "$ROOT/bench.py" --cpu-baseline none "$@"; st=$?; ok $st || exit $st
find "$OUT/prof" -name "*stats*" | head
exit 0
