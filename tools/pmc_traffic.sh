#!/bin/bash
# HBM traffic of each pipeline kernel from rocprofv3 PMC counters, collected as the MI355X guide
# prescribes: FETCH_SIZE and WRITE_SIZE in SEPARATE --pmc passes (FETCH_SIZE takes 3 TCC slots,
# WRITE_SIZE 2), no trace domains combined with --pmc.  Writes profiles/pmc_traffic.json (read by
# bench.py for roofline.traffic) and the raw CSVs under gpurun_out/pmc_*.
#   usage (on the GPU box, repo root): bash tools/pmc_traffic.sh [bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
    echo "[$(date +%T)] pmc pass $C"
    timeout -k 10 600 rocprofv3 --pmc "$C" --output-format csv -d "$OUT/pmc_$C" -o pmc -- \
        python3 "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-baseline none --no-timing "$@" \
        > "$OUT/pmc_$C.log" 2>&1
    st=$?
    echo "[$(date +%T)] pmc pass $C exit=$st"
    [ $st -eq 0 ] || exit $st
done
python3 "$ROOT/tools/pmc_traffic.py" "$OUT" "$@" && cp "$ROOT/profiles/pmc_traffic.json" "$OUT/pmc_traffic.json"
