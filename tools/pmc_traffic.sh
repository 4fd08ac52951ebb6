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
# third pass: the FP64 VALU counters (6 SQ slots of 8) -- FLOPs and instructions of the pose LM
FP64="SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"
for C in FETCH_SIZE WRITE_SIZE FP64; do
    echo "[$(date +%T)] pmc pass $C"
    CTRS="$C"
    [ "$C" = "FP64" ] && CTRS="$FP64"
    timeout -k 10 600 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/pmc_$C" -o pmc -- \
        python3 "$ROOT/bench.py" --steps 3 --warmup 1 --cpu-baseline none --no-timing "$@" \
        > "$OUT/pmc_$C.log" 2>&1
    st=$?
    echo "[$(date +%T)] pmc pass $C exit=$st"
    [ $st -eq 0 ] || exit $st
done
python3 "$ROOT/tools/pmc_traffic.py" "$OUT" "$@" && cp "$ROOT/profiles/pmc_traffic.json" "$OUT/pmc_traffic.json"
