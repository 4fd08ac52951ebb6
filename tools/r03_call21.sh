#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03c21
mkdir -p $O
B="python3 bench.py --tracker lk --steps 2 --warmup 1 --cpu-baseline none --no-timing --png-steps 0 --loop-handler-frames 0 --e2e-steps 0"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU --kernel-include-regex "lk_kernel" --output-format csv -d $O -o lk_a -- $B > $O/lk_a.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH --kernel-include-regex "lk_kernel" --output-format csv -d $O -o lk_b -- $B > $O/lk_b.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "lk_kernel" --output-format csv -d $O -o lk_c -- $B > $O/lk_c.log 2>&1
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o lk_kt -- $B > $O/lk_kt.log 2>&1
