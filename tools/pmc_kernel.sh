#!/bin/bash
# SQ counters for one kernel of the bench (separate passes, kernel-trace-free):
#   bash tools/pmc_kernel.sh REGEX TAG [extra bench.py args, e.g. --tracker lk]
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
RE=$1; TAG=$2
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-include-regex "$RE" --output-format csv -d gpurun_out/pmc -o ${TAG}_a -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline none --no-timing --png-steps 0 --loop-handler-frames 0 --e2e-steps 0 "${@:3}" > gpurun_out/pmc/${TAG}_a.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT --kernel-include-regex "$RE" --output-format csv -d gpurun_out/pmc -o ${TAG}_b -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline none --no-timing --png-steps 0 --loop-handler-frames 0 --e2e-steps 0 "${@:3}" > gpurun_out/pmc/${TAG}_b.log 2>&1
# pass c: LDS behaviour and scalar work
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA --kernel-include-regex "$RE" --output-format csv -d gpurun_out/pmc -o ${TAG}_c -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline none --no-timing --png-steps 0 --loop-handler-frames 0 --e2e-steps 0 "${@:3}" > gpurun_out/pmc/${TAG}_c.log 2>&1
