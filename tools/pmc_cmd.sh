#!/bin/bash
# SQ counters (two separate --pmc passes, no traces) for kernels matching REGEX while running a command:
#   bash tools/pmc_cmd.sh REGEX TAG -- python3 script.py args...
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
RE=$1; TAG=$2; shift 3
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex "$RE" --output-format csv -d gpurun_out/pmc -o ${TAG}_a -- "$@" > gpurun_out/pmc/${TAG}_a.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT --kernel-include-regex "$RE" --output-format csv -d gpurun_out/pmc -o ${TAG}_b -- "$@" > gpurun_out/pmc/${TAG}_b.log 2>&1
