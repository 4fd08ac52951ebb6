#!/bin/bash
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/r03c17
mkdir -p $O
RE=inflate_kernel
CMD="python3 tools/png_gpu_probe.py --frames 256"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex "$RE" --output-format csv -d $O -o inf_a -- $CMD > $O/inf_a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM --kernel-include-regex "$RE" --output-format csv -d $O -o inf_b -- $CMD > $O/inf_b.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU --kernel-include-regex "$RE" --output-format csv -d $O -o inf_c -- $CMD > $O/inf_c.log 2>&1
