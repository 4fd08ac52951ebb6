set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex pose_lm --output-format csv -d gpurun_out/pmc -o lm1 -- python3 tools/lm_profile.py --plain > gpurun_out/pmc/lm1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex pose_lm --output-format csv -d gpurun_out/pmc -o lm2 -- python3 tools/lm_profile.py --plain > gpurun_out/pmc/lm2.log 2>&1
