set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_rg4
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --output-format csv -d gpurun_out/pmc_rg4/p1 -o run -- python3 tools/probes/profile_ab.py 500 30 255 42 rg4 > gpurun_out/pmc_rg4/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc_rg4/p2 -o run -- python3 tools/probes/profile_ab.py 500 30 255 42 rg4 > gpurun_out/pmc_rg4/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_rg4/p3 -o run -- python3 tools/probes/profile_ab.py 500 30 255 42 rg4 > gpurun_out/pmc_rg4/p3.log 2>&1 || exit 1
echo done
