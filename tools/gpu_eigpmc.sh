set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/eigpmc
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/eigpmc/p1 -o run --output-format csv -- ./tools/eig_bench12nb 192 1 32 > gpurun_out/eigpmc/p1.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM -d gpurun_out/eigpmc/p2 -o run --output-format csv -- ./tools/eig_bench12nb 192 1 32 > gpurun_out/eigpmc/p2.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MFMA_F64 SQ_LDS_BANK_CONFLICT -d gpurun_out/eigpmc/p3 -o run --output-format csv -- ./tools/eig_bench12nb 192 1 32 > gpurun_out/eigpmc/p3.log 2>&1; echo rc=$?
