set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I optimalcontrolmps_amd/csrc -o /tmp/ube tools/ubench_engine.hip &&
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/ube_pmc1 -o run --output-format csv -- /tmp/ube > gpurun_out/ube_pmc1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM -d gpurun_out/ube_pmc2 -o run --output-format csv -- /tmp/ube > gpurun_out/ube_pmc2.log 2>&1 && echo done
