set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench tools/ubench.hip &&
timeout -k 10 120 /tmp/ubench > gpurun_out/ubench.log 2>&1 && echo ubench ok &&
OCG_PROF_NT=64 timeout -k 10 300 python tools/profile_phases.py > gpurun_out/phases_nt64.log 2>&1 && echo phases ok
