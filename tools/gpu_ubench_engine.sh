set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for nt in ${NTS:-64}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DOCG_NT=$nt -I optimalcontrolmps_amd/csrc -o /tmp/ube$nt tools/ubench_engine.hip &&
  timeout -k 10 120 /tmp/ube$nt > gpurun_out/ubench_engine_nt$nt.log 2>&1 &&
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DOCG_NT=$nt -DOCG_PROFILE -I optimalcontrolmps_amd/csrc -o /tmp/ubp$nt tools/ubench_engine.hip &&
  timeout -k 10 120 /tmp/ubp$nt > gpurun_out/ubench_engine_prof_nt$nt.log 2>&1 || exit 1
done
echo done
