# check (smoke, parity, bench) + phase profiles at 64 and 256 threads per chain
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh &&
OCG_PROF_NT=256 timeout -k 10 300 python tools/profile_phases.py > gpurun_out/phases_nt256.log 2>&1 && echo "phases256 ok"
