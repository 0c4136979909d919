# phase profiles of the chain engine at 64/128/256 threads per chain
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for nt in 64 128 256; do
  OCG_PROF_NT=$nt timeout -k 10 300 python tools/profile_phases.py > gpurun_out/phases_nt$nt.log 2>&1 || exit 1
  echo "nt $nt ok"
done
