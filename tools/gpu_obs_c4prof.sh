# observables GPU tests + kernel-trace statistics of the config-4 Hessian slice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_observables.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pt_obs.log 2>&1
echo "obs pytest exit $?"
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4rows --steps 1 --warmup 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_c4.log 2>&1
echo "prof exit $?"
find $GRAFT_REPO_ROOT/gpurun_out/prof_c4 -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/c4_kernel_stats.csv \;
find $GRAFT_REPO_ROOT/gpurun_out/prof_c4 -name "*.db" -delete
head -12 $GRAFT_REPO_ROOT/gpurun_out/c4_kernel_stats.csv
