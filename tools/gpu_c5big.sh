# kernel trace of the blocked-eigensolver parity test, then the config-5 Hessian slice bench
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_big
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_big -o run -- python3 -m pytest $R/tests/test_config4.py -m gpu -q -k blocked > $R/gpurun_out/prof_big.log 2>&1 || exit $?
python3 -c "
import sys; sys.path.insert(0, '$R/tools'); import prof_summary as P
for r in P.kernel_stats('$R/gpurun_out/prof_big/run_results.db'): print(r)
" > $R/gpurun_out/big_kernel_stats.txt
rm -rf $R/gpurun_out/prof_big
cd $R && timeout -k 10 600 python bench.py --workload c5rows --steps 1 --warmup 0 > gpurun_out/c5rows_big.log 2>&1; echo rc=$?
