# kernel-trace statistics of the config-4 Hessian slice (summarised on the box)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_c4
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4 -o run -- python3 $R/bench.py --workload c4rows --steps 1 --warmup 0 > $R/gpurun_out/prof_c4.log 2>&1 || exit $?
python3 -c "
import sys; sys.path.insert(0, '$R/tools'); import prof_summary as P
for r in P.kernel_stats('$R/gpurun_out/prof_c4/run_results.db'): print(r)
" > $R/gpurun_out/c4_kernel_stats.txt
rm -rf $R/gpurun_out/prof_c4
cat $R/gpurun_out/c4_kernel_stats.txt
