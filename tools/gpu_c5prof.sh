# kernel-trace statistics of config 5 (warm-up to chi=512 dominates: a chi=512 step mix)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_c5
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c5 -o run -- python3 $R/bench.py --workload c5rows --c5-nt 3 --steps 1 --warmup 0 > $R/gpurun_out/prof_c5.log 2>&1 || exit $?
python3 -c "
import sys; sys.path.insert(0, '$R/tools'); import prof_summary as P
for r in P.kernel_stats('$R/gpurun_out/prof_c5/run_results.db'): print(r)
" > $R/gpurun_out/c5_kernel_stats.txt
rm -rf $R/gpurun_out/prof_c5
cat $R/gpurun_out/c5_kernel_stats.txt
