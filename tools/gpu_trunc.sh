# k_truncate rewrite: HBM-engine tests, then c4rows kernel stats (rocprof) and the slice time
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_config4.py tests/test_eigensolver_gpu.py tests/test_checkpoint.py tests/test_config5_chi512.py > gpurun_out/t_trunc.txt 2>&1 || exit 1
B="python bench.py --workload c4rows --steps 2 --warmup 1 --no-cpu-baseline --state-cache /tmp/c4s.npz"
timeout -k 10 200 $B > gpurun_out/c4_trunc.json 2> /dev/null || exit 1
timeout -k 10 200 $B > gpurun_out/c4_trunc2.json 2> /dev/null || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trunc -o trunc -- python bench.py --workload c4rows --steps 1 --warmup 1 --no-cpu-baseline --profiled --state-cache /tmp/c4s.npz > gpurun_out/prof_trunc.log 2>&1
