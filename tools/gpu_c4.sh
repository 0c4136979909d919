# config-4 chain benches (HBM engine): Hessian slice rows/s and full-horizon gradient
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python bench.py --workload c4rows --steps 1 --warmup 1 > gpurun_out/c4rows.log 2>&1 && tail -1 gpurun_out/c4rows.log
timeout -k 10 500 python bench.py --workload c4grad --steps 1 --warmup 0 > gpurun_out/c4grad.log 2>&1 && tail -1 gpurun_out/c4grad.log
