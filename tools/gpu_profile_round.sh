# Round-end evidence: GPU parity tests, default bench (with CPU baseline),
# rocprofv3 kernel-trace stats of the bench, and FETCH_SIZE / WRITE_SIZE PMC
# passes (separate runs; no tracing domains combined with --pmc).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
make -s -C oracle &&
timeout -k 10 900 python -m pytest tests -m gpu -x -q -rf --tb=short > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && echo "bench ok" &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 && echo "kernel-trace ok" &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch_$TAG.log 2>&1 && echo "pmc fetch ok" &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write_$TAG.log 2>&1 && echo "pmc write ok"
