#!/bin/bash
# round 4: GPU suite, default bench line, 2-rank dry run of bench.py's own launcher
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a_tests.log 2>&1 || { tail -30 gpurun_out/r04a_tests.log; exit 1; }
tail -3 gpurun_out/r04a_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || { tail -20 gpurun_out/r04a_bench.err; exit 1; }
cut -c1-600 gpurun_out/r04a_bench.json
OCG_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04a_bench2.json 2> gpurun_out/r04a_bench2.err || { tail -20 gpurun_out/r04a_bench2.err; exit 1; }
cut -c1-300 gpurun_out/r04a_bench2.json
timeout -k 10 120 ./tools/build/ube128 > gpurun_out/r04a_ube.log 2>&1 && timeout -k 10 120 ./tools/build/ubp128 > gpurun_out/r04a_ubp.log 2>&1 || exit 1
cat gpurun_out/r04a_ube.log gpurun_out/r04a_ubp.log
