#!/bin/bash
# round 4: chain-engine microbenchmarks, default bench line, 2-rank dry run of
# bench.py's own launcher, the GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in ube128_old ube128 ubp128_old ubp128 ubp64; do timeout -k 10 120 ./tools/build/$b > gpurun_out/r04a_$b.log 2>&1 || exit 1; done
tail -n 12 gpurun_out/r04a_ube128_old.log gpurun_out/r04a_ube128.log
timeout -k 10 300 python -u bench.py > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || { tail -20 gpurun_out/r04a_bench.err; exit 1; }
cut -c1-400 gpurun_out/r04a_bench.json
OCG_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04a_bench2.json 2> gpurun_out/r04a_bench2.err || { tail -20 gpurun_out/r04a_bench2.err; exit 1; }
cut -c1-300 gpurun_out/r04a_bench2.json
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r04a_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|c5 w512|gs L=10" gpurun_out/r04a_tests.log | grep -v "^tests.*PASSED" | tail -30
tail -3 gpurun_out/r04a_tests.log
exit $rc
