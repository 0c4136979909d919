#!/bin/bash
# round 4: full GPU suite, default bench line, A/B of this round's library (A) against the
# round-start build (ab/libprev.so, B) on config 1 and the c4rows slice, c4rows line with its CPU baseline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r04c_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|c5 w512|gs L=10" gpurun_out/r04c_tests.log | tail -20
tail -2 gpurun_out/r04c_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r04c_bench.json 2> gpurun_out/r04c_bench.err || { tail -20 gpurun_out/r04c_bench.err; exit 1; }
cut -c1-300 gpurun_out/r04c_bench.json
timeout -k 10 300 python -u bench.py --workload c4rows --steps 3 --warmup 1 --state-cache /tmp/c4.npz > gpurun_out/r04c_c4rows.json 2> gpurun_out/r04c_c4rows.err || { tail -20 gpurun_out/r04c_c4rows.err; exit 1; }
cut -c1-300 gpurun_out/r04c_c4rows.json
for v in A B A B; do
  if [ $v = B ]; then export OCG_LIB=$PWD/ab/libprev.so; else unset OCG_LIB; fi
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 --warmup 2 > gpurun_out/r04c_ab1_$v.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py --workload c4rows --steps 3 --warmup 1 --no-cpu-baseline --state-cache /tmp/c4.npz > gpurun_out/r04c_ab4_$v.json 2>/dev/null || exit 1
  python -c "import json; a=json.load(open('gpurun_out/r04c_ab1_$v.json')); b=json.load(open('gpurun_out/r04c_ab4_$v.json')); print('$v', 'c1', round(a['ms_per_step'],3), 'ms', 'c4rows', round(b['ms_per_step'],1), 'ms')"
done
exit $rc
