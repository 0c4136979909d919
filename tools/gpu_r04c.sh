#!/bin/bash
# round 4: full GPU suite, default bench line, population-exact profiles c4 (N_t=129) and c5 (N_t=17)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r04c_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|c5 w512|gs L=10" gpurun_out/r04c_tests.log | tail -20
tail -2 gpurun_out/r04c_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r04c_bench.json 2> gpurun_out/r04c_bench.err || { tail -20 gpurun_out/r04c_bench.err; exit 1; }
cut -c1-300 gpurun_out/r04c_bench.json
timeout -k 10 300 python -u tools/c5_warm_L12.py > gpurun_out/r04c_warmL12.log 2>&1 || { tail -5 gpurun_out/r04c_warmL12.log; exit 1; }
tail -3 gpurun_out/r04c_warmL12.log
timeout -k 10 900 bash tools/profile_r04.sh c4l c5 > gpurun_out/r04c_prof.log 2>&1 || { tail -20 gpurun_out/r04c_prof.log; exit 1; }
tail -12 gpurun_out/r04c_prof.log
exit $rc
