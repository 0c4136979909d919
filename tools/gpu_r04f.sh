#!/bin/bash
# round 4 final: the full GPU suite (all oracle fixtures present), the default bench line, smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r04f_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|long_vs_oracle|L12|c5 w512" gpurun_out/r04f_tests.log | tail -20
tail -2 gpurun_out/r04f_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f_smoke.log 2>&1 || { tail -5 gpurun_out/r04f_smoke.log; exit 1; }
tail -2 gpurun_out/r04f_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r04f_bench.json 2> gpurun_out/r04f_bench.err || { tail -20 gpurun_out/r04f_bench.err; exit 1; }
cut -c1-400 gpurun_out/r04f_bench.json
exit $rc
