#!/bin/bash
# round 4: the long-horizon chi=256 oracle test, population-exact profiles c4 (N_t=129) and c5 (N_t=17)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_config4.py -m gpu -v -s -k long --timeout 300 --timeout-method thread > gpurun_out/r04d_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r04d_tests.log | tail -6
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 1000 bash tools/profile_r04.sh c4l c5 > gpurun_out/r04d_prof.log 2>&1 || { tail -20 gpurun_out/r04d_prof.log; exit 1; }
tail -12 gpurun_out/r04d_prof.log
exit $rc
