#!/bin/bash
# round 4: chi=512 tests, the chi=512 Hessian diagnostic, population-exact profiles c1 + c4 (N_t=33)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_config5_chi512.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r04b_c5tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|c5 w512|passed|failed" gpurun_out/r04b_c5tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/c5_hess_diag.py > gpurun_out/r04b_c5diag.log 2>&1 || { tail -5 gpurun_out/r04b_c5diag.log; exit 1; }
cat gpurun_out/r04b_c5diag.log
timeout -k 10 900 bash tools/profile_r04.sh c1 c4 > gpurun_out/r04b_prof.log 2>&1 || { tail -20 gpurun_out/r04b_prof.log; exit 1; }
tail -20 gpurun_out/r04b_prof.log
