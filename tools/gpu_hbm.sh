#!/bin/bash
# HBM-engine parity tests, then the config-4 strong bench line (N_t = 33)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -rf -m gpu \
  tests/test_eigensolver_gpu.py tests/test_config4.py tests/test_config5.py tests/test_engines_agree.py ${EXTRA_TESTS} \
  > gpurun_out/pytest_hbm.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_hbm.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_hbm.log | head -30; exit $rc; }
timeout -k 10 300 python -u bench.py --workload c4rows --steps 2 --warmup 1 > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -5 gpurun_out/c4.err; exit 1; }
cut -c1-900 gpurun_out/c4.json
