#!/bin/bash
# Maxm-boundary eigenvalue resolution: eigensolver + config-4 parity tests, c4rows with it on / off
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_eigensolver_gpu.py tests/test_config4.py -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_thr.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_thr.log | tail -40; [ $rc -ne 0 ] && exit $rc
for t in 1 0; do
  OCG_HBM_THRESH=$t timeout -k 10 300 python -u bench.py --workload c4rows --steps 2 --warmup 1 > gpurun_out/c4thr$t.json 2> gpurun_out/c4thr$t.err || { tail -5 gpurun_out/c4thr$t.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c4thr$t.json')); print('THRESH=$t', d['value'], d['ms_per_step'], d['single_chain_steps_per_sec'], d['mfma_gemm']['share_of_time'])"
done
