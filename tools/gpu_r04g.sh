#!/bin/bash
# round 4: the pipelined getHessian's memory estimate (chain pools at 1.5x): c5rows pipelined vs
# two-phase, c4rows N_t=33/129, and the HBM-engine GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload c5rows --prepare-only --state-cache /tmp/c5.npz > /dev/null 2>&1 || exit 1
for pipe in 1 0; do
  OCG_PIPE_DEBUG=0 OCG_HBM_PIPE=$pipe timeout -k 10 300 python -u bench.py --workload c5rows --steps 1 --warmup 1 --no-cpu-baseline --state-cache /tmp/c5.npz > gpurun_out/r04g_c5_$pipe.json 2>/dev/null || exit 1
  python -c "import json; b=json.load(open('gpurun_out/r04g_c5_$pipe.json')); print('c5rows pipe=$pipe', round(b['ms_per_step'],1), 'ms', round(b['value'],3), 'rows/s')"
done
timeout -k 10 300 python -u bench.py --workload c4rows --steps 3 --warmup 1 > gpurun_out/r04g_c4.json 2>/dev/null || exit 1
python -c "import json; b=json.load(open('gpurun_out/r04g_c4.json')); print('c4rows', round(b['ms_per_step'],1), 'ms', round(b['value'],2), 'rows/s', 'cpu', b['cpu_baseline']['value'])"
timeout -k 10 300 python -u bench.py --workload c4rows --c4-nt 129 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r04g_c4l.json 2>/dev/null || exit 1
python -c "import json; b=json.load(open('gpurun_out/r04g_c4l.json')); print('c4rows N_t=129', round(b['ms_per_step'],1), 'ms', round(b['value'],2), 'rows/s')"
timeout -k 10 900 python -u -m pytest tests/test_config4.py tests/test_config5.py tests/test_config5_chi512.py tests/test_checkpoint.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04g_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR" gpurun_out/r04g_tests.log | tail; tail -1 gpurun_out/r04g_tests.log
exit $rc
