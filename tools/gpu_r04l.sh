#!/bin/bash
# round 4: stream-priority mode 2 (default): c5rows A/B, the c4rows line, profiles c4 (N_t=33) and c5, HBM tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload c5rows --prepare-only --state-cache /tmp/c5.npz > /dev/null 2>&1 || exit 1
for pr in 2 0 2 0; do
  OCG_HBM_PRIO=$pr timeout -k 10 300 python -u bench.py --workload c5rows --steps 1 --warmup 1 --no-cpu-baseline --state-cache /tmp/c5.npz > gpurun_out/r04l_c5.json 2>/dev/null || exit 1
  python -c "import json; a=json.load(open('gpurun_out/r04l_c5.json')); print('c5rows prio $pr', round(a['ms_per_step'],1), 'ms')"
done
timeout -k 10 300 python -u bench.py --workload c4rows --steps 3 --warmup 1 > gpurun_out/r04l_c4rows.json 2> gpurun_out/r04l_c4rows.err || { tail -5 gpurun_out/r04l_c4rows.err; exit 1; }
cut -c1-300 gpurun_out/r04l_c4rows.json
timeout -k 10 600 python -u -m pytest tests/test_config4.py tests/test_config5.py tests/test_config5_chi512.py tests/test_checkpoint.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r04l_tests.log 2>&1 || { tail -20 gpurun_out/r04l_tests.log; exit 1; }
tail -1 gpurun_out/r04l_tests.log
timeout -k 10 1000 bash tools/profile_r04.sh c4 c5 > gpurun_out/r04l_prof.log 2>&1 || { tail -20 gpurun_out/r04l_prof.log; exit 1; }
grep '"metric"' gpurun_out/r04l_prof.log | cut -c1-250
