#!/bin/bash
# round 4: stream priorities on by default: the GPU suite, the c4rows / c5rows lines, profiles c4 (N_t=33) and c5
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04j_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR" gpurun_out/r04j_tests.log | tail -20
tail -1 gpurun_out/r04j_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c4rows --steps 3 --warmup 1 > gpurun_out/r04j_c4rows.json 2> gpurun_out/r04j_c4rows.err || { tail -5 gpurun_out/r04j_c4rows.err; exit 1; }
cut -c1-300 gpurun_out/r04j_c4rows.json
timeout -k 10 1000 bash tools/profile_r04.sh c4 c5 > gpurun_out/r04j_prof.log 2>&1 || { tail -20 gpurun_out/r04j_prof.log; exit 1; }
grep '"metric"' gpurun_out/r04j_prof.log | cut -c1-250
