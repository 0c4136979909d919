#!/bin/bash
# pipelined HBM getHessian: parity tests, the c4rows bench line, eigensolver phase stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SEL=${SEL:-tests/test_config4.py tests/test_group_device.py tests/test_checkpoint.py tests/test_engines_agree.py tests/test_ground_state.py}
timeout -k 10 600 python -u -m pytest $SEL -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_pipe.log 2>&1
rc=$?; grep -E "PASS|FAIL|gs L=10|Error" gpurun_out/pytest_pipe.log | tail -40; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload c4rows --steps 2 --warmup 1 > gpurun_out/c4pipe.json 2> gpurun_out/c4pipe.err
rc=$?; cut -c1-1500 gpurun_out/c4pipe.json; tail -3 gpurun_out/c4pipe.err; [ $rc -ne 0 ] && exit $rc
( for a in "192 1 64" "128 1 32" "96 1 32"; do timeout -k 5 120 ./tools/build/eig_bench_st $a || exit 1; done ) > gpurun_out/eig_st.log 2>&1
rc=$?; cat gpurun_out/eig_st.log; exit $rc
