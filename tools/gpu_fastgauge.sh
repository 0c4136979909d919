#!/bin/bash
# certified gauge moves: the HBM-engine tests, then config 4 with the path on / off and its counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread -rf -m gpu \
  tests/test_eigensolver_gpu.py tests/test_config4.py tests/test_config5.py tests/test_engines_agree.py \
  tests/test_ground_state.py tests/test_checkpoint.py tests/test_group_device.py \
  > gpurun_out/pytest_fg.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_fg.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_fg.log | head -30; exit $rc; }
for f in 1 0; do
  OCG_HBM_FASTGAUGE=$f OCG_GEMM_STATS=1 timeout -k 10 300 python -u bench.py --workload c4rows --steps 2 --warmup 1 > gpurun_out/c4_fg$f.json 2> gpurun_out/c4_fg$f.err || { tail -5 gpurun_out/c4_fg$f.err; exit 1; }
  echo "fastgauge=$f"; cut -c1-330 gpurun_out/c4_fg$f.json; grep "stream ms" gpurun_out/c4_fg$f.err
done
