#!/bin/bash
# quick GPU check: parity tests, component timings, one bench line (no CPU baseline)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 120 python -u tools/time_parts.py || exit $?
timeout -k 10 240 python -u bench.py --no-cpu-baseline --steps 20 || exit $?
if [ "$1" = "prof" ]; then
  OCG_PROF_NT=128 timeout -k 10 180 python -u tools/profile_phases.py 2>&1 | sed -n '/trajectory(2/,/div_t/p'
fi
