#!/bin/bash
# A/B of the row-overlap launch shape (one-wave vs two-wave workgroups, resident grid size)
./tools/gpu_quick.sh > gpurun_out/q.log 2>&1 || { tail -20 gpurun_out/q.log; exit 1; }
for cfg in "1 4096" "1 2048" "1 8192" "1 1024" "0 2048" "1 0"; do
  set -- $cfg
  echo "== wave=$1 grid=$2" >> gpurun_out/q.log
  OCG_ROWOV_WAVE=$1 OCG_ROWOV_GRID=$2 timeout -k 10 120 python -u tools/time_parts.py 2>&1 | head -1 >> gpurun_out/q.log || exit 1
done
grep -v amdgpu.ids gpurun_out/q.log | cut -c1-200
