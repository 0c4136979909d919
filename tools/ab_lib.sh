#!/bin/bash
# A/B of the in-tree library against tools/build/libocg_old.so (alternating component timings)
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
for k in 1 2 3; do
  for lib in optimalcontrolmps_amd/liboptimalcontrolmps_amd.so tools/build/libocg_old.so; do
    echo "== $lib"
    OCG_LIB=$lib timeout -k 10 120 python -u tools/time_parts.py 2>&1 | grep -v amdgpu.ids | sed -n '1p;5p' || exit 1
  done
done
