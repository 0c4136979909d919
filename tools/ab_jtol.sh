#!/bin/bash
# A/B of the Jacobi rotation threshold (OCG_JTOL2 builds under tools/build/): accuracy + speed
mkdir -p gpurun_out
for lib in optimalcontrolmps_amd/liboptimalcontrolmps_amd.so tools/build/libocg_jt1e-24.so tools/build/libocg_jt1e-20.so; do
  echo "== $lib"
  OCG_LIB=$lib timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids || exit 1
  OCG_LIB=$lib timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
  OCG_LIB=$lib timeout -k 10 120 python -u tools/time_parts.py 2>&1 | head -1 || exit 1
  OCG_LIB=$lib timeout -k 10 120 python -u tools/time_parts.py 2>&1 | head -1 || exit 1
done
