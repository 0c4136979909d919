#!/bin/bash
# A/B of the workgroup width (OCG_NT builds under tools/build/): parity + speed
mkdir -p gpurun_out
for lib in tools/build/libocg_nt256.so; do
  echo "== $lib"
  OCG_LIB=$lib timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids || exit 1
  OCG_LIB=$lib timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
  OCG_LIB=$lib timeout -k 10 120 python -u tools/time_parts.py 2>&1 | grep -v amdgpu.ids || exit 1
done
