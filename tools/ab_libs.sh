#!/bin/bash
# A/B/C of library builds under tools/build/ (parity per build, alternating component timings)
mkdir -p gpurun_out
LIBS="tools/build/libocg_old.so tools/build/libocg_A.so tools/build/libocg_B.so"
for lib in $LIBS; do
  echo "== parity $lib"
  OCG_LIB=$lib timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
done
for k in 1 2; do
  for lib in $LIBS; do
    echo "== $lib"
    OCG_LIB=$lib timeout -k 10 120 python -u tools/time_parts.py 2>&1 | grep -v amdgpu.ids | sed -n '1p;5p' || exit 1
  done
done
