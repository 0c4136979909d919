#!/bin/bash
# round-3 rocprofv3 evidence (kernel trace + FETCH / WRITE / MFMA-issue PMC passes,
# tools/prof_passes.sh) of the bench commands whose lines carry a roofline:
#   r03       python bench.py (config 1, the driver's default line)
#   r03c4n33  python bench.py --workload c4rows (pipelined HBM getHessian, GROUP M=40)
#   r03c5n17  python bench.py --workload c5rows
#   r03c4n129 python bench.py --workload c4rows --c4-nt 129 (larger row batches)
set -o pipefail
R=$GRAFT_REPO_ROOT
for w in ${@:-c1 c4 c5}; do
  case $w in
    c1) bash $R/tools/prof_passes.sh r03 --no-cpu-baseline --steps 5 --warmup 1 || exit $? ;;
    c4) bash $R/tools/prof_passes.sh r03c4n33 --workload c4rows --steps 1 --warmup 1 || exit $? ;;
    c5) bash $R/tools/prof_passes.sh r03c5n17 --workload c5rows --steps 1 --warmup 0 || exit $? ;;
    c4l) bash $R/tools/prof_passes.sh r03c4n129 --workload c4rows --c4-nt 129 --steps 1 --warmup 1 || exit $? ;;
  esac
  echo "profiled $w"
done
