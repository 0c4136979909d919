#!/bin/bash
# rocprofv3 evidence of one round (TAG, default r05) (kernel trace + FETCH / WRITE / MFMA-issue PMC passes,
# tools/prof_passes.sh) of the bench commands whose lines carry a roofline.  The
# c4 / c5 commands run --profiled on states an unprofiled run cached in /tmp, so
# every k_gemm dispatch in their profiles belongs to the warm-up + timed getHessian
# population the bench line's roofline divides by:
#   <tag>       python bench.py --no-slices (config 1 + the config-2 gradient block)
#   <tag>c4n33  python bench.py --workload c4rows --profiled
#   <tag>c4n129 python bench.py --workload c4rows --c4-nt 129 --profiled
#   <tag>c5n17  python bench.py --workload c5rows --profiled
#   <tag>c4n801 python bench.py --workload c4rows --c4-nt 801 --row-stride 25 --profiled (the default
#               line's config4_horizon_sample block; no MFMA pass, to fit one call)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${TAG:-r05}
for w in ${@:-c1 c4 c5}; do
  case $w in
    c1) bash $R/tools/prof_passes.sh $T --no-cpu-baseline --no-slices --steps 5 --warmup 1 || exit $? ;;
    c4) PREP_ARGS="--workload c4rows --prepare-only --state-cache /tmp/ocg_c4.npz" \
        bash $R/tools/prof_passes.sh ${T}c4n33 --workload c4rows --steps 1 --warmup 1 --profiled --state-cache /tmp/ocg_c4.npz || exit $? ;;
    c4l) PREP_ARGS="--workload c4rows --prepare-only --state-cache /tmp/ocg_c4.npz" \
        bash $R/tools/prof_passes.sh ${T}c4n129 --workload c4rows --c4-nt 129 --steps 1 --warmup 1 --profiled --state-cache /tmp/ocg_c4.npz || exit $? ;;
    c4h) PREP_ARGS="--workload c4rows --prepare-only --state-cache /tmp/ocg_c4.npz" PROF_TMO=420 PMC_TMO=360 PROF_MFMA=0 \
        bash $R/tools/prof_passes.sh ${T}c4n801 --workload c4rows --c4-nt 801 --row-stride 25 --steps 1 --warmup 0 --profiled --state-cache /tmp/ocg_c4.npz || exit $? ;;
    c5) PREP_ARGS="--workload c5rows --prepare-only --state-cache /tmp/ocg_c5.npz" \
        bash $R/tools/prof_passes.sh ${T}c5n17 --workload c5rows --steps 1 --warmup 0 --profiled --state-cache /tmp/ocg_c5.npz || exit $? ;;
  esac
  echo "profiled $w"
done
