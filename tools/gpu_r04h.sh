#!/bin/bash
# round 4: config-5 profile re-taken on the pipelined getHessian (the path the c5rows line runs)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 bash tools/profile_r04.sh c5 > gpurun_out/r04h_prof.log 2>&1 || { tail -20 gpurun_out/r04h_prof.log; exit 1; }
tail -6 gpurun_out/r04h_prof.log
