#!/bin/bash
# GEMM launch/shape histograms (OCG_GEMM_STATS) of one c4rows getHessian at N_t = 33 and 129
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for nt in 33 129; do
  OCG_GEMM_STATS=1 timeout -k 10 400 python -u bench.py --workload c4rows --c4-nt $nt --steps 1 --warmup 0 > gpurun_out/gstats$nt.json 2> gpurun_out/gstats$nt.err || { tail -5 gpurun_out/gstats$nt.err; exit 1; }
  echo "== N_t=$nt"; grep -E "^\[gemm\]" gpurun_out/gstats$nt.err
done
