#!/bin/bash
# config-4 shape statistics: GEMM launch/shape histogram and Gram-block order
# histogram of one c4rows getHessian (OCG_GEMM_STATS), then the eigensolver
# latency per order at config-4 batch sizes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OCG_GEMM_STATS=1 timeout -k 10 300 python -u bench.py --workload c4rows --steps 1 --warmup 0 > gpurun_out/c4stats.json 2> gpurun_out/c4stats.err || { tail -5 gpurun_out/c4stats.err; exit 1; }
grep -E "^\[gemm\]|^\[eig\]" gpurun_out/c4stats.err | head -60
( for a in "32 256 32" "64 256 64" "96 128 96" "128 64 128" "160 64 100" "192 64 100" "256 32 128"; do timeout -k 5 120 ./tools/build/eig_bench $a || exit 1; done ) > gpurun_out/eigsizes.log 2>&1 || exit 1
grep "^n=" gpurun_out/eigsizes.log
