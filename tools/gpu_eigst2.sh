#!/bin/bash
# eigensolver latency per order (B = 1) and orthogonalisation phase stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( for a in "32 1 32" "64 1 64" "96 1 96" "128 1 128" "192 1 100" "160 1 64" "32 256 32" "96 128 96"; do timeout -k 5 60 ./tools/build/eig_bench $a || exit 1; done
  for a in "96 1 96" "192 1 100"; do timeout -k 5 60 ./tools/build/eig_bench_st $a || exit 1; done ) > gpurun_out/eigst2.log 2>&1
rc=$?; grep -v "^stamps\|^vecs stamps" gpurun_out/eigst2.log | grep -v "vecs slow" ; grep "vecs slow" gpurun_out/eigst2.log | tail -2; exit $rc
