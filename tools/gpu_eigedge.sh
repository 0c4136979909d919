# eigensolver edge cases: rank-deficient Gram blocks (reduced columns, tau = 0) on every path
set -o pipefail
mkdir -p gpurun_out
( for a in "448 1 30 16 0 40" "300 2 60 16 0 20" "256 1 64 16 0 1" "192 1 40 16 0 10" "209 1 64 16 0 209" "512 1 100 16 0 100"; do timeout -k 5 120 ./tools/build/eig_bench $a || exit 1; done ) > gpurun_out/eigedge.log 2>&1; echo rc=$?
