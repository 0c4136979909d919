# register eigenvalue kernel with and without its bisection (HBM_NO_BISECT timing build)
set -o pipefail
mkdir -p gpurun_out
( for a in "192 1 64" "128 1 64" "96 1 32" "192 64 64"; do timeout -k 5 60 ./tools/build/eig_bench $a && timeout -k 5 60 ./tools/build/eig_bench_nb $a || exit 1; done ) > gpurun_out/eigbis.log 2>&1; echo rc=$?
