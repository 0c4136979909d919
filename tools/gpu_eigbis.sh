# eigensolver timing: multisection inside the reduction kernels (eig_bench_old) vs k_heev_bisect
set -o pipefail
mkdir -p gpurun_out
( for a in "128 300 32" "192 300 64" "96 600 32" "160 256 48"; do timeout -k 5 60 ./tools/build/eig_bench_old $a && timeout -k 5 60 ./tools/build/eig_bench $a || exit 1; done ) > gpurun_out/eigbis.log 2>&1; echo rc=$?
