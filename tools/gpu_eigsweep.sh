# eigensolver kernels on random Gram blocks: vals / vecs(+bt) time and residuals per (n, batch, kept)
set -o pipefail
mkdir -p gpurun_out
( for a in "192 1 64" "192 1 100" "224 1 64" "256 1 128" "320 1 64" "448 1 40" "448 1 64" "448 1 128" "448 1 200" "512 1 128" "448 32 128" "300 48 100"; do timeout -k 5 120 ./tools/build/eig_bench $a || exit 1; done ) > gpurun_out/eigsweep.log 2>&1; echo rc=$?
