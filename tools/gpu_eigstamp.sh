# phase stamps of the eigensolver kernels (HBM_STAMP build of tools/eig_bench)
set -o pipefail
mkdir -p gpurun_out
( for a in "192 1 64" "128 1 32" "448 1 64"; do timeout -k 5 120 ./tools/build/eig_bench_st $a || exit 1; done ) > gpurun_out/eig_st.log 2>&1; echo rc=$?
