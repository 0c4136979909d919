# phase stamps of the large-order eigenvalue kernel, then the timing sweep
set -o pipefail
mkdir -p gpurun_out
( timeout -k 5 120 ./tools/build/eig_bench_st 448 1 64 ) > gpurun_out/eig_st.log 2>&1 && bash tools/gpu_eigsweep.sh; echo rc=$?
