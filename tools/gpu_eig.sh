set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( for n in 64 192; do timeout -k 5 60 ./tools/eig_bench_st $n 1 5 || exit 1; timeout -k 5 60 ./tools/eig_bench_st $n 1 46 || exit 1; done ) > gpurun_out/eig12.log 2>&1; echo rc=$?
