set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( for n in 20 40 64 100 150 192 208; do timeout -k 5 60 ./tools/eig_bench13 $n 1 5 || exit 1; timeout -k 5 60 ./tools/eig_bench13 $n 1 32 || exit 1; done; timeout -k 5 60 ./tools/eig_bench13 192 1 64 || exit 1 ) > gpurun_out/eig8.log 2>&1; echo rc=$?
