# multisection shifts per thread: EIG_KS=1 (bisection) vs 4 (round 5), register kernel
set -o pipefail
mkdir -p gpurun_out
cd gpurun_out
(
for a in "192 1 64" "128 1 64" "96 1 32" "192 32 64"; do
  for K in 4 1; do echo "KS=$K $a"; EIG_KS=$K timeout -k 5 60 ../tools/bin/eig_bench $a | cut -c1-150 || exit 1; done
done
) > eig11.log 2>&1; rc=$?; cat eig11.log; exit $rc
