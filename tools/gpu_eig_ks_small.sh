# multisection shifts per thread for small orders (g >= 4 threads per eigenvalue): EIG_KS=1 vs 4
set -o pipefail
mkdir -p gpurun_out
cd gpurun_out
(
for a in "64 1 40 16" "48 1 30 16" "32 1 20 16" "24 1 16 16" "64 64 40 16"; do
  for K in 4 1 4 1; do echo "KS=$K $a"; EIG_KS=$K timeout -k 5 60 ../tools/bin/eig_bench_lds $a | cut -c1-120 || exit 1; done
done
) > eig_ks_small.log 2>&1; rc=$?; cat eig_ks_small.log; exit $rc
