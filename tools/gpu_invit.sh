# inverse iteration A/B (eig_bench): division sweeps, 3 iterations (eig_bench) vs stored reciprocal pivots, 3 / 2 iterations
set -o pipefail
mkdir -p gpurun_out
cd gpurun_out
(
for a in "192 1 64" "128 1 64" "96 1 32" "192 32 64" "64 1 40"; do
  for B in eig_bench eig_bench_rcp3 eig_bench_rcp2; do echo "$B $a"; timeout -k 5 60 ../tools/bin/$B $a | cut -c1-170 || exit 1; done
done
) > invit.log 2>&1; rc=$?; cat invit.log; exit $rc
