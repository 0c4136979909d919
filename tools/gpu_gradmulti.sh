# config-2 gradients/s with K control vectors per call (ocg_gradient_multi)
set -o pipefail
mkdir -p gpurun_out
for k in 1 8 32 64; do
  timeout -k 10 300 python bench.py --workload gradient --multi $k --no-cpu-baseline > gpurun_out/gm_$k.log 2>&1 || exit $?
  echo "K=$k $(tail -1 gpurun_out/gm_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"], 1), round(d["ms_per_step"], 2))')"
done
