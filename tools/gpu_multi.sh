# config-1 rows/s with K control vectors per GPU in one ocg_hessian_multi launch (K = 1..4, 8)
set -o pipefail
mkdir -p gpurun_out
for k in 1 2 3 4 8; do
  timeout -k 10 300 python bench.py --multi $k --no-cpu-baseline > gpurun_out/multi_$k.log 2>&1 || exit $?
  echo "K=$k $(tail -1 gpurun_out/multi_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 2), round(d["kernels"]["pipeline"]["avg_ms"], 2))')"
done
