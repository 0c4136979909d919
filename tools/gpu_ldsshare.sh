# multi-control getHessian rows/s around the two-chains-per-CU threshold (OCG_MULTI_SHARE_K, default 8)
set -o pipefail
mkdir -p gpurun_out
for k in 4 8 16; do
  timeout -k 10 300 python bench.py --multi $k --no-cpu-baseline > gpurun_out/ls_$k.log 2>&1 || exit $?
  echo "K=$k $(tail -1 gpurun_out/ls_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), round(d["ms_per_step"], 2))')"
done
