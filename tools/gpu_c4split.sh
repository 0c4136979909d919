# c4rows A/B of the split multisection (OCG_HBM_SPLIT_WG: workgroups per CU it may use; SPLITMIN=0: off)
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --workload c4rows --steps 2 --warmup 1 --no-cpu-baseline --state-cache /tmp/c4s.npz"
for cfg in "OCG_HBM_SPLIT_WG=2" "OCG_HBM_SPLIT_WG=1000" "OCG_HBM_SPLITMIN=0" "OCG_HBM_SPLIT_WG=4" "OCG_HBM_SPLIT_WG=2"; do
  env $cfg timeout -k 10 200 $B > gpurun_out/c4ab_tmp.json 2> /dev/null || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/c4ab_tmp.json').read().strip().splitlines()[-1]); print('$cfg', round(d['ms_per_step'],1), round(d['single_chain_steps_per_sec'],2))" >> gpurun_out/c4ab.txt
done
