# c4rows N_t = 129 (127 rows: larger batches) A/B of the split multisection
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --workload c4rows --c4-nt 129 --steps 1 --warmup 1 --no-cpu-baseline --state-cache /tmp/c4s.npz"
for cfg in "OCG_HBM_SPLIT_WG=2" "OCG_HBM_SPLITMIN=0" "OCG_HBM_SPLIT_WG=1000" "OCG_HBM_SPLIT_WG=2"; do
  env $cfg timeout -k 10 200 $B > gpurun_out/c4ab_tmp.json 2> /dev/null || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/c4ab_tmp.json').read().strip().splitlines()[-1]); print('$cfg', round(d['ms_per_step'],1), round(d['single_chain_steps_per_sec'],2))" >> gpurun_out/c4ab129.txt
done
