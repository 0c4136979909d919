#!/bin/bash
# round 4: c4rows / c5rows stream-priority modes (1 high+low, 2 low only, 0 off) with and without the state cache, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload c4rows --prepare-only --state-cache /tmp/c4.npz > /dev/null 2>&1 || exit 1
for rep in 1 2; do for pr in 1 2 0; do for cache in 1 0; do
  if [ $cache = 1 ]; then C="--state-cache /tmp/c4.npz"; else C=""; fi
  OCG_HBM_PRIO=$pr timeout -k 10 300 python -u bench.py --workload c4rows --steps 3 --warmup 1 --no-cpu-baseline $C > gpurun_out/r04k.json 2>/dev/null || exit 1
  python -c "import json; a=json.load(open('gpurun_out/r04k.json')); print('prio $pr cache $cache', round(a['ms_per_step'],1), 'ms gemm', round(a['mfma_gemm']['avg_launch_ms']*1e3,1), 'us')"
done; done; done
