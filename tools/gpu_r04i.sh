#!/bin/bash
# round 4: config 4 at its BASELINE horizon on one GPU: the full getHessian (N_t = 801, 799 rows,
# GROUP M = 40) and the gradient (N_t = 801), one step each (heartbeat lines on stderr every minute)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# stream priorities A/B (OCG_HBM_PRIO=1: the context engine and the dH worker high, the xi worker low)
timeout -k 10 300 python -u bench.py --workload c4rows --prepare-only --state-cache /tmp/c4.npz > /dev/null 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c5rows --prepare-only --state-cache /tmp/c5.npz > /dev/null 2>&1 || exit 1
for rep in 1 2; do for pr in 0 1; do
  OCG_HBM_PRIO=$pr timeout -k 10 300 python -u bench.py --workload c4rows --steps 3 --warmup 1 --no-cpu-baseline --state-cache /tmp/c4.npz > gpurun_out/r04i_c4_$pr.json 2>/dev/null || exit 1
  OCG_HBM_PRIO=$pr timeout -k 10 300 python -u bench.py --workload c5rows --steps 1 --warmup 1 --no-cpu-baseline --state-cache /tmp/c5.npz > gpurun_out/r04i_c5_$pr.json 2>/dev/null || exit 1
  python -c "import json; a=json.load(open('gpurun_out/r04i_c4_$pr.json')); b=json.load(open('gpurun_out/r04i_c5_$pr.json')); print('prio $pr c4rows', round(a['ms_per_step'],1), 'ms  c5rows', round(b['ms_per_step'],1), 'ms')"
done; done
timeout -k 10 300 python -u bench.py --workload c4grad --steps 1 --warmup 0 > gpurun_out/r04i_c4grad.json 2> gpurun_out/r04i_c4grad.err || { tail -5 gpurun_out/r04i_c4grad.err; exit 1; }
cut -c1-300 gpurun_out/r04i_c4grad.json
timeout -k 10 900 python -u bench.py --workload c4rows --c4-nt 801 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04i_c4full.json 2> gpurun_out/r04i_c4full.err || { tail -5 gpurun_out/r04i_c4full.err; exit 1; }
cut -c1-400 gpurun_out/r04i_c4full.json
