#!/bin/bash
# c4rows with GPU_MAX_HW_QUEUES 4 vs 8 (the pipelined getHessian's three streams + torch's)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --workload c4rows --steps 2 --warmup 1 > gpurun_out/c4q$q.json 2> gpurun_out/c4q$q.err || { tail -5 gpurun_out/c4q$q.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c4q$q.json')); print('HWQ=$q', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['single_chain_steps_per_sec'])"
done
