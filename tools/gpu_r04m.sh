#!/bin/bash
# round 4: stream-priority modes 1 / 3 (and 0 / 2) on c4rows and c5rows, with and without the state cache
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload c4rows --prepare-only --state-cache /tmp/c4.npz > /dev/null 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c5rows --prepare-only --state-cache /tmp/c5.npz > /dev/null 2>&1 || exit 1
run() {  # workload mode cache
  if [ $3 = 1 ]; then C="--state-cache /tmp/$1.npz"; else C=""; fi
  if [ $1 = c4 ]; then W="--workload c4rows --steps 3 --warmup 1"; else W="--workload c5rows --steps 1 --warmup 1"; fi
  OCG_HBM_PRIO=$2 timeout -k 10 300 python -u bench.py $W --no-cpu-baseline $C > gpurun_out/r04m.json 2>/dev/null || exit 1
  python -c "import json; a=json.load(open('gpurun_out/r04m.json')); print('$1 prio $2 cache $3', round(a['ms_per_step'],1), 'ms')"
}
for m in 3 1; do for c in 1 0; do run c4 $m $c; run c5 $m $c; done; done
run c5 0 0
run c5 2 0
run c4 3 0
run c4 3 1
