#!/bin/bash
# A/B of an environment switch on one bench command, alternated: tools/gpu_ab.sh VAR "a b" <bench args>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
var=$1; vals=$2; shift 2
for rep in 1 2; do
  for v in $vals; do
    env $var=$v timeout -k 10 300 python -u bench.py "$@" > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$var=$v', 'rep $rep', round(d['ms_per_step'],1), 'ms/step', round(d['value'],3), d['unit'])"
  done
done
