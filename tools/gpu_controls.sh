# rows/s with K concurrent control vectors per GPU (K contexts / streams / host threads)
set -o pipefail
cd $GRAFT_REPO_ROOT
for K in 1 2 3 4; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 6 --warmup 1 --controls $K > gpurun_out/ctl_$K.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/ctl_$K.log').read().strip().splitlines()[-1])
print('K=$K', round(d['value']), 'rows/s', round(d['ms_per_step'],2), 'ms/step')"
done
