#!/bin/bash
# round 4: k_gemm prefetch depth A/B (bitwise check + c4rows timing at N_t = 33 and 129), full GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for pd in 1 2 4; do OCG_HBM_GEMM_PD=$pd timeout -k 10 300 python -u tools/gemm_pd_check.py || exit 1; done
python -c "
import numpy as np
a=np.load('gpurun_out/gemm_pd1.npy')
for pd in (2,4):
    b=np.load(f'gpurun_out/gemm_pd{pd}.npy'); print('pd', pd, 'bitwise equal to pd1:', a.shape == b.shape and np.array_equal(a, b))
"
timeout -k 10 300 python -u bench.py --workload c4rows --prepare-only --state-cache /tmp/c4.npz > /dev/null 2>&1 || exit 1
for rep in 1 2; do for pd in 1 4 2; do
  OCG_HBM_GEMM_PD=$pd timeout -k 10 300 python -u bench.py --workload c4rows --steps 3 --warmup 1 --no-cpu-baseline --state-cache /tmp/c4.npz > gpurun_out/r04e_c4_$pd.json 2>/dev/null || exit 1
  python -c "import json; b=json.load(open('gpurun_out/r04e_c4_$pd.json')); print('N_t=33 pd $pd', round(b['ms_per_step'],1), 'ms', 'gemm avg us', round(b['mfma_gemm']['avg_launch_ms']*1e3,2), 'frac', round(b['roofline']['frac'],3))"
done; done
for pd in 1 4; do
  OCG_HBM_GEMM_PD=$pd timeout -k 10 300 python -u bench.py --workload c4rows --c4-nt 129 --steps 1 --warmup 1 --no-cpu-baseline --state-cache /tmp/c4.npz > gpurun_out/r04e_c4l_$pd.json 2>/dev/null || exit 1
  python -c "import json; b=json.load(open('gpurun_out/r04e_c4l_$pd.json')); print('N_t=129 pd $pd', round(b['ms_per_step'],1), 'ms', 'gemm avg us', round(b['mfma_gemm']['avg_launch_ms']*1e3,2), 'frac', round(b['roofline']['frac'],3))"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r04e_tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|c5 w512" gpurun_out/r04e_tests.log | tail -20
tail -2 gpurun_out/r04e_tests.log
exit $rc
