#!/bin/bash
# k_gemm A/B: the in-tree library (A) and ab/libprev.so (B): HBM-engine GPU tests on A,
# GEMM histograms (N_t = 33, 129) and c4rows timing for each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_config4.py tests/test_checkpoint.py tests/test_config5.py tests/test_eigensolver_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests_A.log 2>&1 || { tail -30 gpurun_out/ab_tests_A.log; exit 1; }
echo "A tests: $(tail -1 gpurun_out/ab_tests_A.log)"
for v in A B A B; do
  if [ $v = B ]; then export OCG_LIB=$PWD/ab/libprev.so; else unset OCG_LIB; fi
  for nt in 33 129; do
    OCG_GEMM_STATS=1 timeout -k 10 400 python -u bench.py --workload c4rows --c4-nt $nt --steps 1 --warmup 0 > gpurun_out/gs_${v}$nt.json 2> gpurun_out/gs_${v}$nt.err || { tail -5 gpurun_out/gs_${v}$nt.err; exit 1; }
    echo "== $v N_t=$nt"; grep -E "^\[gemm\] (launches|>=512|<512|<32 )" gpurun_out/gs_${v}$nt.err | grep -v tasks/launch
  done
  timeout -k 10 300 python -u bench.py --workload c4rows --steps 3 --warmup 1 > gpurun_out/ab_c4rows_$v.json 2> gpurun_out/ab_c4rows_$v.err || { tail -5 gpurun_out/ab_c4rows_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_c4rows_$v.json')); r=d['roofline']; print('$v c4rows', round(d['ms_per_step'],1), 'ms', 'gemm frac', r.get('frac'), 'avg launch ms', r.get('avg_launch_ms'))"
done
