#!/bin/bash
# config-4 row sharding: GPU tests of the HBM shards, a 2-rank gloo dry run of
# bench.py --workload c4rows --mode strong on one GPU, the 1-GPU c4rows line
# (GROUP M=40) and its rocprofv3 kernel trace + PMC passes (tag r03c4n33)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_config4.py -v --timeout 300 --timeout-method thread -k "shards or s32_vs" > gpurun_out/pytest_c4.log 2>&1 || { tail -30 gpurun_out/pytest_c4.log; exit 1; }
tail -3 gpurun_out/pytest_c4.log
OCG_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --workload c4rows --gpus 2 --steps 1 --warmup 1 \
  > gpurun_out/dist_c4.log 2>&1 || { echo "dist c4 failed"; tail -30 gpurun_out/dist_c4.log; exit 1; }
grep '"metric"' gpurun_out/dist_c4.log
timeout -k 10 400 python -u bench.py --workload c4rows --steps 2 --warmup 1 > gpurun_out/c4rows.json 2> gpurun_out/c4rows.err || { tail -20 gpurun_out/c4rows.err; exit 1; }
cat gpurun_out/c4rows.json
[ "$1" = "prof" ] && bash tools/profile_r02.sh r03c4n33 --workload c4rows --steps 1 --warmup 1
exit 0
