# dry run of bench.py's multi-rank path on one GPU: 2 ranks (gloo), weak and strong
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for mode in weak strong; do
  OCG_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --mode $mode \
    > gpurun_out/dist_$mode.log 2>&1 || { echo "dist $mode failed"; tail -20 gpurun_out/dist_$mode.log; exit 1; }
  grep '"metric"' gpurun_out/dist_$mode.log | cut -c1-330
done
