# c4rows A/B of the split multisection: chunk size and threshold
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --workload c4rows --steps 2 --warmup 1 --no-cpu-baseline --state-cache /tmp/c4s.npz"
timeout -k 10 200 $B > gpurun_out/c4_s16_96.json 2> /dev/null || exit 1
OCG_HBM_SPLIT_SPE=8 timeout -k 10 200 $B > gpurun_out/c4_s8_96.json 2> /dev/null || exit 1
OCG_HBM_SPLIT_SPE=32 timeout -k 10 200 $B > gpurun_out/c4_s32_96.json 2> /dev/null || exit 1
OCG_HBM_SPLITMIN=64 timeout -k 10 200 $B > gpurun_out/c4_s16_64.json 2> /dev/null || exit 1
OCG_HBM_SPLITMIN=48 OCG_HBM_SPLIT_SPE=8 timeout -k 10 200 $B > gpurun_out/c4_s8_48.json 2> /dev/null || exit 1
timeout -k 10 200 $B > gpurun_out/c4_s16_96b.json 2> /dev/null || exit 1
