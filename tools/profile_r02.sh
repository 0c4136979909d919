#!/bin/bash
# rocprofv3 evidence for profiles/: kernel trace + stats, then FETCH_SIZE,
# WRITE_SIZE and the MFMA / issue counters, each pass a run of its own
# (MI355X_MICROARCH.md HBM/rocprofv3 recipe), all over the same bench command.
# Usage: tools/profile_r02.sh <tag> [bench args...]
TAG=${1:-r02}
shift
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
ARGS=${@:---no-cpu-baseline --steps 5 --warmup 1}
rm -rf $R/gpurun_out/prof_$TAG $R/gpurun_out/pmc_fetch_$TAG $R/gpurun_out/pmc_write_$TAG $R/gpurun_out/pmc_mfma_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof_$TAG.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_$TAG -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc_fetch_$TAG.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_$TAG -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc_write_$TAG.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_mfma_$TAG -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc_mfma_$TAG.log 2>&1 || exit $?
grep "\"metric\"" $R/gpurun_out/prof_$TAG.log | tail -1
# summarise on the box (the rocpd databases are too large to bring back) and
# keep the stats CSVs of rocprofv3 --stats next to the summary
mkdir -p $R/gpurun_out/profiles_$TAG
python3 $R/tools/prof_summary.py $TAG $R/gpurun_out/profiles_$TAG > $R/gpurun_out/profiles_$TAG/summary_stdout.txt 2>&1
cp $R/gpurun_out/prof_$TAG.log $R/gpurun_out/profiles_$TAG/ 2>/dev/null
rm -rf $R/gpurun_out/prof_$TAG $R/gpurun_out/pmc_fetch_$TAG $R/gpurun_out/pmc_write_$TAG $R/gpurun_out/pmc_mfma_$TAG
