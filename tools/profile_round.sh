#!/bin/bash
# rocprofv3 evidence for profiles/: kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE in passes of their own (MI355X_MICROARCH.md HBM/rocprofv3 recipe),
# all over the same bench command.  Usage: tools/profile_round.sh <tag>
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 1"
rm -rf $R/gpurun_out/prof_$TAG $R/gpurun_out/pmc_fetch_$TAG $R/gpurun_out/pmc_write_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run -- $CMD > $R/gpurun_out/prof_$TAG.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch_$TAG -o run -- $CMD > $R/gpurun_out/pmc_fetch_$TAG.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write_$TAG -o run -- $CMD > $R/gpurun_out/pmc_write_$TAG.log 2>&1 || exit $?
cd $R && find gpurun_out/prof_$TAG gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG -maxdepth 3 | head -20
grep '"metric"' gpurun_out/prof_$TAG.log | tail -1
