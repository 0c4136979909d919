#!/bin/bash
# rocprofv3 evidence for profiles/: kernel trace + stats, then FETCH_SIZE,
# WRITE_SIZE and the MFMA / issue counters, each pass a run of its own
# (MI355X_MICROARCH.md HBM/rocprofv3 recipe), all over the same bench command.
# The rocpd databases go to /tmp (gpurun_out/ must stay under 64 MiB); only the
# summaries and logs land in gpurun_out/profiles_<tag>.
# Usage: tools/prof_passes.sh <tag> [bench args...]   (PROF_TMO / PMC_TMO: per-pass time limits;
# PROF_MFMA=0: no MFMA / issue-counter pass; it is the slowest pass of large runs (its database
# generation), so a pass that runs out of time leaves the other passes' summaries intact)
TAG=${1:-r02}
shift
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
ARGS=${@:---no-cpu-baseline --steps 5 --warmup 1}
T1=${PROF_TMO:-300}
T2=${PMC_TMO:-240}
D=/tmp/ocg_prof_$TAG
rm -rf $D && mkdir -p $D $R/gpurun_out/profiles_$TAG
L=$R/gpurun_out/profiles_$TAG
# heartbeat: the profiler's database generation can run for minutes without output
( while true; do date >> $L/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
# PREP_ARGS: an unprofiled bench run first (e.g. --prepare-only --state-cache ...: the
# c4/c5 warm states), so the profiled command holds only the timed population
if [ -n "$PREP_ARGS" ]; then
  timeout -k 10 ${PREP_TMO:-300} python3 $R/bench.py $PREP_ARGS > $L/prep_$TAG.log 2>&1 || exit $?
fi
timeout -k 10 $T1 rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 $R/bench.py $ARGS > $L/prof_$TAG.log 2>&1 || exit $?
timeout -s KILL $T2 rocprofv3 --pmc FETCH_SIZE -d $D/pmc_fetch -o run -- python3 $R/bench.py $ARGS > $L/pmc_fetch_$TAG.log 2>&1 || exit $?
timeout -s KILL $T2 rocprofv3 --pmc WRITE_SIZE -d $D/pmc_write -o run -- python3 $R/bench.py $ARGS > $L/pmc_write_$TAG.log 2>&1 || exit $?
[ "${PROF_MFMA:-1}" = "0" ] || timeout -s KILL $T2 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE -d $D/pmc_mfma -o run -- python3 $R/bench.py $ARGS > $L/pmc_mfma_$TAG.log 2>&1 || echo "MFMA pass did not finish (the other passes are still summarised)"
grep "\"metric\"" $L/prof_$TAG.log | tail -1 | cut -c1-400
PROF_DB_ROOT=$D python3 -u $R/tools/prof_summary.py $TAG $L > $L/summary_stdout.txt 2>&1
src=$?
rm -rf $D
exit $src
