#!/bin/bash
# one rocprofv3 pass (prof | pmc_fetch | pmc_write) of a long bench command per GPU call:
#   tools/prof_one_pass.sh <kind> <tag> [bench args...]   (PREP_ARGS: an unprofiled preparation run first)
# writes gpurun_out/profiles_<tag>/<tag>_<kind>.json (tools/prof_summary.py --pass; merge with --merge)
set -o pipefail
KIND=$1; TAG=$2; shift 2
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
L=$R/gpurun_out/profiles_$TAG
D=/tmp/ocg_prof1_$TAG
rm -rf $D && mkdir -p $D $L
( while true; do date >> $L/heartbeat_$KIND.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ -n "$PREP_ARGS" ]; then
  timeout -k 10 ${PREP_TMO:-300} python3 $R/bench.py $PREP_ARGS > $L/prep_$KIND.log 2>&1 || exit $?
fi
case $KIND in
  prof) timeout -k 10 ${PASS_TMO:-900} rocprofv3 --kernel-trace --stats -d $D/prof -o run -- python3 $R/bench.py "$@" > $L/$KIND.log 2>&1 || exit $? ;;
  pmc_fetch) timeout -s KILL ${PASS_TMO:-900} rocprofv3 --pmc FETCH_SIZE -d $D/pmc_fetch -o run -- python3 $R/bench.py "$@" > $L/$KIND.log 2>&1 || exit $? ;;
  pmc_write) timeout -s KILL ${PASS_TMO:-900} rocprofv3 --pmc WRITE_SIZE -d $D/pmc_write -o run -- python3 $R/bench.py "$@" > $L/$KIND.log 2>&1 || exit $? ;;
esac
grep "\"metric\"" $L/$KIND.log | tail -1 | cut -c1-300
PROF_DB_ROOT=$D python3 -u $R/tools/prof_summary.py --pass $KIND $TAG $L/${TAG}_$KIND.json
src=$?
rm -rf $D
exit $src
