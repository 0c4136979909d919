#!/bin/bash
# config-1 phase profile (gauge-move share) and the config-5 slice line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OCG_PROF_NT=128 timeout -k 10 200 python -u tools/profile_phases.py > gpurun_out/phases.txt 2>&1 || { tail -5 gpurun_out/phases.txt; exit 1; }
cat gpurun_out/phases.txt | head -32
timeout -k 10 800 python -u bench.py --workload c5rows --steps 1 --warmup 1 > gpurun_out/c5.json 2> gpurun_out/c5.err
rc=$?; cut -c1-1500 gpurun_out/c5.json; tail -3 gpurun_out/c5.err; exit $rc
