#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OCG_PIPE_DEBUG=1 timeout -k 5 100 python -u -m pytest tests/test_config4.py -x -v -s -k pipelined --timeout 90 --timeout-method thread > gpurun_out/pipedbg.log 2>&1
rc=$?; tail -60 gpurun_out/pipedbg.log; exit $rc
