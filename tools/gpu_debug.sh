cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/gpu_debug.py > gpurun_out/debug.log 2>&1
echo "exit $?"
