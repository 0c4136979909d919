cd $GRAFT_REPO_ROOT
timeout -k 10 600 python tools/profile_phases.py > gpurun_out/phases.log 2>&1
echo "exit $?"
