# full GPU suite (verbose, per-test timeout) + default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
make -s -C oracle
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > gpurun_out/pytest.log 2>&1
rc=$?
echo "pytest exit $rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log
