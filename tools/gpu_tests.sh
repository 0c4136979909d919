set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
make -s -C oracle
timeout -k 10 600 python -m pytest tests -m gpu -q -rf --tb=line > gpurun_out/pytest.log 2>&1
echo "pytest exit $?"
