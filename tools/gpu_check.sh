set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
make -s -C oracle
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke $?"
timeout -k 10 600 python -m pytest tests -m gpu -q -rf --tb=short > gpurun_out/pytest.log 2>&1; echo "pytest $?"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1; echo "bench $?"
