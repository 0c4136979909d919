# GPU round-trip: smoke -> parity tests -> short bench -> phase profile.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
make -s -C oracle &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q -rf --tb=short > gpurun_out/pytest.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1 && echo "bench ok" &&
timeout -k 10 300 python tools/time_parts.py > gpurun_out/parts.log 2>&1 && echo "parts ok"
