"""Steps of the HBM engine from a saved state (config-4 chain by default), for
rocprofv3.  usage: python tools/hbm_prof.py state.npz chi nsteps [nchains]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from optimalcontrolmps_amd.native import MPS, Engine  # noqa: E402

path, chi, nsteps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
nch = int(sys.argv[4]) if len(sys.argv) > 4 else 1
L, p, N = 20, 7, 20
z = np.load(path)
m = MPS(L, p, N, z["dims"], z["data"])
eng = Engine(L, p, N, 1.0, 0.005, 1e-8, chi, engine="hbm")
rng = np.random.default_rng(1)
if nch == 1:
    m2 = eng.steps(m, np.full(2, 2.5), True)  # warm
    t = time.time()
    m2 = eng.steps(m, rng.uniform(2, 10, nsteps + 1), True)
    el = time.time() - t
else:
    ms = [m] * nch
    ms = eng.step_batch(ms, np.full(nch, 2.5), np.full(nch, 3.0))
    t = time.time()
    for s in range(nsteps):
        ms = eng.step_batch(ms, rng.uniform(2, 10, nch), rng.uniform(2, 10, nch))
    el = time.time() - t
print(f"{nch} chains x {nsteps} steps: {1e3 * el / nsteps:.1f} ms per batched step, "
      f"{nch * nsteps / el:.2f} sweep-steps/s", flush=True)
g = eng.stats(7)
print(f"gemm: {g['ms']:.1f} ms in {g['launches']} launches, {g['alg_flops'] / max(g['ms'], 1e-9) / 1e9:.2f} TF/s",
      flush=True)
