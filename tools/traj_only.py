"""Diagnostic: k_trajectory alone (config 1, 2 chains x 200 steps, 5 launches),
the command the I-cache / issue PMC passes of tools/pmc_traj.sh profile."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
from optimalcontrolmps_amd import ed
from optimalcontrolmps_amd.native import MPS, Engine
L, p, Q, J, dt = 5, 5, 5, 1.0, 0.01
ini = MPS(L, p, Q, *ed.mps_from_full(ed.ground_state_full(L, p, Q, J, 2.5)[0], L, p, Q))
tgt = MPS(L, p, Q, *ed.mps_from_full(ed.ground_state_full(L, p, Q, J, 50.0)[0], L, p, Q))
eng = Engine(L, p, Q, J, dt, 1e-8, 80)
eng.set_states(tgt, ini)
u = np.random.default_rng(20261015).uniform(2, 10, 201)
for _ in range(5):
    eng.propagate(u, 3)
st = eng.stats(0)
print("trajectory ms/launch", st["ms"] / max(1, st["launches"]), "fast chain", eng.info.fast_chain)
