"""Diagnostic: k_trajectory alone (psi and xi chains, 200 steps each), 5 launches."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from optimalcontrolmps_amd import ed
from optimalcontrolmps_amd.native import MPS, Engine
L, p, Q, J, dt = 5, 5, 5, 1.0, 0.01
ini = MPS(L, p, Q, *ed.mps_from_full(ed.ground_state_full(L, p, Q, J, 2.5)[0], L, p, Q))
tgt = MPS(L, p, Q, *ed.mps_from_full(ed.ground_state_full(L, p, Q, J, 50.0)[0], L, p, Q))
eng = Engine(L, p, Q, J, dt, 1e-8, 80)
u = np.random.default_rng(20261015).uniform(2, 10, 201)
eng.set_states(tgt, ini)
for k in range(5):
    eng.propagate(u, 3)
print("trajectory ms/launch", eng.stats(0)["ms"] / 5)
