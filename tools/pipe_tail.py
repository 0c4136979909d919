"""Config-1 pipeline tail: k_pipeline time with no rows, with only the last
rows, and with all 199 rows (where the time after the psi chain goes)."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from optimalcontrolmps_amd import ed
from optimalcontrolmps_amd.native import MPS, Engine

L, p, N, J, dt, cut, maxm = 5, 5, 5, 1.0, 0.01, 1e-8, 80
Nt = 201
ini = MPS(L, p, N, *ed.mps_from_full(ed.ground_state_full(L, p, N, J, 2.5)[0], L, p, N))
tgt = MPS(L, p, N, *ed.mps_from_full(ed.ground_state_full(L, p, N, J, 50.0)[0], L, p, N))
u = np.random.default_rng(20261015).uniform(2.0, 10.0, Nt)
eng = Engine(L, p, N, J, dt, cut, maxm, device=0)
eng.set_states(tgt, ini)
for name, rows in [("none", []), ("last1", [Nt - 2]), ("last8", list(range(Nt - 9, Nt - 1))),
                   ("first1", [1]), ("all", list(range(1, Nt - 1)))]:
    ts = []
    for rep in range(4):
        eng.reset_stats()
        eng.hessian(u, rows)
        ts.append(eng.stats(5)["ms"])
    print(f"{name:7s} k_pipeline ms: " + " ".join(f"{t:.3f}" for t in ts[1:]), flush=True)
t = []
for rep in range(4):
    eng.reset_stats()
    eng.propagate(u, 3)
    t.append(eng.stats(0)["ms"])
print("trajectory (psi || xi, k_trajectory) ms: " + " ".join(f"{x:.3f}" for x in t[1:]))
