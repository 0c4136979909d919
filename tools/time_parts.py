"""Diagnostic: wall time of the product kernels at config 1 (median of 7).

trajectory = psi and xi chains alone (200 steps each, concurrent): the
single-chain step latency on an otherwise idle GPU; pipeline = one full
ocg_hessian (rows start as psi_i is published), whose critical path is
~N_t - 2 steps of one chain plus one apply_dH."""
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
tr, pl, ro = [], [], []
for k in range(8):
    eng.reset_stats()
    eng.propagate(u, 3)
    t = eng.stats(0)["ms"]
    eng.hessian(u)
    if k:
        tr.append(t)
        pl.append(eng.stats(5)["ms"])
        ro.append(eng.stats(6)["ms"])
tm, pm, rm = np.median(tr), np.median(pl), np.median(ro)
print(f"trajectory {tm:.3f} ms ({1e3 * tm / 200:.1f} us/step)  pipeline {pm:.3f} ms  row_overlaps {rm:.3f} ms  "
      f"pipeline/trajectory {pm / tm:.3f}")
# critical-path probe: the pipeline with row subsets (row 1 is the longest)
for rows in ([1], list(range(1, 200, 8)), list(range(1, 200, 2)), list(range(1, 200))):
    ts = []
    for k in range(5):
        eng.reset_stats()
        eng.hessian(u, rows)
        ts.append(eng.stats(5)["ms"])
    print(f"pipeline with {len(rows):3d} rows: {np.median(ts):.3f} ms")
