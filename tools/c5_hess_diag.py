"""Diagnostic (not a test): the chi = 512 fidelity Hessian vs central differences
of the analytic gradient, with the Maxm-512 warm state evolved under Maxm 512
(binding: the dH psi row states are compressed to 512) and under Maxm 1024
(the bond-doubled dH psi fits), at dt = 0.01 and 0.005, entry by entry."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from optimalcontrolmps_amd.native import Engine  # noqa: E402
from optimalcontrolmps_amd.states import product_state, warm_state  # noqa: E402

L, p, N, J, CUT = 50, 9, 50, 1.0, 1e-8
NT = 4
t0 = time.time()
e = Engine(L, p, N, J, 0.01, CUT, 512, engine="hbm")
ini = warm_state(e, product_state(L, p, N), 2.5, 230, chunk=10)
tgt = e.steps(ini, np.full(3, 6.0), True)
e.close()
print(f"warm {time.time() - t0:.0f} s", flush=True)
u = np.random.default_rng(51).uniform(2.0, 10.0, NT)
for maxm in (512, 1024):
    for dt in (0.01, 0.005):
        t0 = time.time()
        eng = Engine(L, p, N, J, dt, CUT, maxm, engine="hbm")
        eng.set_states(tgt, ini)
        H, divT, F = eng.hessian(u)

        def grad(v):
            eng.propagate(v, 3)
            return dt * (eng.div_t() * eng.overlap_factor() * 1j).real
        rel = np.zeros((2, 2))
        for j in (1, 2):
            up, um = u.copy(), u.copy()
            up[j] += 1e-3
            um[j] -= 1e-3
            col = (grad(up) - grad(um)) / 2e-3
            rel[:, j - 1] = (H[1:3, j] - col[1:3]) / col[1:3]
        print(f"maxm {maxm} dt {dt}: H {H[1:3, 1:3].ravel()} rel gap {rel.ravel()} ({time.time() - t0:.0f} s)",
              flush=True)
        eng.close()
