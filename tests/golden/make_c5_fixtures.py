"""Config-5 fixtures (TEST INFRASTRUCTURE): BASELINE configs[4]'s chain shape
(L=50, Npart=50, d=8 -> p=9, tstep=0.01, cutoff 1e-8) on the CPU oracle,
with Maxm = 16 (binding) so the oracle finishes in seconds:
  psi_init = the Mott state |1..1> evolved 100 steps at U = 2.5 (oracle),
  psi_target = psi_init evolved 20 more steps at U = 6, N_t = 5 GRAPE
  controls U(2,10) (seed 5050): divT, F, gradient, the full fidelity Hessian
  (rows 1..3), fidelities.
Run: python tests/golden/make_c5_fixtures.py
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle_ffi as O  # noqa: E402
from optimalcontrolmps_amd.states import product_state  # noqa: E402

L, p, N, J, DT, CUT, MAXM, NT = 50, 9, 50, 1.0, 0.01, 1e-8, 16, 5
OUT = os.path.join(HERE, "c5.npz")

if __name__ == "__main__":
    st = O.Stepper(L, p, N, J, DT, CUT, MAXM)
    mott = product_state(L, p, N)
    t0 = time.time()
    psi = st.steps(O.MPS(L, p, N, mott.dims, mott.data), np.full(101, 2.5), True)
    print(f"warm-up: bonds {list(psi.bond_dims())} ({time.time() - t0:.1f}s)", flush=True)
    tgt = st.steps(psi, np.full(21, 6.0), True)
    u = np.random.default_rng(5050).uniform(2.0, 10.0, NT)
    oc = O.OC(st, tgt, psi, NT, 0.0)
    t0 = time.time()
    H = oc.hessian(u, 8)
    g = oc.gradient(u)
    divT, F = oc.divT_F()
    fid = oc.fidelities(u)
    print(f"oracle hessian+gradient {time.time() - t0:.1f}s max|H| {np.abs(H).max():.3e} max|g| {np.abs(g).max():.3e}"
          f" |F| {abs(F):.3e}", flush=True)
    np.savez_compressed(OUT, init_dims=psi.dims, init_data=psi.data, tgt_dims=tgt.dims, tgt_data=tgt.data, u=u,
                        H=H, grad=g, divT=divT, F=np.array([F]), fid=fid, maxm=np.array(MAXM))
