"""Fixture input (run on the GPU box): a chi = 512 saturated state of config
5's local dimension on a chain short enough for one oracle step on the CPU
(L = 12, Npart = 12, p = 9, tstep = 0.01, cutoff 1e-8, Maxm 512): the Mott
state evolved at U = 2.5 on the HBM engine until the middle bonds reach 512.
Writes gpurun_out/c5L12_warm.npz (dims, data); tests/golden/make_c5_fixtures.py
w512 then takes one oracle step from it."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from optimalcontrolmps_amd.native import Engine  # noqa: E402
from optimalcontrolmps_amd.states import product_state, warm_state  # noqa: E402

L, p, N, J, DT, CUT, MAXM = 12, 9, 12, 1.0, 0.01, 1e-8, 512
eng = Engine(L, p, N, J, DT, CUT, MAXM, engine="hbm")
psi = product_state(L, p, N)
t0 = time.time()
steps = 0
while steps < 600:
    psi = warm_state(eng, psi, 2.5, 20, chunk=20)
    steps += 20
    b = psi.bond_dims()
    print(f"{steps} steps {time.time() - t0:.0f} s bonds {list(b)}", flush=True)
    if (b == MAXM).sum() >= 3:
        break
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "c5L12_warm.npz"), dims=psi.dims, data=psi.data, steps=steps)
print("size MB", psi.data.nbytes / 1e6)
