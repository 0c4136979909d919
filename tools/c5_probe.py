"""Config-5 feasibility probe (HBM engine): L=50 Npart=50 d=8 (p=9) chi=512
dt=0.01, product state |1..1> warmed up at U=2.5 in chunks; prints the time
per chunk and the bond dimensions, stops at a wall-clock budget."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from optimalcontrolmps_amd.native import Engine  # noqa: E402
from optimalcontrolmps_amd.states import product_state  # noqa: E402

L, p, Q, dt, maxm = 50, 9, 50, 0.01, 512
budget = float(sys.argv[1]) if len(sys.argv) > 1 else 300.0
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 10
eng = Engine(L, p, Q, 1.0, dt, 1e-8, maxm, engine="hbm")
psi = product_state(L, p, Q)
t0 = time.time()
done = 0
while time.time() - t0 < budget:
    t1 = time.time()
    psi = eng.steps(psi, np.full(chunk + 1, 2.5), True)
    done += chunk
    bd = psi.bond_dims()
    print(f"steps {done}: {1e3 * (time.time() - t1) / chunk:.1f} ms/step, max bond {bd.max()}, "
          f"mid bonds {list(bd[20:30])}, nelem {len(psi.data)}", flush=True)
    if bd.max() >= maxm and chunk < 50:
        pass
print("total", time.time() - t0, "s")
