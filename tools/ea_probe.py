"""Localise the host crash of test_engines_agree (prints progress, flushes)."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from conftest import state_key  # noqa: E402
from optimalcontrolmps_amd.native import MPS, Engine  # noqa: E402

z = dict(np.load("tests/golden/states.npz", allow_pickle=False))
L, p, N, J = 5, 5, 5, 1.0


def st(U):
    k = state_key(L, p, N, J, U)
    return MPS(L, p, N, z[k + "/dims"], z[k + "/data"])


Nt = int(sys.argv[2]) if len(sys.argv) > 2 else 201
u = np.random.default_rng(77).uniform(2, 10, Nt)
kind = sys.argv[1]
print("create", kind, flush=True)
eng = Engine(L, p, N, J, 0.01, 1e-8, 80, engine=kind)
print("set_states", flush=True)
eng.set_states(st(50.0), st(2.5))
print("hessian", flush=True)
H, d, F = eng.hessian(u)
print("fidelities", flush=True)
f = eng.fidelities()
print("state", flush=True)
s = eng.state(0, Nt - 1)
print("done", np.abs(H).max(), flush=True)
