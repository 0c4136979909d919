"""Generate the committed fixtures of tests/golden/ (TEST INFRASTRUCTURE).

states.npz : exact ground states (ED, optimalcontrolmps_amd.ed) of the
             Bose-Hubbard chains the reference's tests and BASELINE config 1
             use, in the compact U(1)-block MPS format of include/ocmps.h.
             Key "<tag>/dims", "<tag>/data".  Tags: L{L}_p{p}_N{N}_J{J}_U{U}.
oracle.npz : outputs of the CPU oracle (oracle/, a from-scratch restatement
             of BH_tDMRG + OptimalControl) on seeded controls, so GPU parity
             tests run against fixed vectors even without rebuilding the
             oracle on the box.

The reference cannot be compiled or imported here (ITensor v2, IPOPT and gtest
are absent), so no fixture is produced by the reference itself:
the reference's own golden numbers (tests/CostTests.cpp, tests/
ControlBasisTests.cpp) are restated as constants in tests/reference_goldens.py
and the oracle is pinned against them there.

Run:  python tests/golden/make_fixtures.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from optimalcontrolmps_amd import ed  # noqa: E402
import oracle_ffi as O  # noqa: E402

STATES = [
    # (L, p, N, J, U)
    (5, 6, 5, 1.0, 2.0), (5, 6, 5, 1.0, 12.0), (5, 6, 5, 1.0, 50.0), (5, 6, 5, 1.0, 2.5),   # reference tests (locDim 5)
    (5, 5, 5, 1.0, 2.5), (5, 5, 5, 1.0, 50.0),                                             # BASELINE config 1 (d = 4)
    (3, 4, 3, 2.0, 2.0), (3, 4, 3, 2.0, 12.0),                                             # SequencingTest (L3, locDim 3)
    (4, 3, 4, 1.0, 2.0), (4, 3, 4, 1.0, 10.0),                                             # even-L coverage
]


def tag(L, p, N, J, U):
    return f"L{L}_p{p}_N{N}_J{J:g}_U{U:g}"


def make_states():
    out = {}
    for (L, p, N, J, U) in STATES:
        full, e0 = ed.ground_state_full(L, p, N, J, U)
        dims, data = ed.mps_from_full(full, L, p, N)
        t = tag(L, p, N, J, U)
        out[t + "/dims"] = dims.reshape(-1).astype(np.int32)
        out[t + "/data"] = data.astype(np.complex128)
        out[t + "/energy"] = np.array(e0)
    np.savez_compressed(os.path.join(HERE, "states.npz"), **out)
    return out


def load_state(states, L, p, N, J, U):
    t = tag(L, p, N, J, U)
    return O.MPS(L, p, N, states[t + "/dims"], states[t + "/data"])


CASES = [
    # name, (L, p, N, J), U_init, U_target, dt, cutoff, maxm, Nt, control (lo, hi, seed)
    ("grad_L5p6", (5, 6, 5, 1.0), 2.0, 12.0, 0.01, 1e-8, 0, 16, (2.0, 10.0, 1)),
    ("hess_L5p6", (5, 6, 5, 1.0), 2.0, 12.0, 0.01, 1e-8, 0, 11, (2.0, 10.0, 2)),
    ("seq_L3p4", (3, 4, 3, 2.0), 2.0, 12.0, 0.01, 1e-7, 0, 51, (5.0, 15.0, 3)),
    ("even_L4p3", (4, 3, 4, 1.0), 2.0, 10.0, 0.01, 1e-8, 0, 21, (2.0, 10.0, 4)),
    ("config1", (5, 5, 5, 1.0), 2.5, 50.0, 0.01, 1e-8, 80, 201, (2.0, 10.0, 20261015)),
]


def make_oracle(states, threads=8):
    out = {}
    for name, (L, p, N, J), Ui, Uf, dt, cut, maxm, Nt, (lo, hi, seed) in CASES:
        st = O.Stepper(L, p, N, J, dt, cut, maxm if maxm > 0 else 5000)
        init = load_state(states, L, p, N, J, Ui)
        tgt = load_state(states, L, p, N, J, Uf)
        u = np.random.default_rng(seed).uniform(lo, hi, Nt)
        oc = O.OC(st, tgt, init, Nt, 0.0)
        g = oc.gradient(u)
        divT, F = oc.divT_F()
        fid = oc.fidelities(u)
        H = oc.hessian(u, threads)
        out[name + "/u"] = u
        out[name + "/grad"] = g
        out[name + "/divT"] = divT
        out[name + "/F"] = np.array([F])
        out[name + "/fid"] = fid
        out[name + "/hess"] = H
        out[name + "/psiT_dims"] = oc.state(0, Nt - 1).bond_dims()
        print(name, "done", flush=True)
    np.savez_compressed(os.path.join(HERE, "oracle.npz"), **out)


if __name__ == "__main__":
    s = make_states()
    make_oracle(s)
