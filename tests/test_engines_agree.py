"""The two device engines implement the same algorithm (gate order, ITensor
truncation rule, gauge cutoff, exactApplyMPO compression): the LDS chain engine
(register Jacobi) and the HBM engine (Householder + multisection + inverse
iteration) must agree on config 1 and on a truncation-heavy case to rounding
level, and both with the oracle fixture (tests/golden/oracle.npz, config 1 at
its full N_t = 201)."""
import numpy as np
import pytest

from conftest import state_key

pytestmark = pytest.mark.gpu


def states_of(states, L, p, N, J, Ui, Uf):
    from optimalcontrolmps_amd.native import MPS

    def st(U):
        k = state_key(L, p, N, J, U)
        return MPS(L, p, N, states[k + "/dims"], states[k + "/data"])
    return st(Uf), st(Ui)


@pytest.mark.parametrize("L,p,N,J,Ui,Uf,cut,Nt", [(5, 5, 5, 1.0, 2.5, 50.0, 1e-8, 201),
                                                   (5, 6, 5, 1.0, 2.0, 12.0, 1e-4, 41)])
def test_lds_and_hbm_engines_agree(states, L, p, N, J, Ui, Uf, cut, Nt):
    from optimalcontrolmps_amd.native import Engine
    tgt, ini = states_of(states, L, p, N, J, Ui, Uf)
    u = np.random.default_rng(77).uniform(2, 10, Nt)
    res = {}
    for kind in ("lds", "hbm"):
        eng = Engine(L, p, N, J, 0.01, cut, 80, engine=kind)
        eng.set_states(tgt, ini)
        H, divT, F = eng.hessian(u)
        res[kind] = (H, divT, F, eng.fidelities(), list(eng.state(0, Nt - 1).bond_dims()))
    (H1, d1, F1, f1, b1), (H2, d2, F2, f2, b2) = res["lds"], res["hbm"]
    assert b1 == b2
    assert abs(F1 - F2) < 1e-11
    assert np.abs(d1 - d2).max() < 1e-11
    assert np.abs(f1 - f2).max() < 1e-11
    assert np.abs(H1 - H2).max() <= 1e-9 * np.abs(H1).max()
