"""The CPU oracle (oracle/, a restatement of BH_tDMRG + OptimalControl) pinned
against (1) the committed fixtures it produced (regression), (2) an
independent exact state-vector implementation of the same Trotter scheme
(numpy, full Hilbert space), and (3) its building blocks
(Hermitian eigensolver, ITensor truncation rule).  The reference's own golden
numbers are checked through the facade in test_facade_cpu.py.
"""
import os

import numpy as np
import pytest

import oracle_ffi as O
from conftest import state_key
from optimalcontrolmps_amd import ed

CASES = [  # fixture name, (L, p, N, J), U_init, U_target, dt, cutoff, maxm
    ("grad_L5p6", (5, 6, 5, 1.0), 2.0, 12.0, 0.01, 1e-8, 0),
    ("hess_L5p6", (5, 6, 5, 1.0), 2.0, 12.0, 0.01, 1e-8, 0),
    ("seq_L3p4", (3, 4, 3, 2.0), 2.0, 12.0, 0.01, 1e-7, 0),
    ("even_L4p3", (4, 3, 4, 1.0), 2.0, 10.0, 0.01, 1e-8, 0),
]


def orc_state(states, L, p, N, J, U):
    k = state_key(L, p, N, J, U)
    return O.MPS(L, p, N, states[k + "/dims"], states[k + "/data"])


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_oracle_reproduces_fixtures(states, oracle_golden, case):
    name, (L, p, N, J), Ui, Uf, dt, cut, maxm = case
    u = oracle_golden[name + "/u"]
    oc = O.OC(O.Stepper(L, p, N, J, dt, cut, maxm or 5000), orc_state(states, L, p, N, J, Uf),
              orc_state(states, L, p, N, J, Ui), len(u), 0.0)
    g = oc.gradient(u)
    assert np.abs(g - oracle_golden[name + "/grad"]).max() <= 1e-12
    H = oc.hessian(u, 4)
    Hg = oracle_golden[name + "/hess"]
    assert np.abs(H - Hg).max() <= 1e-12 * np.abs(Hg).max()
    assert list(oc.state(0, len(u) - 1).bond_dims()) == list(oracle_golden[name + "/psiT_dims"])


def test_oracle_config1_gradient_fixture(states, oracle_golden):
    u = oracle_golden["config1/u"]
    oc = O.OC(O.Stepper(5, 5, 5, 1.0, 0.01, 1e-8, 80), orc_state(states, 5, 5, 5, 1.0, 50.0),
              orc_state(states, 5, 5, 5, 1.0, 2.5), len(u), 0.0)
    assert np.abs(oc.gradient(u) - oracle_golden["config1/grad"]).max() <= 1e-12
    assert list(oc.state(0, len(u) - 1).bond_dims()) == list(oracle_golden["config1/psiT_dims"])


def exact_gradient(L, p, Q, J, dt, u, ini, tgt):
    """GRAPE gradient from full state vectors: calcPsi/calcXi/calcDivT
    (src/OptimalControl.cpp:375-419) and g_i = dt Re(divT_i F i) (:240-246)."""
    N = len(u)
    psi = [ini]
    for i in range(N - 1):
        psi.append(ed.exact_step(psi[-1], L, p, J, dt, u[i], u[i + 1], True))
    xi = [None] * N
    xi[N - 1] = tgt
    for i in range(N - 1, 0, -1):
        xi[i - 1] = ed.exact_step(xi[i], L, p, J, dt, u[i], u[i - 1], False)
    dH = ed.dH_full(L, p)
    divT = np.array([np.vdot(xi[i], dH * psi[i]) for i in range(N)])
    F = np.vdot(psi[-1], tgt)
    return dt * (divT * F * 1j).real, divT, F


@pytest.mark.parametrize("L,p,Q,J,Ui,Uf", [(3, 4, 3, 2.0, 2.0, 12.0), (4, 3, 4, 1.0, 2.0, 10.0),
                                            (5, 6, 5, 1.0, 2.0, 12.0)])
def test_oracle_gradient_matches_exact_state_vector(states, L, p, Q, J, Ui, Uf):
    dt = 0.01
    u = np.random.default_rng(L * 10 + p).uniform(2, 10, 12)
    ini_m, tgt_m = orc_state(states, L, p, Q, J, Ui), orc_state(states, L, p, Q, J, Uf)
    full = lambda m: ed.full_from_mps(m.dims, m.data, L, p, Q)
    g_ex, divT_ex, F_ex = exact_gradient(L, p, Q, J, dt, u, full(ini_m), full(tgt_m))
    # cutoff 1e-14 (the gauge-move cutoff too) discards Schmidt weight < 1e-14
    # per decomposition, i.e. amplitude errors up to ~1e-7 per step
    oc = O.OC(O.Stepper(L, p, Q, J, dt, 1e-14), tgt_m, ini_m, len(u), 0.0)
    g = oc.gradient(u)
    divT, F = oc.divT_F()
    assert abs(F - F_ex) < 1e-8
    assert np.abs(divT - divT_ex).max() < 1e-7
    assert np.abs(g - g_ex).max() < 1e-9


def test_oracle_step_matches_exact_trotter_step(states):
    L, p, Q, J = 5, 6, 5, 1.0
    m = orc_state(states, L, p, Q, J, 2.0)
    st = O.Stepper(L, p, Q, J, 0.01, 1e-14)
    v = ed.full_from_mps(m.dims, m.data, L, p, Q)
    for fwd in (True, False):
        out = st.step(m, 3.0, 7.0, fwd)
        w = ed.full_from_mps(out.dims, out.data, L, p, Q)
        ref = ed.exact_step(v, L, p, J, 0.01, 3.0, 7.0, fwd)
        assert abs(abs(np.vdot(ref, w)) - 1.0) < 1e-12
        assert np.abs(w - ref * np.vdot(ref, w)).max() < 1e-9


def test_oracle_heev_matches_numpy():
    rng = np.random.default_rng(0)
    for n in (1, 2, 5, 17):
        A = rng.normal(size=(n, n)) + 1j * rng.normal(size=(n, n))
        A = A @ A.conj().T
        w, V = O.heev(A)
        assert np.allclose(np.sort(w), np.linalg.eigvalsh(A), atol=1e-12 * np.abs(w).max())
        assert np.allclose(A @ V, V * w, atol=1e-11 * np.abs(w).max())
        assert np.allclose(V.conj().T @ V, np.eye(n), atol=1e-12)


def test_truncation_rule():
    # discard smallest weights while the discarded sum stays < cutoff * total; Maxm cap; Minm = 1
    P = np.array([0.5, 0.3, 0.15, 0.04, 0.009, 0.001])
    assert O.truncate(P, 0.0, 100) == 6
    assert O.truncate(P, 0.002, 100) == 5
    assert O.truncate(P, 0.0101, 100) == 4
    assert O.truncate(P, 0.06, 100) == 3
    assert O.truncate(P, 0.06, 2) == 2
    assert O.truncate(P, 0.99, 100) == 1
    assert O.truncate(np.array([1.0]), 0.5, 100) == 1


def test_hessian_vs_gradient_derivative_truncation(states):
    """calcHessianRow (src/OptimalControl.cpp:251-279) differentiates the
    propagation with the truncation held fixed.  When Maxm does not bind, its
    entries equal central differences of the analytic gradient up to a small
    O(dt) term (config-1 chain, N_t = 4: 9e-5 at dt = 0.01, 6e-5 at 0.005; at
    config 4's chain with Maxm 4096: 2e-4 / 1e-4); when Maxm binds, the
    truncation of dH psi_i and of the trajectories, which the analytic
    derivative ignores, dominates (here 43 % at Maxm 3; config 4's chain at
    Maxm 32: 3.7 %; config 5 at chi = 512: 1.4 %, tests/test_config5_chi512.py)."""
    import oracle_ffi as O
    from conftest import state_key
    L, p, N, J, CUT = 5, 5, 5, 1.0, 1e-8
    k0, k1 = state_key(L, p, N, J, 2.5), state_key(L, p, N, J, 50.0)
    ini = O.MPS(L, p, N, states[k0 + "/dims"], states[k0 + "/data"])
    tgt = O.MPS(L, p, N, states[k1 + "/dims"], states[k1 + "/data"])
    u = np.random.default_rng(51).uniform(2.0, 10.0, 4)

    def gap(maxm, dt):
        oc = O.OC(O.Stepper(L, p, N, J, dt, CUT, maxm), tgt, ini, 4, 0.0)
        H = oc.hessian(u, 1)
        g = 0.0
        for j in (1, 2):
            up, um = u.copy(), u.copy()
            up[j] += 1e-3
            um[j] -= 1e-3
            col = (oc.gradient(up) - oc.gradient(um)) / 2e-3
            g = max(g, float(np.max(np.abs(H[1:3, j] - col[1:3]) / np.abs(col[1:3]))))
        return g
    g1, g2 = gap(80, 0.01), gap(80, 0.005)
    assert g1 < 3e-4 and g2 < g1
    assert gap(3, 0.01) > 1e-1


@pytest.mark.parametrize("n", [1, 2, 3, 7, 64, 160])
def test_heev_ql_vs_numpy_and_jacobi(n):
    """the oracle's Householder + QL eigensolver (ORC_HEEV=ql: zheev's
    algorithm, used to generate the large chi fixtures) against numpy and the
    default cyclic Jacobi on PSD Gram blocks with a spectrum spread over
    twelve orders (the density matrices denmatDecomp diagonalises)"""
    rng = np.random.default_rng(n)
    X = rng.normal(size=(n, n + 2)) + 1j * rng.normal(size=(n, n + 2))
    X *= np.logspace(0, -6, n)[:, None]
    A = X @ X.conj().T
    w, V = O.heev_ql(A)
    wj, Vj = O.heev(A)
    wn = np.sort(np.linalg.eigvalsh(A))[::-1]
    scale = np.abs(wn).max()
    assert np.all(np.diff(w) <= 0)
    assert np.abs(w - wn).max() <= 1e-14 * scale * max(1, n / 16)
    assert np.abs(w - wj).max() <= 1e-14 * scale * max(1, n / 16)
    assert np.abs(V.conj().T @ V - np.eye(n)).max() <= 1e-13
    assert np.abs(A @ V - V * w).max() <= 1e-14 * scale * max(1, n / 16)


def test_sector_parallel_oracle_bitwise(states, oracle_golden):
    """The sector-parallel oracle (ORC_SECTOR_THREADS / the nested getHessian the
    large configs' CPU baselines use) computes every U(1) block with the same
    loops on one thread, so its Hessian, gradient and states equal the serial
    oracle's bit for bit."""
    name, (L, p, N, J), Ui, Uf, dt, cut, maxm = CASES[1]
    u = oracle_golden[name + "/u"]

    def make():
        return O.OC(O.Stepper(L, p, N, J, dt, cut, maxm or 5000), orc_state(states, L, p, N, J, Uf),
                    orc_state(states, L, p, N, J, Ui), len(u), 0.0)
    ref = make()
    H0 = ref.hessian(u, 1)
    par = make()
    par.set_nested(True)
    H1 = par.hessian(u, 6)
    assert np.array_equal(H0, H1)
    st = O.Stepper(L, p, N, J, dt, cut, maxm or 5000)
    psi = orc_state(states, L, p, N, J, Ui)
    a = st.steps(psi, u[:6])
    O.set_sector_threads(4)
    try:
        b = st.steps(psi, u[:6])
    finally:
        O.set_sector_threads(1)
    assert np.array_equal(a.dims, b.dims) and np.array_equal(a.data, b.data)
