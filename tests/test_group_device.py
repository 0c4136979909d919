"""GROUP path on the device: ControlBasis::convertHessian
(src/ControlBasis.cpp:91-116) as ocg_convert_hessian, and the Hessian at the
control of the last gradient reusing the device trajectories (BH_nlp::eval_h
after eval_grad_f, src/BH_nlp.cpp:189)."""
import numpy as np
import pytest

from conftest import state_key

pytestmark = pytest.mark.gpu


def chopped_sine_V(N, M, dt, T):
    """V[n][i] = S_i f_{i n} of buildChoppedSineBasis (include/ControlBasisFactory.hpp:25-53)"""
    PI = 3.14159265
    x = np.linspace(0.0, 100.0, N)
    S = np.where(np.arange(N) < N // 2, 1.0 / (1.0 + np.exp(-8.0 * (x - 1.1))),
                 1.0 / (1.0 + np.exp(8.0 * (x - 98.9))))
    S[0] = S[-1] = 0.0
    f = np.sin(np.outer(np.arange(N) * dt, (np.arange(M) + 1) * PI / T))
    return (f * S[:, None]).T.copy()


def host_convert(Hu, V):
    """the reference's order: sequential inner products, a*b then +"""
    M, N = V.shape
    HV = np.zeros((M, N))
    for j in range(M):
        vj = V[j].tolist()
        for k in range(N):
            acc = 0.0
            for a, b in zip(Hu[k].tolist(), vj):
                acc = acc + a * b
            HV[j, k] = acc
    Hc = np.zeros((M, M))
    for i in range(M):
        vi = V[i].tolist()
        for j in range(i, M):
            acc = 0.0
            for a, b in zip(vi, HV[j].tolist()):
                acc = acc + a * b
            Hc[i, j] = Hc[j, i] = acc
    return Hc


def engine():
    from optimalcontrolmps_amd.native import Engine
    return Engine(5, 5, 5, 1.0, 0.01, 1e-8, 80)


def test_convert_hessian_bitwise_host_order():
    rng = np.random.default_rng(91)
    N, M = 201, 10
    Hu = rng.normal(size=(N, N))
    Hu = Hu + Hu.T
    V = chopped_sine_V(N, M, 0.01, 2.0)
    Hc = engine().convert_hessian(Hu, V)
    assert np.array_equal(Hc, host_convert(Hu, V))


def test_convert_hessian_config4_shape():
    """config 4's GROUP shape: N_t = 801, M = 40"""
    rng = np.random.default_rng(92)
    N, M = 801, 40
    Hu = rng.normal(size=(N, N))
    Hu = Hu + Hu.T
    V = chopped_sine_V(N, M, 0.005, 4.0)
    Hc = engine().convert_hessian(Hu, V)
    ref = V @ Hu @ V.T
    assert np.abs(Hc - ref).max() <= 1e-12 * np.abs(ref).max()
    assert np.array_equal(Hc, Hc.T)


def test_hessian_reuses_gradient_trajectories(states):
    """HBM engine: getHessian(u) right after the gradient at u skips the
    re-propagation and gives the same Hessian bit for bit"""
    from optimalcontrolmps_amd.native import MPS, Engine
    L, p, N, J = 5, 5, 5, 1.0

    def st(U):
        k = state_key(L, p, N, J, U)
        return MPS(L, p, N, states[k + "/dims"], states[k + "/data"])
    u = np.random.default_rng(93).uniform(2, 10, 21)
    eng = Engine(L, p, N, J, 0.01, 1e-8, 80, engine="hbm")
    eng.set_states(st(50.0), st(2.5))
    H0, d0, F0 = eng.hessian(u)                 # fresh (pipelined: hbm_hessian_pipe, stats kind 5)
    eng.propagate(u, 3)                          # the gradient's propagation
    s0, p0 = eng.stats(0)["launches"], eng.stats(5)["launches"]
    H1, d1, F1 = eng.hessian(u)                  # reuses psi_t / xi_t (no propagation, no pipeline)
    assert eng.stats(0)["launches"] == s0 and eng.stats(5)["launches"] == p0
    assert np.array_equal(H0, H1) and np.array_equal(d0, d1) and F0 == F1
    u2 = u.copy()
    u2[5] += 1e-3
    eng.hessian(u2)                              # a new control propagates again
    assert eng.stats(0)["launches"] + eng.stats(5)["launches"] > s0 + p0
