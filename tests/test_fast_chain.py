"""The one-wave padded chain (csrc/fast_chain.hpp, fast_plan.hpp) that runs
every step of config 1 (L=5, p=5, Npart=5), against the general LDS chain
(OCG_NO_FAST=1) and the CPU oracle: the same bond dimensions after every
truncation, the same states up to rounding (gauge-invariant overlaps), the
same getHessian at the north_star tolerances.  The reference semantics are
BH_tDMRG::step (src/BH_tDMRG.cpp:111-230) and calcHessianRow
(src/OptimalControl.cpp:251-279)."""
import numpy as np
import pytest

import oracle_ffi as O
from optimalcontrolmps_amd import ed

pytestmark = pytest.mark.gpu

L, p, Q, J, DT, CUT = 5, 5, 5, 1.0, 0.01, 1e-8


def _engine(monkeypatch, fast, maxm=80, cutoff=CUT, Lx=L, px=p, Qx=Q):
    from optimalcontrolmps_amd.native import Engine
    if fast:
        monkeypatch.delenv("OCG_NO_FAST", raising=False)
    else:
        monkeypatch.setenv("OCG_NO_FAST", "1")
    e = Engine(Lx, px, Qx, J, DT, cutoff, maxm)
    assert e.info.fast_chain == (1 if fast else 0)
    return e


def _gs(U, Lx=L, px=p, Qx=Q):
    from optimalcontrolmps_amd.native import MPS
    return MPS(Lx, px, Qx, *ed.mps_from_full(ed.ground_state_full(Lx, px, Qx, J, U)[0], Lx, px, Qx))


@pytest.mark.parametrize("maxm,cutoff", [(80, 1e-8), (3, 1e-8), (6, 1e-8), (80, 1e-4)])
def test_fast_steps_match_general_and_oracle(monkeypatch, maxm, cutoff):
    psi = _gs(2.5)
    u = np.random.default_rng(11).uniform(2.0, 10.0, 21)
    fe, ge = _engine(monkeypatch, True, maxm, cutoff), _engine(monkeypatch, False, maxm, cutoff)
    st = O.Stepper(L, p, Q, J, DT, cutoff, maxm)
    for fwd in (True, False):
        a = fe.steps(psi, u, fwd)
        b = ge.steps(psi, u, fwd)
        ref = st.steps(O.MPS(L, p, Q, psi.dims, psi.data), u, fwd)
        assert list(a.bond_dims()) == list(b.bond_dims()) == list(ref.bond_dims())
        assert abs(fe.overlap(a, b) - 1.0) <= 1e-12
        assert abs(abs(st.overlap(ref, O.MPS(L, p, Q, a.dims, a.data))) - 1.0) <= 1e-12
        assert abs(fe.overlap(a, a, True) - ge.overlap(b, b, True)) <= 1e-12
    fe.close()
    ge.close()


def test_fast_hessian_matches_general_full_horizon(monkeypatch, states, oracle_golden):
    """config 1's full getHessian (N_t = 201, 199 rows; the golden fixture's
    controls and ED states) through the fused pipeline on both chains: the
    one-wave chain against the oracle's Hessian, gradient, divT and F
    (tests/golden/oracle.npz `config1`) at the north_star tolerances
    (gradient 1e-6 absolute, Hessian 1e-6 max|H|), and against the general
    chain to rounding (gradient 1e-12, Hessian 1e-10 max|H|: two summation
    orders of the same decompositions)"""
    from conftest import state_key
    from optimalcontrolmps_amd.native import MPS
    k = lambda U: state_key(L, p, Q, J, U)
    tgt = MPS(L, p, Q, states[k(50.0) + "/dims"], states[k(50.0) + "/data"])
    ini = MPS(L, p, Q, states[k(2.5) + "/dims"], states[k(2.5) + "/data"])
    u = oracle_golden["config1/u"]
    assert len(u) == 201
    out = {}
    for fast in (True, False):
        e = _engine(monkeypatch, fast)
        e.set_states(tgt, ini)
        out[fast] = e.hessian(u)
        e.close()
    (Hf, df, Ff), (Hg, dg, Fg) = out[True], out[False]
    gf, gg = DT * (df * Ff * 1j).real, DT * (dg * Fg * 1j).real
    Ho = oracle_golden["config1/hess"]
    assert np.abs(gf - oracle_golden["config1/grad"]).max() < 1e-6
    assert np.abs(df - oracle_golden["config1/divT"]).max() < 1e-9
    assert abs(Ff - oracle_golden["config1/F"][0]) < 1e-9
    assert np.abs(Hf - Ho).max() <= 1e-6 * np.abs(Ho).max()
    assert np.abs(gf - gg).max() <= 1e-12
    assert np.abs(Hf - Hg).max() <= 1e-10 * np.abs(Hg).max()


def test_fast_unfused_equals_fused(monkeypatch):
    """the unfused getHessian (propagate, xi_dH, k_hessian_rows) and the fused
    pipeline both step on the one-wave chain: bitwise the same Hessian"""
    tgt, ini = _gs(50.0), _gs(2.5)
    u = np.random.default_rng(5).uniform(2.0, 10.0, 31)
    e = _engine(monkeypatch, True)
    e.set_states(tgt, ini)
    Hf, df, Ff = e.hessian(u)
    e.propagate(u, 3)
    dv = e.div_t()
    F = e.overlap_factor()
    e.xi_dH()
    Hu = e.hessian_rows(u, list(range(1, 30)), F, dv)
    assert np.array_equal(Hf, Hu)
    e.close()


@pytest.mark.parametrize("cfg", [(5, 6, 5, 2.0), (4, 3, 4, 2.0), (3, 4, 3, 2.0)])
def test_fast_other_small_chains(monkeypatch, cfg):
    """other chains the plan fits (p = 6; even L: the lonely U_to; odd L = 3)"""
    Lx, px, Qx, U = cfg
    psi = _gs(U, Lx, px, Qx)
    u = np.random.default_rng(7).uniform(2.0, 10.0, 9)
    fe = _engine(monkeypatch, True, 5000, CUT, Lx, px, Qx)
    ge = _engine(monkeypatch, False, 5000, CUT, Lx, px, Qx)
    a, b = fe.steps(psi, u, True), ge.steps(psi, u, True)
    assert list(a.bond_dims()) == list(b.bond_dims())
    assert abs(fe.overlap(a, b) - 1.0) <= 1e-12
    fe.close()
    ge.close()
