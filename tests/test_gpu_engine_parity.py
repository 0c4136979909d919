"""GPU parity of the HIP chain engine (through the C-ABI) against the CPU
oracle and the committed golden fixtures.

Tolerances: north_star asks for gradient entries within 1e-6 of the
reference CPU path; Hessians are compared at 1e-6 * max|H|.
Trajectory-level quantities (overlaps, fidelities, divT) are compared at
1e-9 absolute, which the FP64 engine meets with margin (observed ~1e-13).
States are compared only through gauge-invariant quantities (|<a|b>|, norms,
bond dimensions), because eigen-decompositions fix gauges differently.
"""
import numpy as np
import pytest

import oracle_ffi as O
from conftest import state_key

pytestmark = pytest.mark.gpu


def engine(L, p, N, J, dt, cutoff, maxm=0):
    from optimalcontrolmps_amd.native import Engine
    return Engine(L, p, N, J, dt, cutoff, maxm)


def st_of(states, L, p, N, J, U):
    k = state_key(L, p, N, J, U)
    from optimalcontrolmps_amd.native import MPS
    return MPS(L, p, N, states[k + "/dims"], states[k + "/data"])


def as_orc(m):
    return O.MPS(m.L, m.p, m.Q, m.dims, m.data)


CHAINS = [(5, 6, 5, 1.0, 2.0, 12.0), (5, 5, 5, 1.0, 2.5, 50.0), (3, 4, 3, 2.0, 2.0, 12.0), (4, 3, 4, 1.0, 2.0, 10.0)]


@pytest.mark.parametrize("L,p,N,J,Ui,Uf", CHAINS)
@pytest.mark.parametrize("forward", [True, False])
def test_step_matches_oracle(states, L, p, N, J, Ui, Uf, forward):
    eng = engine(L, p, N, J, 0.01, 1e-8)
    orc = O.Stepper(L, p, N, J, 0.01, 1e-8)
    s0 = st_of(states, L, p, N, J, Ui if forward else Uf)
    u = np.random.default_rng(7).uniform(2, 10, 9)
    g = eng.steps(s0, u, forward)
    o = orc.steps(as_orc(s0), u, forward)
    assert list(g.bond_dims()) == list(o.bond_dims())
    ov = orc.overlap(o, as_orc(g))
    assert abs(abs(ov) - 1.0) < 1e-12
    assert abs(orc.overlap(as_orc(g), as_orc(g)) - 1.0) < 1e-12


@pytest.mark.parametrize("L,p,N,J,Ui,Uf", CHAINS)
def test_overlaps_match_oracle(states, L, p, N, J, Ui, Uf):
    eng = engine(L, p, N, J, 0.01, 1e-8)
    orc = O.Stepper(L, p, N, J, 0.01, 1e-8)
    a, b = st_of(states, L, p, N, J, Ui), st_of(states, L, p, N, J, Uf)
    assert abs(eng.overlap(a, b) - orc.overlap(as_orc(a), as_orc(b))) < 1e-12
    assert abs(eng.overlap(a, b, True) - orc.overlap_dH(as_orc(a), as_orc(b))) < 1e-12


@pytest.mark.parametrize("L,p,N,J,Ui,Uf", CHAINS)
def test_apply_dH_matches_oracle(states, L, p, N, J, Ui, Uf):
    eng = engine(L, p, N, J, 0.01, 1e-8)
    orc = O.Stepper(L, p, N, J, 0.01, 1e-8)
    s = st_of(states, L, p, N, J, Ui)
    g, nrm = eng.apply_dH(s)
    o = orc.apply_dH(as_orc(s))
    assert list(g.bond_dims()) == list(o.bond_dims())
    no = np.sqrt(orc.overlap(o, o).real)
    assert abs(nrm - no) < 1e-12 * max(1.0, no)
    assert abs(orc.overlap(o, as_orc(g)).real - no * no) < 1e-11 * no * no


GOLDEN = [
    ("grad_L5p6", (5, 6, 5, 1.0), 2.0, 12.0, 0.01, 1e-8, 0),
    ("hess_L5p6", (5, 6, 5, 1.0), 2.0, 12.0, 0.01, 1e-8, 0),
    ("seq_L3p4", (3, 4, 3, 2.0), 2.0, 12.0, 0.01, 1e-7, 0),
    ("even_L4p3", (4, 3, 4, 1.0), 2.0, 10.0, 0.01, 1e-8, 0),
    ("config1", (5, 5, 5, 1.0), 2.5, 50.0, 0.01, 1e-8, 80),
]


def run_engine_hessian(eng, u, tgt, ini):
    """GPU calcHessian (src/OptimalControl.cpp:341-372) without regularisation."""
    eng.set_states(tgt, ini)
    eng.propagate(u, 3)
    divT = eng.div_t()
    F = eng.overlap_factor()
    fid = eng.fidelities()
    eng.xi_dH()
    N = len(u)
    H = eng.hessian_rows(u, list(range(1, N - 1)), F, divT)
    return divT, F, fid, H


def oracle_check(H, divT, F, L, p, N, J, dt, cut, maxm, tgt, ini, u, threads=8):
    """the CPU oracle's getHessian of the same inputs, so that a path-equality
    test also pins parity: H to the north_star 1e-6 of its scale, divT / F to
    1e-8 / 1e-9 (test_hessian_multi_vs_oracle's bounds)"""
    oc = O.OC(O.Stepper(L, p, N, J, dt, cut, maxm if maxm > 0 else 5000), as_orc(tgt), as_orc(ini), len(u), 0.0)
    Ho = oc.hessian(u, threads)
    do, Fo = oc.divT_F()
    assert abs(F - Fo) <= 1e-9
    assert np.abs(divT - do).max() <= 1e-8 * np.abs(do).max()
    assert np.abs(H - Ho).max() <= 1e-6 * np.abs(Ho).max()


@pytest.mark.parametrize("case", GOLDEN, ids=[c[0] for c in GOLDEN])
def test_trajectories_gradient_hessian_vs_golden(states, oracle_golden, case):
    name, (L, p, N, J), Ui, Uf, dt, cut, maxm = case
    u = oracle_golden[name + "/u"]
    eng = engine(L, p, N, J, dt, cut, maxm)
    if name == "config1":  # config 1 runs on the one-wave padded chain (csrc/fast_chain.hpp)
        assert eng.info.fast_chain == 1
    divT, F, fid, H = run_engine_hessian(eng, u, st_of(states, L, p, N, J, Uf), st_of(states, L, p, N, J, Ui))
    assert np.abs(divT - oracle_golden[name + "/divT"]).max() < 1e-9
    assert abs(F - oracle_golden[name + "/F"][0]) < 1e-9
    assert np.abs(fid - oracle_golden[name + "/fid"]).max() < 1e-9
    # gradient g_i = dt Re(divT_i F i)  (src/OptimalControl.cpp:240-246), gamma = 0
    g = dt * (divT * F * 1j).real
    assert np.abs(g - oracle_golden[name + "/grad"]).max() < 1e-6
    Ho = oracle_golden[name + "/hess"]
    assert np.abs(H - Ho).max() <= 1e-6 * np.abs(Ho).max()
    assert list(eng.state(0, len(u) - 1).bond_dims()) == list(oracle_golden[name + "/psiT_dims"])


def test_hessian_live_oracle_random_controls(states):
    """fresh controls (not in the fixtures) against the live oracle"""
    L, p, N, J = 5, 6, 5, 1.0
    u = np.random.default_rng(99).uniform(2, 10, 13)
    eng = engine(L, p, N, J, 0.01, 1e-8)
    tgt, ini = st_of(states, L, p, N, J, 12.0), st_of(states, L, p, N, J, 2.0)
    divT, F, fid, H = run_engine_hessian(eng, u, tgt, ini)
    oc = O.OC(O.Stepper(L, p, N, J, 0.01, 1e-8), as_orc(tgt), as_orc(ini), len(u), 0.0)
    Ho = oc.hessian(u, 4)
    assert np.abs(H - Ho).max() <= 1e-6 * np.abs(Ho).max()
    go = oc.gradient(u)
    assert np.abs(0.01 * (divT * F * 1j).real - go).max() < 1e-6


def test_deterministic_repeat(states):
    """same inputs -> bitwise identical outputs (SequencingTest's premise)"""
    L, p, N, J = 5, 5, 5, 1.0
    u = np.random.default_rng(5).uniform(2, 10, 21)
    eng = engine(L, p, N, J, 0.01, 1e-8, 80)
    tgt, ini = st_of(states, L, p, N, J, 50.0), st_of(states, L, p, N, J, 2.5)
    a = run_engine_hessian(eng, u, tgt, ini)
    b = run_engine_hessian(eng, u, tgt, ini)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[3], b[3])


def test_rows_subset_sum_equals_full(states):
    """row sharding (multi-GPU path): disjoint row subsets sum to the full Hessian"""
    L, p, N, J = 5, 6, 5, 1.0
    u = np.random.default_rng(11).uniform(2, 10, 12)
    eng = engine(L, p, N, J, 0.01, 1e-8)
    tgt, ini = st_of(states, L, p, N, J, 12.0), st_of(states, L, p, N, J, 2.0)
    divT, F, fid, H = run_engine_hessian(eng, u, tgt, ini)
    Ns = len(u)
    rows = list(range(1, Ns - 1))
    parts = [eng.hessian_rows(u, rows[r::3], F, divT) for r in range(3)]
    assert np.array_equal(sum(parts), H)


def test_cost_golden_via_gpu(states):
    """tests/CostTests.cpp:68-99 through the GPU: cost within 1e-6 of the golden
    value; fidelities within 1e-5 (golden values come from ITensor-DMRG ground
    states, ours from exact diagonalisation: 5.8e-6 offset already at t = 0)."""
    from reference_goldens import COST_LINEAR, FID_LINEAR, COST_ONES, FID_ONES
    L, p, N, J = 5, 6, 5, 1.0
    eng = engine(L, p, N, J, 0.01, 1e-8)
    tgt, ini = st_of(states, L, p, N, J, 50.0), st_of(states, L, p, N, J, 2.0)
    for u, cost, fids in [(np.array([2.0 + 4.8 * i for i in range(11)]), COST_LINEAR, FID_LINEAR),
                          (np.ones(11), COST_ONES, FID_ONES)]:
        eng.set_states(tgt, ini)
        eng.propagate(u, 1)
        F = eng.overlap_factor()
        # 1e-6 in the reference (DMRG states); ED states shift the t=0 overlap by <= 5.8e-6
        assert abs(0.5 * (1 - abs(F) ** 2) - cost) < 5e-6
        f = eng.fidelities()
        assert np.abs(f[:-1] - np.array(fids[:-1])).max() < 1e-5


@pytest.mark.parametrize("case", GOLDEN, ids=[c[0] for c in GOLDEN])
def test_fused_hessian_vs_golden(states, oracle_golden, case):
    """ocg_hessian (pipelined trajectories + rows, batched overlaps) against the fixtures"""
    name, (L, p, N, J), Ui, Uf, dt, cut, maxm = case
    u = oracle_golden[name + "/u"]
    eng = engine(L, p, N, J, dt, cut, maxm)
    if name == "config1":  # the headline path: the one-wave padded chain, not the general one
        assert eng.info.fast_chain == 1
    eng.set_states(st_of(states, L, p, N, J, Uf), st_of(states, L, p, N, J, Ui))
    H, divT, F = eng.hessian(u)
    assert np.abs(divT - oracle_golden[name + "/divT"]).max() < 1e-9
    assert abs(F - oracle_golden[name + "/F"][0]) < 1e-9
    g = dt * (divT * F * 1j).real
    assert np.abs(g - oracle_golden[name + "/grad"]).max() < 1e-6
    Ho = oracle_golden[name + "/hess"]
    assert np.abs(H - Ho).max() <= 1e-6 * np.abs(Ho).max()
    # the device trajectories are left as after propagate(3) + xi_dH
    assert list(eng.state(0, len(u) - 1).bond_dims()) == list(oracle_golden[name + "/psiT_dims"])


def test_fused_equals_unfused_bitwise(states):
    """same per-row arithmetic: the pipelined path reproduces the two-phase path exactly"""
    L, p, N, J = 5, 5, 5, 1.0
    u = np.random.default_rng(17).uniform(2, 10, 31)
    eng = engine(L, p, N, J, 0.01, 1e-8, 80)
    eng.set_states(st_of(states, L, p, N, J, 50.0), st_of(states, L, p, N, J, 2.5))
    divT, F, fid, H1 = run_engine_hessian(eng, u, st_of(states, L, p, N, J, 50.0), st_of(states, L, p, N, J, 2.5))
    H2, divT2, F2 = eng.hessian(u)
    assert np.array_equal(divT, divT2) and F == F2
    assert np.array_equal(H1, H2)
    rows = list(range(1, len(u) - 1))
    parts = [eng.hessian(u, rows[k::4])[0] for k in range(4)]
    assert np.array_equal(sum(parts), H2)
    oracle_check(H2, divT2, F2, L, p, N, J, 0.01, 1e-8, 80, st_of(states, L, p, N, J, 50.0),
                 st_of(states, L, p, N, J, 2.5), u)


def _with_plans(flag, fn):
    """the general chain (OCG_NO_FAST=1: plans belong to it; the one-wave padded
    chain that steps config-1-sized chains by default has fixed layouts) with
    decomposition plans on or off"""
    import os
    old = {k: os.environ.get(k) for k in ("OCG_NO_PLANS", "OCG_NO_FAST")}
    os.environ["OCG_NO_PLANS"] = "0" if flag else "1"
    os.environ["OCG_NO_FAST"] = "1"
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("L,p,N,J,Ui,Uf,cut", [(5, 5, 5, 1.0, 2.5, 50.0, 1e-8), (5, 6, 5, 1.0, 2.0, 12.0, 1e-4),
                                               (4, 3, 4, 1.0, 2.0, 10.0, 1e-3)])
def test_plans_bitwise_neutral(states, L, p, N, J, Ui, Uf, cut):
    """decomposition plans cache index arithmetic only: the fused getHessian with
    plans on equals the general path bitwise, also when truncation changes the
    bond dimensions from step to step (cutoff 1e-4 / 1e-3: plan misses and
    re-recordings)"""
    u = np.random.default_rng(23).uniform(2, 10, 41)
    tgt, ini = st_of(states, L, p, N, J, Uf), st_of(states, L, p, N, J, Ui)

    def run():
        eng = engine(L, p, N, J, 0.01, cut, 80)
        eng.set_states(tgt, ini)
        H, divT, F = eng.hessian(u)
        return H, divT, F, eng.info.lds_bytes

    H1, d1, F1, lds1 = _with_plans(True, run)
    H0, d0, F0, lds0 = _with_plans(False, run)
    assert lds1 > lds0  # the plan slots are really there
    assert np.array_equal(H1, H0) and np.array_equal(d1, d0) and F1 == F0
    oracle_check(H1, d1, F1, L, p, N, J, 0.01, cut, 80, tgt, ini, u)


def test_truncation_heavy_vs_oracle(states):
    """cutoff 1e-4: bond dimensions shrink and grow along the trajectories (plan
    misses); Hessian and gradient against the live oracle"""
    L, p, N, J, cut = 5, 6, 5, 1.0, 1e-4
    u = np.random.default_rng(31).uniform(2, 10, 15)
    tgt, ini = st_of(states, L, p, N, J, 12.0), st_of(states, L, p, N, J, 2.0)
    eng = engine(L, p, N, J, 0.01, cut)
    eng.set_states(tgt, ini)
    H, divT, F = eng.hessian(u)
    oc = O.OC(O.Stepper(L, p, N, J, 0.01, cut), as_orc(tgt), as_orc(ini), len(u), 0.0)
    Ho = oc.hessian(u, 4)
    assert np.abs(H - Ho).max() <= 1e-6 * np.abs(Ho).max()
    assert np.abs(0.01 * (divT * F * 1j).real - oc.gradient(u)).max() < 1e-6


@pytest.mark.parametrize("maxm", [3, 6])
def test_maxm_binding_vs_oracle(states, maxm):
    """Maxm binds (bond dimension capped below the exact 14): the general
    ranking path of the truncation, plan misses on capped bonds; Hessian and
    gradient against the live oracle, plans on/off bitwise equal"""
    L, p, N, J = 5, 6, 5, 1.0
    u = np.random.default_rng(41).uniform(2, 10, 13)
    tgt, ini = st_of(states, L, p, N, J, 12.0), st_of(states, L, p, N, J, 2.0)

    def run():
        eng = engine(L, p, N, J, 0.01, 1e-8, maxm)
        eng.set_states(tgt, ini)
        return eng.hessian(u)

    H, divT, F = _with_plans(True, run)
    H0, d0, F0 = _with_plans(False, run)
    assert np.array_equal(H, H0) and np.array_equal(divT, d0) and F == F0
    oc = O.OC(O.Stepper(L, p, N, J, 0.01, 1e-8, maxm), as_orc(tgt), as_orc(ini), len(u), 0.0)
    Ho = oc.hessian(u, 4)
    assert np.abs(H - Ho).max() <= 1e-6 * np.abs(Ho).max()
    assert np.abs(0.01 * (divT * F * 1j).real - oc.gradient(u)).max() < 1e-6
    # the default one-wave padded chain with Maxm binding: the same numbers to rounding
    Hf, df, Ff = run()
    assert np.abs(Hf - Ho).max() <= 1e-6 * np.abs(Ho).max()
    assert np.abs(Hf - H).max() <= 1e-10 * np.abs(H).max()
    assert np.abs(0.01 * (df * Ff * 1j).real - oc.gradient(u)).max() < 1e-6


def _with_env(name, value, fn):
    import os
    old = os.environ.get(name)
    os.environ[name] = value
    try:
        return fn()
    finally:
        if old is None:
            del os.environ[name]
        else:
            os.environ[name] = old


def test_fused_equals_unfused_config1_full_horizon(states):
    """config 1 at its full N_t = 201: the fused pipeline (ticket roles, rows
    overlapped with the trajectories) equals the two-phase path bit for bit"""
    L, p, N, J = 5, 5, 5, 1.0
    u = np.random.default_rng(23).uniform(2, 10, 201)
    eng = engine(L, p, N, J, 0.01, 1e-8, 80)
    tgt, ini = st_of(states, L, p, N, J, 50.0), st_of(states, L, p, N, J, 2.5)
    eng.set_states(tgt, ini)
    H1, d1, F1 = eng.hessian(u)
    divT, F, fid, H2 = run_engine_hessian(eng, u, tgt, ini)
    assert np.array_equal(d1, divT) and F1 == F
    assert np.array_equal(H1, H2)
    oracle_check(H1, d1, F1, L, p, N, J, 0.01, 1e-8, 80, tgt, ini, u)


def test_padded_row_overlaps_vs_general(states):
    """getHessian's row overlaps on the padded layout (csrc/fast_overlap.hpp,
    k_row_overlaps_pad and k_hessian_rows) against the general contraction
    (OCG_NO_FAST_OVL=1): the same Hessian to rounding, a different summation
    order (so the padded kernel really ran), and fused == unfused bitwise on
    both"""
    L, p, N, J = 5, 5, 5, 1.0
    u = np.random.default_rng(29).uniform(2, 10, 41)
    tgt, ini = st_of(states, L, p, N, J, 50.0), st_of(states, L, p, N, J, 2.5)

    def run():
        eng = engine(L, p, N, J, 0.01, 1e-8, 80)
        eng.set_states(tgt, ini)
        H1, d1, F1 = eng.hessian(u)
        divT, F, fid, H2 = run_engine_hessian(eng, u, tgt, ini)
        assert np.array_equal(H1, H2) and np.array_equal(d1, divT) and F1 == F
        return H1

    Hp = run()
    Hg = _with_env("OCG_NO_FAST_OVL", "1", run)
    assert np.abs(Hp - Hg).max() <= 1e-12 * np.abs(Hg).max()
    assert not np.array_equal(Hp, Hg)
    oc = O.OC(O.Stepper(L, p, N, J, 0.01, 1e-8, 80), as_orc(tgt), as_orc(ini), len(u), 0.0)
    Ho = oc.hessian(u, 8)
    assert np.abs(Hp - Ho).max() <= 1e-6 * np.abs(Ho).max()


def test_long_horizon_rows_exceed_cus(states):
    """N_t = 801 (T = 8 at config 1's dt): 799 Hessian rows, more workgroups
    than the device has CUs.  Roles are taken by ticket, so the pipeline makes
    progress whatever the dispatch order; it must equal the unfused path."""
    L, p, N, J = 5, 5, 5, 1.0
    u = np.random.default_rng(801).uniform(2, 10, 801)
    eng = engine(L, p, N, J, 0.01, 1e-8, 80)
    tgt, ini = st_of(states, L, p, N, J, 50.0), st_of(states, L, p, N, J, 2.5)
    eng.set_states(tgt, ini)
    H1, d1, F1 = eng.hessian(u)
    divT, F, fid, H2 = run_engine_hessian(eng, u, tgt, ini)
    assert np.array_equal(d1, divT) and F1 == F
    assert np.array_equal(H1, H2)
    assert np.isfinite(H1).all() and np.abs(H1).max() > 0


@pytest.mark.parametrize("K,Nt", [(3, 201), (2, 41)])
def test_hessian_multi_equals_single(states, K, Nt):
    """ocg_hessian_multi: K control vectors in one pipeline launch give each
    control's ocg_hessian bit for bit (config 1 at its full horizon, and a short
    one with a row subset), and leave control 0's trajectories in the context"""
    L, p, N, J = 5, 5, 5, 1.0
    U = np.random.default_rng(300 + K).uniform(2, 10, (K, Nt))
    rows = list(range(1, Nt - 1)) if Nt == 201 else [1, 5, 17, Nt - 2]
    eng = engine(L, p, N, J, 0.01, 1e-8, 80)
    tgt, ini = st_of(states, L, p, N, J, 50.0), st_of(states, L, p, N, J, 2.5)
    eng.set_states(tgt, ini)
    Hm, dm, Fm = eng.hessian_multi(U, rows)
    fid_m = eng.fidelities()
    for k in range(K):
        Hs, ds, Fs = eng.hessian(U[k], rows)
        assert np.array_equal(Hm[k], Hs), k
        assert np.array_equal(dm[k], ds) and Fm[k] == Fs, k
        if k == 0:
            assert np.array_equal(fid_m, eng.fidelities())


def test_hessian_multi_vs_oracle(states):
    """ocg_hessian_multi (one-wave chains, aliased LDS, two chains per CU) against
    the CPU oracle rather than against itself: three controls at N_t = 31, every
    Hessian to the north_star 1e-6 of its scale, divT and F to 1e-8 / 1e-9"""
    L, p, N, J, dt = 5, 5, 5, 1.0, 0.01
    Nt, K = 31, 3
    U = np.random.default_rng(505).uniform(2, 10, (K, Nt))
    tgt, ini = st_of(states, L, p, N, J, 50.0), st_of(states, L, p, N, J, 2.5)
    eng = engine(L, p, N, J, dt, 1e-8, 80)
    eng.set_states(tgt, ini)
    Hm, dm, Fm = eng.hessian_multi(U)
    eng.close()
    st = O.Stepper(L, p, N, J, dt, 1e-8, 80)
    for k in range(K):
        oc = O.OC(st, O.MPS(L, p, N, tgt.dims, tgt.data), O.MPS(L, p, N, ini.dims, ini.data), Nt, 0.0)
        Ho = oc.hessian(U[k], 4)
        do, Fo = oc.divT_F()
        assert abs(Fm[k] - Fo) <= 1e-9, k
        assert np.abs(dm[k] - do).max() <= 1e-8 * np.abs(do).max(), k
        assert np.abs(Hm[k] - Ho).max() <= 1e-6 * np.abs(Ho).max(), k


def test_hessian_multi_shared_cu_layout_bitwise(states, monkeypatch):
    """K >= OCG_MULTI_SHARE_K runs the chains with the two-per-CU LDS layout
    (smaller plan slots): the same Hessians bit for bit"""
    monkeypatch.setenv("OCG_MULTI_SHARE_K", "2")
    L, p, N, J = 5, 5, 5, 1.0
    U = np.random.default_rng(404).uniform(2, 10, (2, 61))
    eng = engine(L, p, N, J, 0.01, 1e-8, 80)
    tgt, ini = st_of(states, L, p, N, J, 50.0), st_of(states, L, p, N, J, 2.5)
    eng.set_states(tgt, ini)
    Hm, dm, Fm = eng.hessian_multi(U)
    for k in range(2):
        Hs, ds, Fs = eng.hessian(U[k])
        assert np.array_equal(Hm[k], Hs) and np.array_equal(dm[k], ds) and Fm[k] == Fs, k
        oracle_check(Hs, ds, Fs, L, p, N, J, 0.01, 1e-8, 80, tgt, ini, U[k])


@pytest.mark.parametrize("K", [1, 5])
def test_gradient_multi_equals_single(states, K):
    """ocg_gradient_multi: K controls' psi || xi (one launch of 2K chains) and
    batched divT / F equal ocg_propagate(.., 3) + ocg_div_t + ocg_overlap_factor
    per control bit for bit; control 0's trajectories stay"""
    L, p, N, J = 5, 5, 5, 1.0
    U = np.random.default_rng(500 + K).uniform(2, 10, (K, 201))
    eng = engine(L, p, N, J, 0.01, 1e-8, 80)
    tgt, ini = st_of(states, L, p, N, J, 50.0), st_of(states, L, p, N, J, 2.5)
    eng.set_states(tgt, ini)
    dm, Fm = eng.gradient_multi(U)
    fid_m = eng.fidelities()
    for k in range(K):
        eng.propagate(U[k], 3)
        assert np.array_equal(dm[k], eng.div_t()) and Fm[k] == eng.overlap_factor(), k
        if k == 0:
            assert np.array_equal(fid_m, eng.fidelities())


def test_flag_layout_change_between_launches(states):
    """ocg_hessian on one context at N_t = 201, then 101, then 201 (and a K = 2
    multi launch in between): the flag buffer's per-control progress and ticket
    counters move with (N, K), so stale counters must never read as published
    flags.  The last Hessian equals a fresh context's bit for bit."""
    L, p, N, J = 5, 5, 5, 1.0
    tgt, ini = st_of(states, L, p, N, J, 50.0), st_of(states, L, p, N, J, 2.5)
    rng = np.random.default_rng(1201)
    u201, u101 = rng.uniform(2, 10, 201), rng.uniform(2, 10, 101)
    eng = engine(L, p, N, J, 0.01, 1e-8, 80)
    eng.set_states(tgt, ini)
    eng.hessian(u201)
    eng.hessian(u101)
    eng.hessian_multi(rng.uniform(2, 10, (2, 101)))
    H3, d3, F3 = eng.hessian(u201)
    fresh = engine(L, p, N, J, 0.01, 1e-8, 80)
    fresh.set_states(tgt, ini)
    H0, d0, F0 = fresh.hessian(u201)
    assert np.array_equal(H3, H0) and np.array_equal(d3, d0) and F3 == F0
