"""Trajectory checkpointing of the HBM engine: the
Hessian with psi_t / xi_t kept every K steps, segments recomputed and
xiHlist formed segment by segment (hbm_hessian_ckpt, selected automatically
when psi_t + xi_t + xiH_t would not fit half the free HBM — config 5 at full
N_t — or by OCG_HBM_CKPT=K) must equal the stored-trajectory path bit for bit:
the same steps, decompositions and overlaps run in another order, and every
HBM-engine kernel is batch-independent and deterministic."""
import os

import numpy as np
import pytest

import oracle_ffi as O
from conftest import state_key

HERE = os.path.dirname(os.path.abspath(__file__))
pytestmark = pytest.mark.gpu


def stored(eng, u, rows):
    eng.propagate(u, 3)
    divT = eng.div_t()
    F = eng.overlap_factor()
    eng.xi_dH()
    return eng.hessian_rows(u, rows, F, divT), divT, F


def ckpt(eng, u, rows, K, mid="1"):
    os.environ["OCG_HBM_CKPT"] = str(K)
    os.environ["OCG_HBM_CKPT_MID"] = mid
    try:
        return eng.hessian(u, rows)
    finally:
        del os.environ["OCG_HBM_CKPT"]
        del os.environ["OCG_HBM_CKPT_MID"]


@pytest.mark.parametrize("mid", ["1", "0"])
@pytest.mark.parametrize("K", [1, 3, 8])
def test_ckpt_config1_states_bitwise(states, K, mid):
    """mid "1": divT / F from psi || xi meeting in the middle (checkpoints stored on
    the way), row passes recompute only their segments; "0": the checkpoint-only
    pass, divT in the first row pass"""
    from optimalcontrolmps_amd.native import MPS, Engine
    L, p, N, J = 5, 5, 5, 1.0

    def st(U):
        k = state_key(L, p, N, J, U)
        return MPS(L, p, N, states[k + "/dims"], states[k + "/data"])
    u = np.random.default_rng(31).uniform(2, 10, 21)
    rows = list(range(1, 20))
    eng = Engine(L, p, N, J, 0.01, 1e-8, 80, engine="hbm")
    eng.set_states(st(50.0), st(2.5))
    H1, d1, F1 = stored(eng, u, rows)
    H2, d2, F2 = ckpt(eng, u, rows, K, mid)
    assert F1 == F2 and np.array_equal(d1, d2)
    assert np.array_equal(H1, H2)
    # and the CPU oracle's getHessian of the same inputs (north_star 1e-6)
    oc = O.OC(O.Stepper(L, p, N, J, 0.01, 1e-8, 80), O.MPS(L, p, N, st(50.0).dims, st(50.0).data),
              O.MPS(L, p, N, st(2.5).dims, st(2.5).data), len(u), 0.0)
    Ho = oc.hessian(u, 8)
    do, Fo = oc.divT_F()
    assert abs(F2 - Fo) <= 1e-9 and np.abs(d2 - do).max() <= 1e-8 * np.abs(do).max()
    assert np.abs(H2 - Ho).max() <= 1e-6 * np.abs(Ho).max()
    # a row subset in two batches of the time-major sweep
    sub = [3, 4, 11, 17]
    H3, _, _ = ckpt(eng, u, sub, K, mid)
    for i in sub:
        assert np.array_equal(H3[i, i:19], H1[i, i:19]) and np.array_equal(H3[i:19, i], H1[i:19, i])


def test_ckpt_config4_s32_vs_oracle():
    """config 4's chain (L=20 p=7, Maxm 32): checkpointed Hessian vs the oracle
    fixture at the north_star tolerances and bitwise vs the stored path"""
    from optimalcontrolmps_amd.native import MPS, Engine
    L, p, N, J, DT, CUT = 20, 7, 20, 1.0, 0.005, 1e-8
    c4 = dict(np.load(os.path.join(HERE, "golden", "c4.npz"), allow_pickle=False))
    u = c4["s32/u"]
    Nt = len(u)
    eng = Engine(L, p, N, J, DT, CUT, int(c4["s32/maxm"]), engine="hbm")
    eng.set_states(MPS(L, p, N, c4["s32/tgt_dims"], c4["s32/tgt_data"]),
                   MPS(L, p, N, c4["s32/init_dims"], c4["s32/init_data"]))
    rows = list(range(1, Nt - 1))
    H1, d1, F1 = stored(eng, u, rows)
    H2, d2, F2 = ckpt(eng, u, rows, 3)
    assert np.array_equal(H1, H2) and np.array_equal(d1, d2) and F1 == F2
    Ho = c4["s32/H"]
    assert np.abs(H2 - Ho).max() <= 1e-6 * np.abs(Ho).max()


def _mid(eng, u, mode):
    os.environ["OCG_HBM_MID"] = mode
    try:
        return eng.gradient(u)
    finally:
        del os.environ["OCG_HBM_MID"]


@pytest.mark.parametrize("N", [2, 3, 20, 21])
def test_gradient_meet_in_the_middle_bitwise(states, N):
    """ocg_gradient's memory-lean path (psi || xi meeting in the middle, N states
    instead of 2N: config 5 at N_t = 1001) == propagate + div_t + overlap_factor
    bit for bit, odd and even N, down to N = 2"""
    from optimalcontrolmps_amd.native import MPS, Engine
    L, p, Q, J = 5, 5, 5, 1.0

    def st(U):
        k = state_key(L, p, Q, J, U)
        return MPS(L, p, Q, states[k + "/dims"], states[k + "/data"])
    u = np.random.default_rng(40 + N).uniform(2, 10, N)
    eng = Engine(L, p, Q, J, 0.01, 1e-8, 80, engine="hbm")
    eng.set_states(st(50.0), st(2.5))
    d1, F1 = _mid(eng, u, "0")
    d2, F2 = _mid(eng, u, "1")
    assert F1 == F2 and np.array_equal(d1, d2)
    eng.close()
    oc = O.OC(O.Stepper(L, p, Q, J, 0.01, 1e-8, 80), O.MPS(L, p, Q, st(50.0).dims, st(50.0).data),
              O.MPS(L, p, Q, st(2.5).dims, st(2.5).data), N, 0.0)
    oc.gradient(u)
    do, Fo = oc.divT_F()
    assert abs(F2 - Fo) <= 1e-9 and np.abs(d2 - do).max() <= 1e-8 * np.abs(do).max()


def test_gradient_meet_in_the_middle_config4_vs_oracle():
    """config 4's chain (Maxm 32): the meet-in-the-middle gradient == the stored
    path bitwise and the oracle fixture's divT / F at the north_star tolerance"""
    from optimalcontrolmps_amd.native import MPS, Engine
    L, p, N, J, DT, CUT = 20, 7, 20, 1.0, 0.005, 1e-8
    c4 = dict(np.load(os.path.join(HERE, "golden", "c4.npz"), allow_pickle=False))
    u = c4["s32/u"]
    eng = Engine(L, p, N, J, DT, CUT, int(c4["s32/maxm"]), engine="hbm")
    eng.set_states(MPS(L, p, N, c4["s32/tgt_dims"], c4["s32/tgt_data"]),
                   MPS(L, p, N, c4["s32/init_dims"], c4["s32/init_data"]))
    d1, F1 = _mid(eng, u, "0")
    d2, F2 = _mid(eng, u, "1")
    assert F1 == F2 and np.array_equal(d1, d2)
    assert np.abs(d2 - c4["s32/divT"]).max() <= 1e-8 * np.abs(c4["s32/divT"]).max()
    g = DT * (d2 * F2 * 1j).real
    assert np.abs(g - c4["s32/grad"]).max() <= 1e-6
    eng.close()


@pytest.mark.parametrize("engine", ["hbm", "lds"])
def test_ocg_gradient_vs_oracle_config1(states, engine):
    """ocg_gradient against the CPU oracle (not a path equality): config 1's chain,
    N_t = 41, divT to 1e-8 of its scale, F to 1e-9, the GRAPE gradient to the
    north_star 1e-6 -- through the meet-in-the-middle path on the HBM engine and
    the stored trajectories on the LDS engine (the one-wave chain)"""
    import oracle_ffi as O
    from optimalcontrolmps_amd.native import MPS, Engine
    L, p, Q, J, DT = 5, 5, 5, 1.0, 0.01

    def st(U):
        k = state_key(L, p, Q, J, U)
        return states[k + "/dims"], states[k + "/data"]
    (dt_, xt), (di, xi) = st(50.0), st(2.5)
    N = 41
    u = np.random.default_rng(77).uniform(2, 10, N)
    oc = O.OC(O.Stepper(L, p, Q, J, DT, 1e-8, 80), O.MPS(L, p, Q, dt_, xt), O.MPS(L, p, Q, di, xi), N, 0.0)
    go = oc.gradient(u)
    do, Fo = oc.divT_F()
    if engine == "hbm":
        os.environ["OCG_HBM_MID"] = "1"
    try:
        eng = Engine(L, p, Q, J, DT, 1e-8, 80, engine=engine)
        eng.set_states(MPS(L, p, Q, dt_, xt), MPS(L, p, Q, di, xi))
        d, F = eng.gradient(u)
        eng.close()
    finally:
        os.environ.pop("OCG_HBM_MID", None)
    assert abs(F - Fo) <= 1e-9
    assert np.abs(d - do).max() <= 1e-8 * np.abs(do).max()
    g = DT * (d * F * 1j).real
    assert np.abs(g - go).max() <= 1e-6
