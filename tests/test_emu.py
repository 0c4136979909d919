"""CPU emulation of the device bodies (tests/emu: one std::thread per lane,
the wave intrinsics DPP / bpermute / permute / ballot emulated): the one-wave
padded chain (csrc/fast_chain.hpp) against the general chain and the oracle
without a GPU.  Test infrastructure only; the GPU parity is in
test_fast_chain.py."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_ffi as O
from optimalcontrolmps_amd import ed

HERE = os.path.dirname(os.path.abspath(__file__))
EMU = os.path.join(HERE, "emu")


@pytest.fixture(scope="module")
def E():
    subprocess.check_call(["make", "-s", "-C", EMU], stdout=subprocess.DEVNULL)
    sys.path.insert(0, EMU)
    import emu_ffi
    return emu_ffi


def _gs(Lx, px, Qx, J, U):
    return ed.mps_from_full(ed.ground_state_full(Lx, px, Qx, J, U)[0], Lx, px, Qx)


@pytest.mark.parametrize("cfg", [(5, 5, 5, 1.0, 80, 1e-8, 2.5), (5, 5, 5, 1.0, 3, 1e-8, 2.5),
                                 (5, 5, 5, 1.0, 80, 1e-4, 2.5), (4, 3, 4, 1.0, 5000, 1e-8, 2.0)])
def test_emulated_fast_steps(E, cfg):
    Lx, px, Qx, J, maxm, cut, U = cfg
    d, x = _gs(Lx, px, Qx, J, U)
    u = np.random.default_rng(1).uniform(2.0, 10.0, 4)
    st = O.Stepper(Lx, px, Qx, J, 0.01, cut, maxm)
    fast = E.Emu(Lx, px, Qx, J, 0.01, cut, maxm, True)
    for fwd in (True, False):
        d2, x2 = fast.steps(d, x, u, fwd)
        ref = st.steps(O.MPS(Lx, px, Qx, d, x), u, fwd)
        b = O.MPS(Lx, px, Qx, d2, x2)
        assert list(ref.bond_dims()) == list(b.bond_dims())
        assert abs(abs(st.overlap(ref, b)) - 1.0) <= 1e-12


def test_emulated_fast_pipeline(E):
    """the fused getHessian pipeline with the one-wave chain in every step role
    (psi / xi chains with write-through publication, rows after the general
    chain's exactApplyMPO) against the general chain and the oracle"""
    Lx, px, Qx, J, dt, cut, maxm = 5, 5, 5, 1.0, 0.01, 1e-8, 80
    di, xi = _gs(Lx, px, Qx, J, 2.5)
    dtg, xtg = _gs(Lx, px, Qx, J, 50.0)
    N = 5
    u = np.random.default_rng(3).uniform(2.0, 10.0, N)
    Hf, dvf, Ff = E.Emu(Lx, px, Qx, J, dt, cut, maxm, True).hessian_fused(dtg, xtg, di, xi, u)
    Hg, dvg, Fg = E.Emu(Lx, px, Qx, J, dt, cut, maxm, False).hessian_fused(dtg, xtg, di, xi, u)
    oc = O.OC(O.Stepper(Lx, px, Qx, J, dt, cut, maxm), O.MPS(Lx, px, Qx, dtg, xtg), O.MPS(Lx, px, Qx, di, xi), N, 0.0)
    Ho = oc.hessian(u, 2)
    assert np.abs(Hf - Ho).max() <= 1e-12 * np.abs(Ho).max()
    assert np.abs(Hf - Hg).max() <= 1e-12 * np.abs(Ho).max()
    assert np.abs(dvf - dvg).max() <= 1e-14 and abs(Ff - Fg) <= 1e-14


def test_emulated_padded_overlap(E, monkeypatch):
    """the row overlaps on the padded layout (csrc/fast_overlap.hpp): fused
    (k_row_overlaps_pad) == unfused (k_hessian_rows on the one-wave chain)
    bitwise, both against the general contraction (OCG_NO_FAST_OVL=1) and the
    oracle"""
    Lx, px, Qx, J, dt, cut, maxm = 5, 5, 5, 1.0, 0.01, 1e-8, 80
    di, xi = _gs(Lx, px, Qx, J, 2.5)
    dtg, xtg = _gs(Lx, px, Qx, J, 50.0)
    N = 6
    u = np.random.default_rng(5).uniform(2.0, 10.0, N)
    e = E.Emu(Lx, px, Qx, J, dt, cut, maxm, True)
    Hf, dvf, Ff = e.hessian_fused(dtg, xtg, di, xi, u)
    Hu, dvu, Fu = e.hessian(dtg, xtg, di, xi, u)
    monkeypatch.setenv("OCG_NO_FAST_OVL", "1")
    Hg, _, _ = E.Emu(Lx, px, Qx, J, dt, cut, maxm, True).hessian_fused(dtg, xtg, di, xi, u)
    monkeypatch.delenv("OCG_NO_FAST_OVL")
    oc = O.OC(O.Stepper(Lx, px, Qx, J, dt, cut, maxm), O.MPS(Lx, px, Qx, dtg, xtg), O.MPS(Lx, px, Qx, di, xi), N, 0.0)
    Ho = oc.hessian(u, 2)
    m = np.abs(Ho).max()
    assert np.array_equal(Hf, Hu)
    assert np.abs(Hf - Hg).max() <= 1e-13 * m
    assert np.abs(Hf - Ho).max() <= 1e-12 * m
    assert not np.array_equal(Hf, Hg)  # the padded contraction ran (a different summation order)


@pytest.mark.parametrize("cfg", [(5, 5, 5, 1.0, 2.5, 50.0), (4, 3, 4, 1.0, 2.0, 10.0)])
def test_emulated_padded_overlap_pairs(E, cfg):
    """<x|y> and <x|dH|y> on the padded contraction (k_overlaps_pad's body:
    divT, F, fidelities on the one-wave contexts) against the oracle, also for
    stepped states whose bond dimensions sit below the padded bounds"""
    Lx, px, Qx, J, U1, U2 = cfg
    d1, x1 = _gs(Lx, px, Qx, J, U1)
    d2, x2 = _gs(Lx, px, Qx, J, U2)
    st = O.Stepper(Lx, px, Qx, J, 0.01, 1e-4, 80)
    e = E.Emu(Lx, px, Qx, J, 0.01, 1e-4, 80, True)
    d3, x3 = e.steps(d1, x1, np.random.default_rng(9).uniform(2.0, 10.0, 6), True)
    for (da, xa), (db, xb) in [((d1, x1), (d2, x2)), ((d2, x2), (d3, x3)), ((d3, x3), (d3, x3))]:
        a, b = O.MPS(Lx, px, Qx, da, xa), O.MPS(Lx, px, Qx, db, xb)
        assert abs(e.overlap_pad(da, xa, db, xb) - st.overlap(a, b)) <= 1e-12
        assert abs(e.overlap_pad(da, xa, db, xb, True) - st.overlap_dH(a, b)) <= 1e-12 * max(1.0, abs(st.overlap_dH(a, b)))
