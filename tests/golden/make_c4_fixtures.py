"""Config-4 fixtures (TEST INFRASTRUCTURE): BASELINE configs[3]'s chain
(L=20, Npart=20, d=6 -> p=7, tstep=0.005, cutoff 1e-8) on the CPU oracle.

c4.npz:
  s32/*   Maxm = 32 (binding): psi_init = the Mott state |1..1> evolved 200
          steps at U = 2.5 by the oracle, psi_target = psi_init evolved 40
          more steps at U = 6 (config 4's |1..1> target has ~1e-10 overlap
          with psi_init, which would make every tolerance vacuous), N_t = 9
          GRAPE controls U(2,10) (seed 4040): divT, F, gradient, full fidelity
          Hessian (rows 1..7), fidelities.
  w256/*  Maxm = 256: psi_init = tests/golden/c4_warm256.npz (the Mott state
          evolved 400 steps at U = 2.5 on the GPU engine, bonds saturated at
          256); one oracle step u 2.5 -> 3.0 forward: bond dims, <psi_0|psi_1>,
          <psi_1|dH|psi_1>.
  w256h/* Maxm = 256, N_t = 5: gradient and full fidelity Hessian from the
          saturated warm state (make_w256h).
  c4_w256h<N>.npz: the w256h setting at N_t = N (make_w256hN, oracle with the
          Householder + QL eigensolver).
Run: python tests/golden/make_c4_fixtures.py [s32] [w256] [w256h]  |  w256h17
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle_ffi as O  # noqa: E402
from optimalcontrolmps_amd.states import product_state  # noqa: E402

L, p, N, J, DT, CUT = 20, 7, 20, 1.0, 0.005, 1e-8
OUT = os.path.join(HERE, "c4.npz")


def load_out():
    return dict(np.load(OUT, allow_pickle=False)) if os.path.exists(OUT) else {}


def make_s32(out):
    maxm, Nt = 32, 9
    st = O.Stepper(L, p, N, J, DT, CUT, maxm)
    mott = product_state(L, p, N)
    t0 = time.time()
    psi = st.steps(O.MPS(L, p, N, mott.dims, mott.data), np.full(201, 2.5), True)
    print(f"s32 warm-up: bonds {list(psi.bond_dims())} ({time.time() - t0:.1f}s)", flush=True)
    tgt = st.steps(psi, np.full(41, 6.0), True)
    u = np.random.default_rng(4040).uniform(2.0, 10.0, Nt)
    oc = O.OC(st, tgt, psi, Nt, 0.0)
    t0 = time.time()
    H = oc.hessian(u, 8)
    g = oc.gradient(u)
    divT, F = oc.divT_F()
    fid = oc.fidelities(u)
    print(f"s32 oracle hessian+gradient {time.time() - t0:.1f}s  max|H| {np.abs(H).max():.3e} "
          f"max|g| {np.abs(g).max():.3e}", flush=True)
    out.update({"s32/init_dims": psi.dims, "s32/init_data": psi.data, "s32/tgt_dims": tgt.dims, "s32/tgt_data": tgt.data,
                "s32/u": u, "s32/H": H, "s32/grad": g, "s32/divT": divT, "s32/F": np.array([F]),
                "s32/fid": fid, "s32/maxm": np.array(maxm)})


def make_w256(out):
    z = np.load(os.path.join(HERE, "c4_warm256.npz"), allow_pickle=False)
    st = O.Stepper(L, p, N, J, DT, CUT, 256)
    psi0 = O.MPS(L, p, N, z["dims"], z["data"])
    t0 = time.time()
    psi1 = st.steps(psi0, np.array([2.5, 3.0]), True)
    ov = st.overlap(psi0, psi1)
    dh = st.overlap_dH(psi1, psi1)
    print(f"w256 oracle step {time.time() - t0:.1f}s bonds {list(psi1.bond_dims())} <0|1> {ov} <1|dH|1> {dh}",
          flush=True)
    out.update({"w256/bonds1": np.asarray(psi1.bond_dims()), "w256/ov01": np.array([ov]),
                "w256/dH11": np.array([dh])})


def make_w256h(out, Nt=5):
    """w256h/*: config 4's real bond dimension (Maxm 256) from the saturated
    warm state: psi_target = psi_init stepped once at U = 6 (an overlapping
    target, see make_s32), N_t = 5 GRAPE controls U(2,10) (seed 5256): divT, F,
    the GRAPE gradient (gamma = 0: dt Re(divT_i F i), calcFidelityGrad
    src/OptimalControl.cpp:240-246) and the full fidelity Hessian (rows 1..3,
    calcHessianRow :251-279) on the oracle with psi || xi and the row pool on
    8 threads (~1 h on this container)."""
    z = np.load(os.path.join(HERE, "c4_warm256.npz"), allow_pickle=False)
    st = O.Stepper(L, p, N, J, DT, CUT, 256)
    psi0 = O.MPS(L, p, N, z["dims"], z["data"])
    t0 = time.time()
    tgt = st.step(psi0, 6.0, 6.0, True)
    print(f"w256h target {time.time() - t0:.1f}s bonds {list(tgt.bond_dims())}", flush=True)
    u = np.random.default_rng(5256).uniform(2.0, 10.0, Nt)
    oc = O.OC(st, tgt, psi0, Nt, 0.0)
    t0 = time.time()
    H = oc.hessian(u, 8)
    divT, F = oc.divT_F()
    g = DT * (divT * F * 1j).real
    print(f"w256h oracle hessian {time.time() - t0:.1f}s  max|H| {np.abs(H).max():.3e} "
          f"max|g| {np.abs(g).max():.3e} F {F}", flush=True)
    out.update({"w256h/tgt_dims": tgt.dims, "w256h/tgt_data": tgt.data, "w256h/u": u, "w256h/H": H,
                "w256h/grad": g, "w256h/divT": divT, "w256h/F": np.array([F])})


def make_w256hN(Nt):
    """c4_w256h<Nt>.npz: the w256h setting (same saturated psi_init and
    psi_target, Maxm 256) at a longer horizon, N_t GRAPE controls U(2,10)
    (seed 9000 + N_t): divT, F, gradient and the full fidelity Hessian (rows
    1..N_t-2, up to N_t-3 row steps each) on the oracle with 8 threads and the
    Householder + QL block eigensolver (ORC_HEEV=ql: LAPACK zheev's algorithm;
    the same bond dims and overlaps as the default cyclic Jacobi to ~5e-13 on
    the w256 step, tests/test_oracle.py::test_heev_ql_vs_numpy_and_jacobi, and
    ~14x faster: 27 s per chi = 256 step).  A file of its own; the target
    comes from c4.npz's w256h/tgt_*."""
    assert os.environ.get("ORC_HEEV") == "ql"
    z = np.load(os.path.join(HERE, "c4_warm256.npz"), allow_pickle=False)
    c = load_out()
    st = O.Stepper(L, p, N, J, DT, CUT, 256)
    psi0 = O.MPS(L, p, N, z["dims"], z["data"])
    tgt = O.MPS(L, p, N, c["w256h/tgt_dims"], c["w256h/tgt_data"])
    u = np.random.default_rng(9000 + Nt).uniform(2.0, 10.0, Nt)
    oc = O.OC(st, tgt, psi0, Nt, 0.0)
    t0 = time.time()
    H = oc.hessian(u, 8)
    divT, F = oc.divT_F()
    g = DT * (divT * F * 1j).real
    print(f"w256h{Nt} oracle hessian {time.time() - t0:.1f}s  max|H| {np.abs(H).max():.3e} "
          f"max|g| {np.abs(g).max():.3e} F {F}", flush=True)
    np.savez_compressed(os.path.join(HERE, f"c4_w256h{Nt}.npz"), u=u, H=H, grad=g, divT=divT, F=np.array([F]))


if __name__ == "__main__":
    if len(sys.argv) == 2 and sys.argv[1].startswith("w256h") and sys.argv[1][5:].isdigit():
        os.environ["ORC_HEEV"] = "ql"   # read by the oracle library at its first decomposition
        make_w256hN(int(sys.argv[1][5:]))
        sys.exit(0)
    which = sys.argv[1:] or ["s32", "w256"]
    out = load_out()
    if "s32" in which:
        make_s32(out)
    if "w256" in which:
        make_w256(out)
    if "w256h" in which:
        make_w256h(out)
    np.savez_compressed(OUT, **out)
