"""Diagnostic: the HBM engine against the oracle on small chains (prints, does not assert).
usage: python tools/hbm_check.py [stage]   (stage: step | ovl | dh | hess | all)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_ffi as O  # noqa: E402
from conftest import state_key  # noqa: E402
from optimalcontrolmps_amd.native import MPS, Engine  # noqa: E402

states = dict(np.load(os.path.join(ROOT, "tests", "golden", "states.npz"), allow_pickle=False))


def st(L, p, N, J, U):
    k = state_key(L, p, N, J, U)
    return MPS(L, p, N, states[k + "/dims"], states[k + "/data"])


def orc(m):
    return O.MPS(m.L, m.p, m.Q, m.dims, m.data)


stage = sys.argv[1] if len(sys.argv) > 1 else "all"
for (L, p, N, J, Ui, Uf) in [(5, 5, 5, 1.0, 2.5, 50.0), (4, 3, 4, 1.0, 2.0, 10.0), (5, 6, 5, 1.0, 2.0, 12.0)]:
    print(f"== L={L} p={p} N={N}", flush=True)
    eng = Engine(L, p, N, J, 0.01, 1e-8, 0, engine="hbm")
    o = O.Stepper(L, p, N, J, 0.01, 1e-8)
    a, b = st(L, p, N, J, Ui), st(L, p, N, J, Uf)
    if stage in ("ovl", "all"):
        t = time.time()
        g1, o1 = eng.overlap(a, b), o.overlap(orc(a), orc(b))
        g2, o2 = eng.overlap(a, b, True), o.overlap_dH(orc(a), orc(b))
        print(f"overlap  gpu {g1:.12f} orc {o1:.12f} |d|={abs(g1 - o1):.2e}; dH |d|={abs(g2 - o2):.2e} "
              f"({time.time() - t:.2f}s)", flush=True)
    if stage in ("step", "all"):
        for fwd in (True, False):
            t = time.time()
            u = np.random.default_rng(7).uniform(2, 10, 4)
            g = eng.steps(a, u, fwd)
            r = o.steps(orc(a), u, fwd)
            ov = o.overlap(r, orc(g))
            print(f"steps fwd={fwd}: dims gpu {list(g.bond_dims())} orc {list(r.bond_dims())} "
                  f"|<o|g>|-1 = {abs(ov) - 1:.2e} norm-1 = {abs(o.overlap(orc(g), orc(g))) - 1:.2e} "
                  f"({time.time() - t:.2f}s)", flush=True)
    if stage in ("dh", "all"):
        t = time.time()
        g, nrm = eng.apply_dH(a)
        r = o.apply_dH(orc(a))
        no = np.sqrt(o.overlap(r, r).real)
        print(f"apply_dH: dims gpu {list(g.bond_dims())} orc {list(r.bond_dims())} norm gpu {nrm:.12f} orc {no:.12f} "
              f"<o|g>/n^2-1 = {o.overlap(r, orc(g)).real / no / no - 1:.2e} ({time.time() - t:.2f}s)", flush=True)
    if stage in ("hess", "all"):
        u = np.random.default_rng(99).uniform(2, 10, 9)
        t = time.time()
        eng.set_states(b, a)
        eng.propagate(u, 3)
        divT = eng.div_t()
        F = eng.overlap_factor()
        eng.xi_dH()
        H = eng.hessian_rows(u, list(range(1, len(u) - 1)), F, divT)
        tg = time.time() - t
        oc = O.OC(O.Stepper(L, p, N, J, 0.01, 1e-8), orc(b), orc(a), len(u), 0.0)
        Ho = oc.hessian(u, 4)
        go = oc.gradient(u)
        g = 0.01 * (divT * F * 1j).real
        print(f"hessian: rel err {np.abs(H - Ho).max() / np.abs(Ho).max():.2e}  grad err {np.abs(g - go).max():.2e} "
              f"({tg:.2f}s)", flush=True)
    eng.close()
