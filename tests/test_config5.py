"""BASELINE configs[4]'s chain shape on the HBM-resident engine: L=50,
Npart=50, d=8 (p=9), tstep=0.01, cutoff 1e-8 (the LDS chain engine stops at
48 sites; ocg_create picks the HBM engine).  Maxm 16 (binding) so the CPU
oracle produces the golden vectors in seconds (tests/golden/c5.npz, made by
tests/golden/make_c5_fixtures.py); N_t = 5: divT, F, fidelities, gradient and
the full fidelity Hessian.  Tolerances relative to the quantities' scale
(|F| = 4.6e-3 here, so absolute 1e-6 would be vacuous): gradient and Hessian
1e-6 * max, divT 1e-8 * max.  The chi = 512 step itself is exercised by
bench.py --workload c5rows (warm-up to saturation takes minutes)."""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
L, p, N, J, DT, CUT = 50, 9, 50, 1.0, 0.01, 1e-8

pytestmark = pytest.mark.gpu


def test_c5_shape_s16_vs_oracle():
    from optimalcontrolmps_amd.native import MPS, Engine
    z = dict(np.load(os.path.join(HERE, "golden", "c5.npz"), allow_pickle=False))
    u = z["u"]
    Nt = len(u)
    eng = Engine(L, p, N, J, DT, CUT, int(z["maxm"]))  # auto: L = 50 selects the HBM engine
    eng.set_states(MPS(L, p, N, z["tgt_dims"], z["tgt_data"]), MPS(L, p, N, z["init_dims"], z["init_data"]))
    eng.propagate(u, 3)
    divT = eng.div_t()
    F = eng.overlap_factor()
    fid = eng.fidelities()
    eng.xi_dH()
    H = eng.hessian_rows(u, list(range(1, Nt - 1)), F, divT)
    g = DT * (divT * F * 1j).real
    Fo = complex(z["F"][0])
    assert abs(F - Fo) <= 1e-9 * abs(Fo)
    assert np.abs(divT - z["divT"]).max() <= 1e-8 * np.abs(z["divT"]).max()
    assert np.abs(fid - z["fid"]).max() <= 1e-12
    assert np.abs(g - z["grad"]).max() <= 1e-6 * np.abs(z["grad"]).max()
    assert np.abs(H - z["H"]).max() <= 1e-6 * np.abs(z["H"]).max()
    # the fused entry point gives the same Hessian on this engine
    H2, d2, F2 = eng.hessian(u)
    assert np.array_equal(H2, H) and F2 == F
