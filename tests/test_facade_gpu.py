"""The C++ facade over the HIP engine: OptimalControl<GpuTDMRG> runs the
restated reference tests (SequencingTest caching, CostTests goldens,
GradientTests FD, HessianTests seq-vs-parallel) and one getHessian that is
compared with OptimalControl<OracleTDMRG> on the same inputs
(gradient within 1e-6, Hessian within 1e-6 max|H|, north_star tolerances)."""
import numpy as np
import pytest

import facade_build as fb

# absolute floor of the central-difference gradient (eps = 1e-5): the cost
# carries ~1e-13 jitter from truncation decisions (cutoff 1e-8), i.e. ~1e-8 in
# (J+ - J-)/2eps; the reference's purely relative check is flaky on entries
# that small (it seeds with srand(time), tests/GradientTests.cpp:43)
FD_FLOOR = 5e-8
import reference_goldens as RG

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def statedir(tmp_path_factory):
    d = tmp_path_factory.mktemp("states")
    fb.write_states(str(d))
    return str(d)


def A(x):
    return np.asarray(x, dtype=float)


def test_gpu_facade_sequencing(statedir):
    r = fb.run("gpu", "sequencing", statedir)
    assert all(v is True for v in r.values()), r


def test_gpu_facade_cost_goldens(statedir):
    r = fb.run("gpu", "cost", statedir)
    assert abs(r["grape_lin_cost"] - RG.COST_LINEAR) < 5e-6
    assert abs(r["grape_ones_cost"] - RG.COST_ONES) < 5e-6
    assert abs(r["group_lin_cost"] - RG.COST_GROUP_LIN) < 5e-6
    assert abs(r["grape_lin_cost_reg"] - RG.COST_LINEAR_GAMMA1) < 1e-1
    assert abs(r["group_lin_cost_reg"] - RG.COST_GROUP_LIN_GAMMA1) < 1e-1
    assert np.abs(A(r["grape_lin_fid"])[:-1] - A(RG.FID_LINEAR)[:-1]).max() < 1e-5
    assert np.abs(A(r["group_lin_fid"])[:-1] - A(RG.FID_GROUP_LIN)[:-1]).max() < 1e-5


def test_gpu_facade_gradient_fd(statedir):
    r = fb.run("gpu", "gradient", statedir)
    for mode in ("", "_bfgs"):
        for alg, rel in [("grape", 1e-3), ("group", 2e-3)]:
            a, n = A(r[f"{alg}_ana{mode}"]), A(r[f"{alg}_num{mode}"])
            assert np.all(np.abs(a - n)[1:-1] <= np.abs(n[1:-1]) * rel + FD_FLOOR)
    assert np.abs(A(r["grad_seq"]) - A(r["grad_par"]))[1:-1].max() <= 1e-11


def test_gpu_facade_hessian_seq_vs_parallel(statedir):
    r = fb.run("gpu", "hessian", statedir)
    a, n = A(r["grape_ana"]), A(r["grape_num"])
    inner = (slice(1, -1), slice(1, -1))
    assert np.all(np.abs(a - n)[inner] <= np.abs(n)[inner] * 5e-3 + 1e-9)
    assert np.abs(A(r["hess_seq"]) - A(r["hess_par"]))[inner].max() <= 1e-11


def test_gpu_facade_matches_oracle_facade(statedir):
    g = fb.run("gpu", "golden", statedir)
    o = fb.run("oracle", "golden", statedir)
    assert abs(g["cost"] - o["cost"]) < 1e-9
    assert np.abs(A(g["grad"]) - A(o["grad"])).max() < 1e-6
    Ho = A(o["hess"])
    assert np.abs(A(g["hess"]) - Ho).max() <= 1e-6 * np.abs(Ho).max()
    assert np.abs(A(g["fid"]) - A(o["fid"])).max() < 1e-9
    assert g["psiT_bond_dims"] == o["psiT_bond_dims"]
    assert g["step_bond_dims"] == o["step_bond_dims"]


def test_gpu_facade_stub_tnlp_matches_oracle(statedir):
    """the BH_nlp call sequence through the GPU facade follows the same Newton
    path as through the oracle facade (costs 1e-9, final coefficients 1e-6,
    GROUP / GRAPE Hessians within 1e-6 max|H|)"""
    g = fb.run("gpu", "nlp", statedir)
    o = fb.run("oracle", "nlp", statedir)
    assert g["grad_consistent"] and g["hess_symmetric"]
    assert np.abs(A(g["costs"]) - A(o["costs"])).max() < 1e-9
    assert np.abs(A(g["x_final"]) - A(o["x_final"])).max() < 1e-6
    for k in ("hess_group", "hess_grape"):
        Ho = A(o[k])
        assert np.abs(A(g[k]) - Ho).max() <= 1e-6 * np.abs(Ho).max()
