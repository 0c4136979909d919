"""The HBM engine's decomposition path (Gram -> Hermitian eigensolver ->
truncation -> eigenvectors -> factors: ITensor denmatDecomp, called at
src/BH_tDMRG.cpp:178, :191, :209) on caller-supplied blocks through
ocg_denmat_decomp, against numpy's SVD (an independent LAPACK result).

Config 5 (chi = 512, p = 9) produces Gram blocks of order 209..512, which run
on the blocked kernels (k_heev_vals_big, k_heev_bt / CholeskyQR2); the config
tests at Maxm 16/32 never reach them.  Checked per block, all gauge-invariant:
* kept count = the truncation rule on numpy's spectrum (oracle truncate_count:
  discard the smallest while their sum < cutoff * total, cap Maxm);
* resolved eigenvalues = numpy's squared singular values (1e-12 of the largest);
* A has orthonormal columns (1e-11);
* A B = the best rank-k approximation of M (1e-9 of ||M||_F: the Gram route
  resolves directions of singular value s to ~eps s_max^2 / s^2).
"""
import numpy as np
import pytest

import oracle_ffi as O

pytestmark = pytest.mark.gpu

L, p, NPART = 20, 7, 20   # an HBM-engine context (the chain shape does not enter)


def block(rng, n, c, spec, rank=None):
    """n x c complex with singular values spec (length min(n, c) or rank)"""
    r = len(spec) if rank is None else rank
    U, _ = np.linalg.qr(rng.normal(size=(n, r)) + 1j * rng.normal(size=(n, r)))
    V, _ = np.linalg.qr(rng.normal(size=(c, r)) + 1j * rng.normal(size=(c, r)))
    return (U * np.asarray(spec[:r])) @ V.conj().T


def check(M, res, cutoff, maxm):
    k, w, A, B = res
    s = np.linalg.svd(M, compute_uv=False)
    lam = s ** 2
    k_ref = O.truncate(lam, cutoff, maxm)
    assert k == k_ref, (M.shape, k, k_ref)
    # resolved eigenvalues (the kept ones and every one above the unresolved threshold)
    wd = np.sort(w)[::-1]
    assert np.abs(wd[:k] - lam[:k]).max() <= 1e-12 * lam[0], M.shape
    assert np.abs(A.conj().T @ A - np.eye(k)).max() <= 1e-11, M.shape
    U, s2, Vh = np.linalg.svd(M, full_matrices=False)
    Mk = (U[:, :k] * s2[:k]) @ Vh[:k]
    assert np.linalg.norm(A @ B - Mk) <= 1e-9 * np.linalg.norm(M), M.shape


@pytest.fixture(scope="module")
def eng():
    from optimalcontrolmps_amd.native import Engine
    e = Engine(L, p, NPART, 1.0, 0.005, 1e-8, 512, engine="hbm")
    yield e
    e.close()


@pytest.mark.parametrize("n,c", [(209, 240), (256, 256), (320, 448), (448, 560), (512, 512)])
def test_blocked_orders_vs_numpy(eng, n, c):
    """one block per call on the blocked large-order path, geometric spectrum
    (cutoff 1e-8 keeps ~90 of n)"""
    rng = np.random.default_rng(n * 1000 + c)
    spec = np.exp(-np.arange(n) / 5.0)
    M = block(rng, n, c, spec)
    check(M, eng.denmat_decomp([M], 1e-8, 512)[0], 1e-8, 512)


def test_mixed_orders_one_batch(eng):
    """register, LDS and blocked kernels in one decomposition pass (the blocked
    one on the side stream), slow spectra so that Maxm binds on the big ones"""
    rng = np.random.default_rng(77)
    shapes = [(12, 30), (48, 64), (130, 200), (208, 208), (209, 300), (300, 300), (512, 700)]
    Ms = [block(rng, n, c, 1.0 / (1.0 + np.arange(n)) ** 1.5) for n, c in shapes]
    res = eng.denmat_decomp(Ms, 1e-8, 128)
    for M, r in zip(Ms, res):
        check(M, r, 1e-8, 128)
    assert max(r[0] for r in res) == 128


def test_rank_deficient_and_clustered(eng):
    """exact null space (rank 100 of order 300) and a degenerate cluster inside
    the kept set (k_heev_vecs / CholeskyQR2 on repeated eigenvalues)"""
    rng = np.random.default_rng(5)
    M1 = block(rng, 300, 320, np.exp(-np.arange(100) / 10.0), rank=100)
    spec = np.exp(-np.arange(450) / 6.0)
    spec[3:9] = spec[3]  # six-fold degenerate singular value
    M2 = block(rng, 450, 450, spec)
    res = eng.denmat_decomp([M1, M2], 1e-8, 512)
    check(M1, res[0], 1e-8, 512)
    check(M2, res[1], 1e-8, 512)


def test_lds_engine_refuses(states):
    from optimalcontrolmps_amd.native import Engine, OcgError
    e = Engine(5, 5, 5, 1.0, 0.01, 1e-8, 80, engine="lds")
    with pytest.raises(OcgError):
        e.denmat_decomp([np.eye(4, dtype=complex)])
    e.close()


def test_maxm_boundary_threshold(eng, monkeypatch):
    """OCG_HBM_THRESH=1: decompositions with more than Maxm + 1 eigenvalues
    resolve only those above the (Maxm + 1)-th largest (k_heev_thresh +
    k_heev_bisect): Maxm binding (slow spectrum) and the cutoff binding first
    (fast spectrum, the rule's suffix sums from the exact trace), against numpy,
    and against the default path that resolves every eigenvalue: same kept
    counts, same factors to rounding"""
    from optimalcontrolmps_amd.native import Engine
    rng = np.random.default_rng(2024)
    Ms = [block(rng, 200, 260, np.exp(-np.arange(200) / 15.0)),
          block(rng, 200, 200, np.exp(-np.arange(200) / 3.0)),
          block(rng, 150, 180, np.exp(-np.arange(150) / 8.0))]
    monkeypatch.setenv("OCG_HBM_THRESH", "1")
    e1 = Engine(L, p, NPART, 1.0, 0.005, 1e-8, 512, engine="hbm")
    res = e1.denmat_decomp(Ms, 1e-8, 60)
    e1.close()
    for M, r in zip(Ms, res):
        check(M, r, 1e-8, 60)
    assert res[0][0] == 60 and res[1][0] < 60
    ref = eng.denmat_decomp(Ms, 1e-8, 60)
    for r, r0 in zip(res, ref):
        assert r[0] == r0[0]
        assert np.abs(r[2] @ r[3] - r0[2] @ r0[3]).max() <= 1e-12 * np.abs(r0[2] @ r0[3]).max()


def _decomp_env(monkeypatch, env, Ms, cutoff, maxm):
    from optimalcontrolmps_amd.native import Engine
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    e = Engine(L, p, NPART, 1.0, 0.005, 1e-8, 512, engine="hbm")
    res = e.denmat_decomp(Ms, cutoff, maxm)
    st = e.path_stats()
    e.close()
    for k in env:
        monkeypatch.delenv(k)
    return res, st


def test_split_multisection_vs_numpy_and_in_kernel(monkeypatch):
    """register-path blocks of order >= 96 (config 4's largest sectors) leave
    their eigenvalues to k_heev_bisect_split (16 per
    workgroup, 16 threads each): against numpy, and against the in-kernel
    multisection (OCG_HBM_SPLITMIN=0) to rounding, including a rank-deficient
    block (unresolved eigenvalues below the threshold: the last workgroup sets their mean)
    and a degenerate cluster; orders below the threshold stay in-kernel"""
    rng = np.random.default_rng(96)
    spec = np.exp(-np.arange(160) / 6.0)
    spec[4:9] = spec[4]
    Ms = [block(rng, 96, 130, np.exp(-np.arange(96) / 5.0)),
          block(rng, 150, 170, np.exp(-np.arange(60) / 4.0), rank=60),
          block(rng, 160, 160, spec),
          block(rng, 192, 230, 1.0 / (1.0 + np.arange(192)) ** 1.5),
          block(rng, 208, 208, np.exp(-np.arange(208) / 9.0)),
          block(rng, 64, 80, np.exp(-np.arange(64) / 3.0))]
    for maxm in (512, 70):
        res, _ = _decomp_env(monkeypatch, {}, Ms, 1e-8, maxm)
        ref, _ = _decomp_env(monkeypatch, {"OCG_HBM_SPLITMIN": "0"}, Ms, 1e-8, maxm)
        for M, r, r0 in zip(Ms, res, ref):
            check(M, r, 1e-8, maxm)
            assert r[0] == r0[0]
            assert np.abs(r[2] @ r[3] - r0[2] @ r0[3]).max() <= 1e-11 * np.abs(r0[2] @ r0[3]).max()


def test_coop_members_bitwise_and_vs_one_cu(monkeypatch):
    """k_heev_vals_coop (hbm_coop.hpp): the multi-CU reduction gives the same
    bits whatever the number G of workgroups per block (1, 3, 8, 16: the
    host picks G from the CUs a launch leaves, so batched / pipelined runs must
    not depend on it), matches numpy, and matches the one-CU kernels
    (OCG_HBM_COOP=0) to rounding; orders 209..512 (config 5's sectors at
    chi = 512)"""
    rng = np.random.default_rng(606)
    shapes = [(209, 230), (256, 300), (384, 384), (512, 640)]
    Ms = [block(rng, n, c, np.exp(-np.arange(n) / 9.0)) for n, c in shapes]
    ref, st = _decomp_env(monkeypatch, {"OCG_HBM_COOPG": "1"}, Ms, 1e-8, 512)
    assert st["coop_groups"] == len(Ms) and st["coop_fallbacks"] == 0
    for M, r in zip(Ms, ref):
        check(M, r, 1e-8, 512)
    for g in ("3", "8", "16"):
        res, st = _decomp_env(monkeypatch, {"OCG_HBM_COOPG": g}, Ms, 1e-8, 512)
        assert st["coop_fallbacks"] == 0
        for r, r0 in zip(res, ref):
            assert r[0] == r0[0] and np.array_equal(r[1], r0[1]), g
            assert np.array_equal(r[2], r0[2]) and np.array_equal(r[3], r0[3]), g
    one, st = _decomp_env(monkeypatch, {"OCG_HBM_COOP": "0"}, Ms, 1e-8, 512)
    assert st["coop_groups"] == 0
    for r, r0 in zip(one, ref):
        assert r[0] == r0[0]
        assert np.abs(r[2] @ r[3] - r0[2] @ r0[3]).max() <= 1e-11 * np.abs(r0[2] @ r0[3]).max()


def test_coop_fallback_one_cu(monkeypatch):
    """a group that gives up a wait (OCG_HBM_COOP_TMO=0: at its first wait)
    raises its abort word; k_heev_vals_coop_fix restores the block's lower
    triangle from the untouched upper one and reduces it on one CU: the
    result is the one-CU kernel's on that (exactly Hermitian) block, i.e. the
    one-CU kernel's to rounding (the Gram GEMM's two triangles differ in the
    last bits), and path_stats counts it"""
    rng = np.random.default_rng(707)
    Ms = [block(rng, n, c, np.exp(-np.arange(n) / 7.0)) for n, c in [(240, 260), (400, 420)]]
    fb, st = _decomp_env(monkeypatch, {"OCG_HBM_COOP_TMO": "0", "OCG_HBM_COOPG": "4"}, Ms, 1e-8, 512)
    assert st["coop_fallbacks"] == len(Ms)
    one, _ = _decomp_env(monkeypatch, {"OCG_HBM_COOP": "0", "OCG_HBM_BIGMIN": "193"}, Ms, 1e-8, 512)
    for M, r, r1 in zip(Ms, fb, one):
        check(M, r, 1e-8, 512)
        assert r[0] == r1[0]
        assert np.abs(r[1][:r[0]] - r1[1][:r[0]]).max() <= 1e-13 * r1[1][0]
        assert np.abs(r[2] @ r[3] - r1[2] @ r1[3]).max() <= 1e-11 * np.abs(r1[2] @ r1[3]).max()
