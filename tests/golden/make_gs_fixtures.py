"""Ground-state fixtures at L = 10 (TEST INFRASTRUCTURE): the reference
prepares psi_init / psi_target with ITensor DMRG (include/InitializeState.hpp:
18-117); the build prepares them by imaginary-time evolution on the device
(ocg_ground_state).  Pinned here by exact diagonalisation of the same
Hamiltonian, H = -J sum_i (a_i a^dag_{i+1} + h.c.) + U/2 sum_i n_i (n_i - 1),
in the N-particle sector of L = 10 sites with local dimension p = 5
(d = 4, as BASELINE config 1): scipy's sparse Lanczos (eigsh) on the ~85k
sector states.  Stored: E0, <n_i>, Re <a^dag_i a_{i+1}> per U.

Run: python tests/golden/make_gs_fixtures.py  ->  tests/golden/gs_L10.npz
"""
import os
import sys

import numpy as np
import scipy.sparse as sp
from scipy.sparse.linalg import eigsh

HERE = os.path.dirname(os.path.abspath(__file__))
L, P, NPART, J = 10, 5, 10, 1.0
US = (2.0, 6.0)


def digits(L, p):
    """digit k (site k+1, most significant first) of every full index"""
    return np.indices((p,) * L, dtype=np.int8).reshape(L, -1)


def sector(L, p, N):
    dg = digits(L, p)
    idx = np.nonzero(dg.sum(axis=0, dtype=np.int32) == N)[0]
    return idx, dg[:, idx].astype(np.int64)


def hamiltonian(L, p, N, J, U):
    idx, dg = sector(L, p, N)
    D = len(idx)
    diag = 0.5 * U * (dg * (dg - 1)).sum(axis=0)
    rows, cols, vals = [np.arange(D)], [np.arange(D)], [diag]
    w = p ** np.arange(L - 1, -1, -1, dtype=np.int64)   # weight of site k (0-based)
    for i in range(L - 1):
        n1, n2 = dg[i], dg[i + 1]
        ok = (n1 >= 1) & (n2 + 1 < p)                       # a_i a^dag_{i+1}
        tgt = idx[ok] - w[i] + w[i + 1]
        amp = -J * np.sqrt(n1[ok] * (n2[ok] + 1.0))
        r = np.searchsorted(idx, tgt)
        rows += [r, np.nonzero(ok)[0]]
        cols += [np.nonzero(ok)[0], r]
        vals += [amp, amp]                                   # and its Hermitian conjugate
    H = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(D, D))
    return H, idx, dg


def observables_sector(v, dg, idx, L, p):
    """<n_i>, Re <a^dag_i a_{i+1}> of a normalised sector vector v"""
    pr = np.abs(v) ** 2
    n = (dg * pr).sum(axis=1)
    w = p ** np.arange(L - 1, -1, -1, dtype=np.int64)
    hop = []
    for i in range(L - 1):
        n1, n2 = dg[i], dg[i + 1]
        ok = (n2 >= 1) & (n1 + 1 < p)                        # a^dag_i a_{i+1} |x>
        tgt = idx[ok] + w[i] - w[i + 1]
        r = np.searchsorted(idx, tgt)
        hop.append(float(np.real(np.vdot(v[r], v[ok] * np.sqrt((n1[ok] + 1.0) * n2[ok])))))
    return n, np.array(hop)


def main():
    out = {}
    for U in US:
        H, idx, dg = hamiltonian(L, P, NPART, J, U)
        w, v = eigsh(H, k=2, which="SA", tol=1e-13)
        o = np.argsort(w)
        E0, E1, g = w[o[0]], w[o[1]], v[:, o[0]]
        n, hop = observables_sector(g, dg, idx, L, P)
        Echk = -J * 2 * hop.sum() + 0.5 * U * ((dg * (dg - 1)) * np.abs(g) ** 2).sum()
        print(f"U={U}: D={len(idx)} E0={E0:.12f} gap={E1 - E0:.6f} (E from observables {Echk:.12f}) "
              f"<n>={np.round(n, 6)}", flush=True)
        key = f"U{U:g}"
        out.update({f"{key}/E0": np.array(E0), f"{key}/gap": np.array(E1 - E0), f"{key}/n": n, f"{key}/hop": hop})
    np.savez_compressed(os.path.join(HERE, "gs_L10.npz"), **out)


if __name__ == "__main__":
    sys.exit(main())
