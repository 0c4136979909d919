"""Ground-state preparation by exact diagonalisation + dense helpers.

Host-side utility, NOT on the hot path: stands in for the reference's
ITensor-DMRG `InitializeState` (include/InitializeState.hpp:18-65), which is
out of scope (§8f rank 3).  For the small chains of the
reference's tests and of BASELINE config 1 (L=5) the fixed-N sector is tiny
(<= 126 states), so the ground state is solved exactly: same Hamiltonian
    H = -J sum_i (a_i a^dag_{i+1} + h.c.) + U/2 sum_i n_i (n_i - 1)
in the fixed-particle-number sector.  `exact_step` is an untruncated dense
restatement of one Trotter step used by tests as a state-vector cross-check.

Compact MPS format (shared with include/ocmps.h and the oracle):
    dims: int32[(L+1)*(Q+1)]  bond b, sector q (left particle count)
    data: complex128, for k=1..L, q=0..Q, n=0..p-1 (q+n<=Q): block of
          dims[k-1][q] x dims[k][q+n], row-major.
"""
from __future__ import annotations

import itertools

import numpy as np


# --------------------------------------------------------------------- basis
def sector_basis(L: int, p: int, N: int):
    confs = [c for c in itertools.product(range(p), repeat=L) if sum(c) == N]
    return confs, {c: i for i, c in enumerate(confs)}


def bh_hamiltonian(L: int, p: int, N: int, J: float, U: float) -> np.ndarray:
    confs, index = sector_basis(L, p, N)
    D = len(confs)
    H = np.zeros((D, D))
    for col, c in enumerate(confs):
        H[col, col] += 0.5 * U * sum(n * (n - 1) for n in c)
        for i in range(L - 1):
            n1, n2 = c[i], c[i + 1]
            # a_i a^dag_{i+1}
            if n1 >= 1 and n2 + 1 < p:
                d = list(c); d[i] -= 1; d[i + 1] += 1
                H[index[tuple(d)], col] += -J * np.sqrt(n1) * np.sqrt(n2 + 1)
            # a^dag_i a_{i+1}
            if n2 >= 1 and n1 + 1 < p:
                d = list(c); d[i] += 1; d[i + 1] -= 1
                H[index[tuple(d)], col] += -J * np.sqrt(n1 + 1) * np.sqrt(n2)
    return H


def ground_state_full(L: int, p: int, N: int, J: float, U: float):
    """Ground state as a dense p**L vector (site 1 most significant)."""
    confs, _ = sector_basis(L, p, N)
    H = bh_hamiltonian(L, p, N, J, U)
    w, v = np.linalg.eigh(H)
    g = v[:, 0]
    g = g * np.sign(g[np.argmax(np.abs(g))])
    full = np.zeros(p ** L, dtype=complex)
    for amp, c in zip(g, confs):
        full[conf_index(c, p)] = amp
    return full, w[0]


def conf_index(c, p):
    i = 0
    for n in c:
        i = i * p + n
    return i


def counts(nsites: int, p: int) -> np.ndarray:
    """particle count of every config of `nsites` sites (site 1 most significant)."""
    if nsites == 0:
        return np.zeros(1, dtype=int)
    g = np.indices((p,) * nsites).reshape(nsites, -1)
    return g.sum(axis=0)


# -------------------------------------------------------------- MPS <-> vector
def mps_from_full(psi: np.ndarray, L: int, p: int, Q: int, rel_cut: float = 1e-16):
    """Right-canonical MPS (centre at site 1) from a dense fixed-N vector by
    per-sector SVDs from the right.  Returns (dims[(L+1),(Q+1)], data)."""
    dims = np.zeros((L + 1, Q + 1), dtype=np.int32)
    dims[0, 0] = 1
    dims[L, Q] = 1
    qn_k = np.array([Q])                     # labels of bond L states
    cur = psi.reshape(p ** L, 1)
    sites = {}
    total = np.vdot(psi, psi).real
    for k in range(L, 1, -1):
        chi = cur.shape[1]
        M = cur.reshape(p ** (k - 1), p * chi)          # cols: n*chi + c
        rowq = counts(k - 1, p)
        coln = np.repeat(np.arange(p), chi)
        colc = np.tile(np.arange(chi), p)
        colq = qn_k[colc] - coln
        new_cols, new_q, blocks = [], [], {}
        for q in range(Q + 1):
            R = np.where(rowq == q)[0]
            C = np.where(colq == q)[0]
            if len(R) == 0 or len(C) == 0:
                continue
            B = M[np.ix_(R, C)]
            U_, S, Vh = np.linalg.svd(B, full_matrices=False)
            keep = S ** 2 > rel_cut * total
            kq = int(keep.sum())
            if kq == 0:
                continue
            blocks[q] = (R, C, U_[:, :kq] * S[:kq], Vh[:kq])
            dims[k - 1, q] = kq
        # assemble new cur (p^(k-1) x chi_{k-1}) sorted by q, and site k blocks
        offs = np.concatenate([[0], np.cumsum(dims[k - 1])])
        chi_new = int(dims[k - 1].sum())
        cur_new = np.zeros((p ** (k - 1), chi_new), dtype=complex)
        qn_new = np.zeros(chi_new, dtype=int)
        offs_k = np.concatenate([[0], np.cumsum(dims[k])])
        site = {}
        for q, (R, C, US, Vh) in blocks.items():
            cur_new[np.ix_(R, np.arange(offs[q], offs[q + 1]))] = US
            qn_new[offs[q]:offs[q + 1]] = q
            for n in range(p):
                qr = q + n
                if qr > Q or dims[k, qr] == 0:
                    continue
                blk = np.zeros((dims[k - 1, q], dims[k, qr]), dtype=complex)
                for ci, col in enumerate(C):
                    if coln[col] == n:
                        blk[:, colc[col] - offs_k[qr]] = Vh[:, ci]
                site[(q, n)] = blk
        sites[k] = site
        cur = cur_new
        qn_k = qn_new
    # site 1: bond 0 is (q=0, dim 1)
    offs1 = np.concatenate([[0], np.cumsum(dims[1])])
    site = {}
    for n in range(p):
        if n <= Q and dims[1, n] > 0:
            site[(0, n)] = cur[n, offs1[n]:offs1[n + 1]].reshape(1, -1).copy()
    sites[1] = site
    data = []
    for k in range(1, L + 1):
        for q in range(Q + 1):
            for n in range(p):
                if q + n > Q:
                    continue
                r, c = dims[k - 1, q], dims[k, q + n]
                if r == 0 or c == 0:
                    continue
                data.append(sites[k].get((q, n), np.zeros((r, c), complex)).ravel())
    data = np.concatenate(data) if data else np.zeros(0, complex)
    return dims, data


def mps_blocks(dims, data, L, p, Q):
    """yield (k, q, n, block) in compact order."""
    dims = np.asarray(dims).reshape(L + 1, Q + 1)
    off = 0
    for k in range(1, L + 1):
        for q in range(Q + 1):
            for n in range(p):
                if q + n > Q:
                    continue
                r, c = dims[k - 1, q], dims[k, q + n]
                if r == 0 or c == 0:
                    continue
                yield k, q, n, np.asarray(data[off:off + r * c]).reshape(r, c)
                off += r * c


def nelem(dims, L, p, Q):
    dims = np.asarray(dims).reshape(L + 1, Q + 1)
    s = 0
    for k in range(1, L + 1):
        for q in range(Q + 1):
            for n in range(p):
                if q + n <= Q:
                    s += int(dims[k - 1, q]) * int(dims[k, q + n])
    return s


def full_from_mps(dims, data, L, p, Q) -> np.ndarray:
    dims = np.asarray(dims).reshape(L + 1, Q + 1)
    dense = []
    for k in range(1, L + 1):
        chil, chir = int(dims[k - 1].sum()), int(dims[k].sum())
        dense.append(np.zeros((chil, p, chir), complex))
    offs = [np.concatenate([[0], np.cumsum(dims[b])]) for b in range(L + 1)]
    for k, q, n, blk in mps_blocks(dims, data, L, p, Q):
        a0, c0 = offs[k - 1][q], offs[k][q + n]
        dense[k - 1][a0:a0 + blk.shape[0], n, c0:c0 + blk.shape[1]] = blk
    T = np.ones((1, 1), complex)
    for k in range(L):
        A = dense[k]
        T = np.einsum("xa,anc->xnc", T, A).reshape(-1, A.shape[2])
    return T.reshape(-1)


# ------------------------------------------------------- exact Trotter steps
def hop_gate(p: int, J: float, tau: float) -> np.ndarray:
    D = p * p
    h = np.zeros((D, D))
    for n1 in range(p):
        for n2 in range(p):
            if n1 >= 1 and n2 + 1 < p:
                h[(n1 - 1) * p + n2 + 1, n1 * p + n2] += -J * np.sqrt(n1) * np.sqrt(n2 + 1)
            if n2 >= 1 and n1 + 1 < p:
                h[(n1 + 1) * p + n2 - 1, n1 * p + n2] += -J * np.sqrt(n1 + 1) * np.sqrt(n2)
    w, v = np.linalg.eigh(h)
    return (v * np.exp(-1j * tau * w)) @ v.T


def gate_list(L: int):
    g = [(i, i + 1) for i in range(1, L, 2)]
    off = 2 if L % 2 == 0 else 1
    g += [(i, i + 1) for i in range(L - off, 0, -2)]
    return g


def exact_step(psi: np.ndarray, L: int, p: int, J: float, dt: float, u_from: float, u_to: float,
               forward: bool = True) -> np.ndarray:
    """Untruncated version of BH_tDMRG::step (same gate order, same U split)."""
    tau = dt if forward else -dt
    n = np.arange(p)
    ph_f = np.exp(-1j * 0.25 * u_from * tau * n * (n - 1))
    ph_t = np.exp(-1j * 0.25 * u_to * tau * n * (n - 1))
    G = hop_gate(p, J, tau).reshape(p, p, p, p)
    T = psi.reshape((p,) * L)
    for k in range(L):
        shape = [1] * L; shape[k] = p
        T = T * ph_f.reshape(shape)
    for (i1, i2) in gate_list(L):
        T = np.tensordot(G, T, axes=([2, 3], [i1 - 1, i2 - 1]))
        T = np.moveaxis(T, [0, 1], [i1 - 1, i2 - 1])
    for k in range(L):
        shape = [1] * L; shape[k] = p
        T = T * ph_t.reshape(shape)
    out = T.reshape(-1)
    return out / np.linalg.norm(out)


def dH_full(L: int, p: int) -> np.ndarray:
    """diagonal of sum_k 0.5 n_k (n_k - 1) on the full p**L space."""
    g = np.indices((p,) * L).reshape(L, -1)
    return (0.5 * g * (g - 1)).sum(axis=0)
