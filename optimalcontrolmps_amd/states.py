"""Input states of the config-4 chains (host side, interchange format of
include/ocmps.h).

product_state: the reference's initial particle distribution
    (include/InitializeState.hpp:26-40: "Occ1" on the Npart right-most sites,
    "Emp" elsewhere) as an MPS with all bond dimensions 1.  For Npart = L it is
    the Mott state |1...1>, config 4's psi_target.
warm_state: config 4's psi_init — the product state evolved in real time at a
    constant U until the bonds saturate at Maxm (the reference
    prepares its states with ITensor DMRG, InitializeState.hpp:42-60).  Runs on
    the given engine (the GPU stepper), not timed.
ground_state: InitializeState's ground state prepared on the device by
    imaginary-time evolution of the product state (ocg_imag_steps).
"""
from __future__ import annotations

import numpy as np

from .native import MPS


def product_state(L: int, p: int, npart: int) -> MPS:
    """|0..0 1..1> with npart bosons on the right-most sites (InitializeState.hpp:26-40)."""
    if npart > L:
        raise ValueError("Npart > N not supported (include/InitializeState.hpp:29)")
    Q1 = npart + 1
    occ = [0] * (L - npart) + [1] * npart     # site k (1-based) holds occ[k-1]
    dims = np.zeros((L + 1) * Q1, np.int32)
    q = 0
    dims[0 * Q1 + 0] = 1
    for b in range(1, L + 1):
        q += occ[b - 1]
        dims[b * Q1 + q] = 1
    return MPS(L, p, npart, dims, np.ones(L, np.complex128))


def warm_state(engine, psi: MPS, U: float, nsteps: int, chunk: int = 50) -> MPS:
    """nsteps forward steps at constant control U (BH_tDMRG::step, src/BH_tDMRG.cpp:111-125)."""
    done = 0
    while done < nsteps:
        k = min(chunk, nsteps - done)
        psi = engine.steps(psi, np.full(k + 1, float(U)), True)
        done += k
    return psi


# tau schedule of ground_state: each stage runs to its Trotter fixed point;
# the fixed point's infidelity with the exact ground state falls as tau^2
# (L=5 p=5 N=5: 5.5e-7 at 2e-3, 5.9e-8 at 5e-4 for U=2.5)
GS_TAUS = (0.05, 0.01, 0.002, 0.001, 0.0005)


def ground_state(engine, U: float, taus=GS_TAUS, block: int = 25, tol: float = 1e-13,
                 max_steps: int = 8000, psi: MPS = None) -> MPS:
    """InitializeState(sites, Npart, J, U) (include/InitializeState.hpp:18-117) on
    the device: imaginary-time evolution exp(-tau H) of the product state
    |0..0 1..1> (the reference's DMRG starting guess), per tau in blocks of
    `block` steps until 1 - |<prev|new>| < tol, the whole schedule in one
    ocg_ground_state call (the state stays on the device)."""
    if psi is None:
        psi = product_state(engine.L, engine.p, engine.Q)
    return engine.ground_state(psi, U, taus, block, tol, max_steps)[0]
