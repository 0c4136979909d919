"""One getHessian sharded over ranks (the reference's row pool
src/OptimalControl.cpp:306-335 spread over processes, one per GPU).

Every rank recomputes psi_t, xi_t, divT, xiHlist for the control (O(N_t)
steps) and evaluates only its zig-zag share of the rows (O(N_t^2) steps in
total); rows write disjoint entries (i, j >= i) and their mirrors, so one
reduce(SUM) of the N_t x N_t partial matrices onto rank 0 is the whole
exchange.  Rank 0 then adds the regularisation Hessian and, in GROUP mode,
projects H_c = V H_u V^T on its device (ControlBasis::convertHessian,
src/ControlBasis.cpp:92-119).

The rank-local Hessian evaluation and the collective are passed in, so the
same code drives the GPU bench (HIP engine + RCCL) and the CPU tests (CPU
oracle + gloo).
"""
from __future__ import annotations

import numpy as np

from .control_basis import regularization_hessian
from .sharding import zigzag_rows


def torch_reduce(dist, device, n):
    """reduce(SUM) of an n x n float64 numpy matrix onto rank 0 over
    torch.distributed (backend nccl = RCCL over xGMI on MI355X, or gloo);
    returns the sum on rank 0, None elsewhere."""
    import torch
    buf = torch.zeros((n, n), dtype=torch.float64, device=device)

    def reduce(H):
        buf.copy_(torch.from_numpy(np.ascontiguousarray(H)))
        dist.reduce(buf, dst=0)
        return buf.cpu().numpy() if dist.get_rank() == 0 else None
    return reduce


def sharded_hessian(hessian_rows, u, rank, world, reduce_to_root, gamma=0.0, tstep=None, project=None):
    """getHessian(u) (src/OptimalControl.cpp:523-562) with its rows dealt over
    `world` ranks.

    hessian_rows(u, rows) -> (H_partial, divT, F): this rank's fidelity-Hessian
        entries of `rows` (zeros elsewhere), e.g. Engine.hessian (ocg_hessian);
    reduce_to_root(H) -> sum over ranks on rank 0 (None elsewhere);
    gamma, tstep: the regularisation Hessian added on rank 0 (:124-143);
    project(H_u) -> H_c: GROUP projection on rank 0 (Engine.convert_hessian
        with the basis matrix), None for GRAPE.
    Returns (H, divT, F, rows): H on rank 0 (None on the others); divT and F
    (for the gradient) are every rank's own."""
    n = len(u)
    rows = zigzag_rows(n - 2, rank, world)
    H, divT, F = hessian_rows(u, rows)
    if world > 1:
        H = reduce_to_root(H)
    if H is not None:
        if gamma:
            H = H + regularization_hessian(n, gamma, tstep)
        if project is not None:
            H = project(H)
    return H, divT, F, rows
