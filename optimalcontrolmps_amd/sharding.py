"""Row sharding of getHessian over ranks.

calcHessianRow i (reference src/OptimalControl.cpp:251-279) costs N_t-2-i
Trotter steps, so rows are dealt out serpentine-wise ("zig-zag"): block b of
`world` consecutive rows goes to ranks 0..world-1, reversed on odd blocks.
Rows write disjoint (i, j>=i) entries and their mirrors, so the partial
N_t x N_t matrices of all ranks sum exactly to the full Hessian (one
RCCL/gloo reduce, no other exchange).  The C++ facade uses the same dealing
(include/optimalcontrolmps/GpuTDMRG.hpp, Engine::hessianRows).
"""


def zigzag_rows(nrows_total, rank, world):
    """rows 1..nrows_total (= N_t-2) owned by `rank` of `world`"""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank {rank} / world {world}")
    rows = list(range(1, nrows_total + 1))
    out = []
    for blk in range(0, len(rows), world):
        chunk = rows[blk:blk + world]
        if (blk // world) % 2 == 1:
            chunk = chunk[::-1]
        if rank < len(chunk):
            out.append(chunk[rank])
    return out


def shard_cost(rows, n_t):
    """Trotter steps of a row set (row i re-propagates N_t-2-i steps)"""
    return sum(n_t - 2 - i for i in rows)
