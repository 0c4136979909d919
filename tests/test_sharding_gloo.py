"""Multi-rank Hessian path on CPU: world_size-2 gloo, each rank computes its
zig-zag row shard (optimalcontrolmps_amd.sharding, the dealing bench.py and
the C++ facade use) with the CPU oracle, one all-reduce(SUM) assembles the
matrix, which must equal the single-process Hessian bit for bit (rows write
disjoint entries)."""
import os
import socket

import numpy as np
import pytest

from optimalcontrolmps_amd.sharding import shard_cost, zigzag_rows


def test_zigzag_partition_and_balance():
    for n_t in (11, 16, 201):
        for world in (1, 2, 3, 4, 8):
            parts = [zigzag_rows(n_t - 2, r, world) for r in range(world)]
            flat = sorted(i for p in parts for i in p)
            assert flat == list(range(1, n_t - 1))
            if n_t == 201 and world > 1:
                cost = [shard_cost(p, n_t) for p in parts]
                assert max(cost) / (sum(cost) / world) < 1.02   # serpentine keeps shards within 2%
    with pytest.raises(ValueError):
        zigzag_rows(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, u, states, out):
    import torch
    import torch.distributed as dist
    import oracle_ffi as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    L, p, Q, J = 3, 4, 3, 2.0
    st = O.Stepper(L, p, Q, J, 0.01, 1e-7)
    tgt = O.MPS(L, p, Q, states["tgt_dims"], states["tgt_data"])
    ini = O.MPS(L, p, Q, states["ini_dims"], states["ini_data"])
    oc = O.OC(st, tgt, ini, len(u), 0.0)
    H = torch.from_numpy(oc.rows(u, zigzag_rows(len(u) - 2, rank, world)))
    dist.all_reduce(H, op=dist.ReduceOp.SUM)
    if rank == 0:
        np.save(out, H.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_hessian_equals_single(states, tmp_path):
    import torch.multiprocessing as mp
    import oracle_ffi as O
    from conftest import state_key
    k0, k1 = state_key(3, 4, 3, 2.0, 2.0), state_key(3, 4, 3, 2.0, 12.0)
    st = dict(ini_dims=states[k0 + "/dims"], ini_data=states[k0 + "/data"],
              tgt_dims=states[k1 + "/dims"], tgt_data=states[k1 + "/data"])
    u = np.random.default_rng(3).uniform(2, 10, 14)
    out = str(tmp_path / "H.npy")
    mp.start_processes(_worker, args=(2, _free_port(), u, st, out), nprocs=2, join=True, start_method="spawn")
    H2 = np.load(out)
    L, p, Q, J = 3, 4, 3, 2.0
    oc = O.OC(O.Stepper(L, p, Q, J, 0.01, 1e-7), O.MPS(L, p, Q, st["tgt_dims"], st["tgt_data"]),
              O.MPS(L, p, Q, st["ini_dims"], st["ini_data"]), len(u), 0.0)
    H1 = oc.hessian(u, 1)
    assert np.array_equal(H1, H2)
