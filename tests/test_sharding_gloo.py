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


def _oracle_rows(L, p, Q, J, states):
    import oracle_ffi as O
    st = O.Stepper(L, p, Q, J, 0.01, 1e-7)
    tgt = O.MPS(L, p, Q, states["tgt_dims"], states["tgt_data"])
    ini = O.MPS(L, p, Q, states["ini_dims"], states["ini_data"])

    def rows_fn(u, rows):   # this rank's fidelity-Hessian entries (ocg_hessian's contract)
        oc = O.OC(st, tgt, ini, len(u), 0.0)
        H = oc.rows(u, rows)
        divT, F = oc.divT_F()
        return H, divT, F
    return rows_fn


def _worker(rank, world, port, u, states, out, gamma, V):
    import torch.distributed as dist
    from optimalcontrolmps_amd.distributed import sharded_hessian, torch_reduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows_fn = _oracle_rows(3, 4, 3, 2.0, states)
    # the strong-scaling path of bench.py (--mode strong): zig-zag rows, reduce onto rank 0,
    # regularisation + GROUP projection there
    H, divT, F, rows = sharded_hessian(rows_fn, u, rank, world, torch_reduce(dist, "cpu", len(u)),
                                       gamma=gamma, tstep=0.01, project=None)
    Hc, _, _, _ = sharded_hessian(rows_fn, u, rank, world, torch_reduce(dist, "cpu", len(u)),
                                  gamma=gamma, tstep=0.01, project=lambda Hu: V @ Hu @ V.T)
    if rank == 0:
        np.save(out, H)
        np.save(out + ".group.npy", Hc)
    else:
        assert H is None and Hc is None
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_hessian_equals_single(states, tmp_path):
    """2 gloo ranks through optimalcontrolmps_amd.distributed.sharded_hessian
    (rows zig-zag, reduce onto rank 0, regularisation, GROUP projection) equal
    the single-process getHessian bit for bit"""
    import torch.multiprocessing as mp
    import oracle_ffi as O
    from conftest import state_key
    from optimalcontrolmps_amd.control_basis import (adiabatic_seed, build_chopped_sine_basis,
                                                     regularization_hessian)
    k0, k1 = state_key(3, 4, 3, 2.0, 2.0), state_key(3, 4, 3, 2.0, 12.0)
    st = dict(ini_dims=states[k0 + "/dims"], ini_data=states[k0 + "/data"],
              tgt_dims=states[k1 + "/dims"], tgt_data=states[k1 + "/data"])
    Nt, gamma = 14, 1e-3
    basis = build_chopped_sine_basis(adiabatic_seed(2.0, 10.0, Nt), 0.01, 0.13, 5)
    u = basis.convert_control(np.random.default_rng(3).uniform(-2, 2, 5))
    out = str(tmp_path / "H.npy")
    mp.start_processes(_worker, args=(2, _free_port(), u, st, out, gamma, basis.V), nprocs=2, join=True,
                       start_method="spawn")
    H2, Hc2 = np.load(out), np.load(out + ".group.npy")
    L, p, Q, J = 3, 4, 3, 2.0
    oc = O.OC(O.Stepper(L, p, Q, J, 0.01, 1e-7), O.MPS(L, p, Q, st["tgt_dims"], st["tgt_data"]),
              O.MPS(L, p, Q, st["ini_dims"], st["ini_data"]), len(u), gamma)
    H1 = oc.hessian(u, 1)   # the oracle starts from the regularisation Hessian and adds the rows
    assert np.array_equal(H1, H2)
    assert np.array_equal(basis.V @ H1 @ basis.V.T, Hc2)
    assert np.abs(regularization_hessian(Nt, gamma, 0.01) - (H1 - O.OC(
        O.Stepper(L, p, Q, J, 0.01, 1e-7), O.MPS(L, p, Q, st["tgt_dims"], st["tgt_data"]),
        O.MPS(L, p, Q, st["ini_dims"], st["ini_data"]), len(u), 0.0).hessian(u, 1))).max() < 1e-12


def test_control_basis_mirror_reference_goldens():
    """optimalcontrolmps_amd.control_basis (the bench's GROUP host code) against
    the reference's ControlBasisTests goldens (tests/ControlBasisTests.cpp:186-343,
    restated in tests/reference_goldens.py), the same inputs as the C++ facade's
    test (tests/cpp/facade_driver.cpp)"""
    import reference_goldens as RG
    from optimalcontrolmps_amd.control_basis import build_chopped_sine_basis, linspace
    b = build_chopped_sine_basis([1 + 0.1 * i for i in range(11)], 0.1, 1.0, 5)
    assert np.abs(b.convert_control(np.zeros(5)) - (1 + 0.1 * np.arange(11))).max() < 1e-6    # :186-192
    assert np.abs(b.convert_control(np.ones(5)) - RG.CS_U2).max() < 5e-6                       # :194-204
    assert np.abs(b.convert_control(np.zeros(5), False) - np.asarray(RG.CS_U2)).max() < 5e-6  # :206-211
    assert np.abs(b.convert_gradient(np.ones(11)) - RG.CS_GRADC2).max() < 5e-6                 # :226-237
    assert np.abs(b.control_jacobian() - np.asarray(RG.CS_JAC)).max() < 5e-6                   # :243-268
    assert np.abs(b.V @ np.ones((11, 11)) @ b.V.T - np.asarray(RG.CS_HESS_ONES)).max() < 1e-4  # :286-310
    assert len(linspace(0, 100, 801)) == 801
