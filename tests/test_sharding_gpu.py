"""The multi-rank Hessian path on the HIP engine: 2 ranks (spawned processes,
gloo collectives, both ranks on cuda:0 as bench.py's OCG_BENCH_BACKEND=gloo dry
run places them) each evaluate their zig-zag row shard with ocg_hessian and
one reduce assembles the matrix on rank 0 (optimalcontrolmps_amd.distributed.
sharded_hessian, the function bench.py --mode strong drives over RCCL).  The
assembled Hessian must equal the single-process getHessian bit for bit (rows
write disjoint entries), with the regularisation and the GROUP
projection (ocg_convert_hessian on rank 0's device) included."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

L, p, Q, J, DT, CUT, MAXM = 5, 5, 5, 1.0, 0.01, 1e-8, 80


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _states(states):
    from conftest import state_key
    k0, k1 = state_key(L, p, Q, J, 2.5), state_key(L, p, Q, J, 50.0)
    return (states[k0 + "/dims"], states[k0 + "/data"], states[k1 + "/dims"], states[k1 + "/data"])


def _engine(st):
    from optimalcontrolmps_amd.native import MPS, Engine
    eng = Engine(L, p, Q, J, DT, CUT, MAXM, device=0)
    eng.set_states(MPS(L, p, Q, st[2], st[3]), MPS(L, p, Q, st[0], st[1]))
    return eng


def _worker(rank, world, port, st, u, V, gamma, out):
    import torch.distributed as dist
    from optimalcontrolmps_amd.distributed import sharded_hessian, torch_reduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = _engine(st)
    H, divT, F, rows = sharded_hessian(lambda uu, rr: eng.hessian(uu, rr), u, rank, world,
                                       torch_reduce(dist, "cpu", len(u)), gamma=gamma, tstep=DT,
                                       project=lambda Hu: eng.convert_hessian(Hu, V))
    if rank == 0:
        np.save(out, H)
    else:
        assert H is None
    dist.barrier()
    dist.destroy_process_group()
    eng.close()


def test_two_rank_hip_hessian_equals_single(states, tmp_path):
    import torch.multiprocessing as mp
    from optimalcontrolmps_amd.control_basis import adiabatic_seed, build_chopped_sine_basis, regularization_hessian
    st = _states(states)
    Nt, M, gamma = 41, 8, 1e-6
    basis = build_chopped_sine_basis(adiabatic_seed(2.0, 10.0, Nt), DT, (Nt - 1) * DT, M)
    u = basis.convert_control(np.random.default_rng(41).uniform(-2.0, 2.0, M))
    out = str(tmp_path / "H.npy")
    mp.start_processes(_worker, args=(2, _free_port(), st, u, basis.V, gamma, out), nprocs=2, join=True,
                       start_method="spawn")
    H2 = np.load(out)
    eng = _engine(st)
    Hu, _, _ = eng.hessian(u)
    H1 = eng.convert_hessian(Hu + regularization_hessian(Nt, gamma, DT), basis.V)
    eng.close()
    assert H2.shape == (M, M)
    assert np.array_equal(H1, H2)
