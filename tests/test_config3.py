"""BASELINE configs[2] (config 3): config 1's shape (L=5 Npart=5 d=4 chi=80,
tstep 0.01, T=2, N_t=201) with the full analytic Hessian's rows sharded
zig-zag over G = 1, 2, 4, 8 shards through the facade's setThreadCount (one
context and stream per shard; shards beyond the visible GPUs share a device),
GRAPE and GROUP M=10.  Row entries of different shards are disjoint, so every
G must give the bit-identical Hessian; G = 1 is compared with the oracle facade
(OptimalControl<OracleTDMRG>) at the north_star tolerances.  The bench's
multi-process path (one rank per GPU, RCCL reduce) shares the dealing
(optimalcontrolmps_amd/sharding.py) and is covered by test_sharding_gloo.py."""
import numpy as np
import pytest

import facade_build as fb


@pytest.fixture(scope="module")
def statedir(tmp_path_factory):
    d = tmp_path_factory.mktemp("states_c3")
    fb.write_states(str(d))
    return str(d)


@pytest.mark.gpu
def test_config3_sharded_hessian(statedir):
    r = fb.run("gpu", "config3", statedir, extra=("1,2,4,8",))
    o = fb.run("oracle", "config3", statedir, extra=("8",))  # 8 row-worker threads (calcHessian_parallel)
    for alg in ("grape", "group"):
        H1 = np.asarray(r[f"{alg}_G1"])
        for G in (2, 4, 8):
            assert np.array_equal(np.asarray(r[f"{alg}_G{G}"]), H1), (alg, G)
        Ho = np.asarray(o[f"{alg}_G8"])
        assert np.abs(H1 - Ho).max() <= 1e-6 * np.abs(Ho).max(), alg
        g, go = np.asarray(r[f"{alg}_grad"]), np.asarray(o[f"{alg}_grad"])
        assert np.abs(g - go).max() <= 1e-6, alg
