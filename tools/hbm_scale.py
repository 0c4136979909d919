"""Scale probe of the HBM engine at the config-4 chain (L=20, Npart=20, p=7,
dt=0.005): evolve the Mott state |1..1> at U=2.5 with maxm = chi for `nsteps`
steps (in chunks), printing bond dims and time per step.
usage: python tools/hbm_scale.py chi nsteps [chunk]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from optimalcontrolmps_amd.native import MPS, Engine  # noqa: E402


def mott(L, p, N):
    Q1 = N + 1
    dims = np.zeros((L + 1) * Q1, np.int32)
    for b in range(L + 1):
        dims[b * Q1 + b] = 1
    return MPS(L, p, N, dims, np.ones(L, np.complex128))


chi = int(sys.argv[1]) if len(sys.argv) > 1 else 32
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
chunk = int(sys.argv[3]) if len(sys.argv) > 3 else 10
L, p, N = 20, 7, 20
eng = Engine(L, p, N, 1.0, 0.005, 1e-8, chi, engine="hbm")
m = mott(L, p, N)
done = 0
while done < nsteps:
    k = min(chunk, nsteps - done)
    t = time.time()
    m = eng.steps(m, np.full(k + 1, 2.5), True)
    el = time.time() - t
    done += k
    bd = m.bond_dims()
    print(f"chi={chi} steps={done} {1e3 * el / k:.1f} ms/step max bond {bd.max()} bonds {list(map(int, bd))}",
          flush=True)
g = eng.stats(7)
print(f"gemm: {g['ms']:.1f} ms in {g['launches']} launches, {g['alg_flops'] / max(g['ms'], 1e-9) / 1e9:.2f} TF/s, "
      f"{g['alg_bytes'] / max(g['ms'], 1e-9) / 1e6:.1f} GB/s", flush=True)
out = os.path.join(ROOT, "gpurun_out", f"mott_chi{chi}_n{done}.npz")
np.savez(out, dims=m.dims, data=m.data)
