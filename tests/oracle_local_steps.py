"""One-step oracle checks of states the GPU engine produced (TEST
INFRASTRUCTURE, run as a CPU-only child process by
tests/test_config4.py::test_c4_full_horizon_local_steps_vs_oracle).

A child process because the oracle picks its block eigensolver once, at its
first decomposition (ORC_HEEV, oracle/tdmrg_oracle.hpp heev_use_ql): the GPU
suite's earlier oracle checks have already fixed the cyclic Jacobi solver in
the test process, and a chi = 256 step needs the Householder + QL one
(tests/golden/make_c4_fixtures.py make_w256hN).  The child never touches the
GPU.

  python tests/oracle_local_steps.py IN.npz OUT.npz

IN.npz: L, p, Q, J, dt, cutoff, maxm; nstep and for j < nstep: s<j>_dims /
s<j>_data (a state), n<j>_dims / n<j>_data (the GPU's next state from it),
u<j> = [u_from, u_to, forward]; ndh and for j < ndh: x<j>_*, y<j>_* (a pair
for <x|dH|y>); ovx_* / ovy_* (a pair for <x|y>).
OUT.npz: bonds<j> (the oracle's next-state bond dims), ov<j> = <oracle|gpu>,
nn<j> = <oracle|oracle>, gg<j> = <gpu|gpu>; dh<j> = <x|dH|y>; ov = <x|y>.
"""
import os
import sys

import numpy as np

os.environ["ORC_HEEV"] = "ql"   # before the oracle's first decomposition
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import oracle_ffi as O  # noqa: E402


def main(src, dst):
    z = np.load(src, allow_pickle=False)
    L, p, Q = int(z["L"]), int(z["p"]), int(z["Q"])
    O.set_sector_threads(int(os.environ.get("ORC_SECTOR_THREADS", "16")))
    st = O.Stepper(L, p, Q, float(z["J"]), float(z["dt"]), float(z["cutoff"]), int(z["maxm"]))
    mps = lambda key: O.MPS(L, p, Q, z[key + "_dims"], z[key + "_data"])
    out = {}
    for j in range(int(z["nstep"])):
        u0, u1, fwd = z[f"u{j}"]
        nxt = st.step(mps(f"s{j}"), float(u0), float(u1), bool(fwd))
        gpu = mps(f"n{j}")
        out[f"bonds{j}"] = np.asarray(nxt.bond_dims())
        out[f"ov{j}"] = np.array([st.overlap(nxt, gpu)])
        out[f"nn{j}"] = np.array([st.overlap(nxt, nxt)])
        out[f"gg{j}"] = np.array([st.overlap(gpu, gpu)])
        print(f"step {j}: bonds {[int(b) for b in nxt.bond_dims()]}", flush=True)
    for j in range(int(z["ndh"])):
        out[f"dh{j}"] = np.array([st.overlap_dH(mps(f"x{j}"), mps(f"y{j}"))])
    if "ovx_dims" in z:
        out["ov"] = np.array([st.overlap(mps("ovx"), mps("ovy"))])
    np.savez(dst, **out)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
