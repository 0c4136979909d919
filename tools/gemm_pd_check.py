"""A/B helper (diagnostic): the config-4 Maxm-32 getHessian (tests/golden/c4.npz s32)
with the k_gemm prefetch depth of this process's OCG_HBM_GEMM_PD, written to
gpurun_out/gemm_pd<PD>.npy so two runs can be compared bit for bit."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from optimalcontrolmps_amd.native import MPS, Engine  # noqa: E402

L, p, N, J, DT, CUT = 20, 7, 20, 1.0, 0.005, 1e-8
c = dict(np.load(os.path.join(ROOT, "tests", "golden", "c4.npz"), allow_pickle=False))
eng = Engine(L, p, N, J, DT, CUT, int(c["s32/maxm"]), engine="hbm")
eng.set_states(MPS(L, p, N, c["s32/tgt_dims"], c["s32/tgt_data"]), MPS(L, p, N, c["s32/init_dims"], c["s32/init_data"]))
H, divT, F = eng.hessian(c["s32/u"])
w = dict(np.load(os.path.join(ROOT, "tests", "golden", "c4_warm256.npz"), allow_pickle=False))
e2 = Engine(L, p, N, J, DT, CUT, 256, engine="hbm")
psi = e2.steps(MPS(L, p, N, w["dims"], w["data"]), np.array([2.5, 3.0, 3.5]), True)
pd = os.environ.get("OCG_HBM_GEMM_PD", "1")
np.save(os.path.join(ROOT, "gpurun_out", f"gemm_pd{pd}.npy"), np.concatenate([H.ravel(), divT.view(np.float64), psi.data.view(np.float64)]))
print("pd", pd, "max|H|", np.abs(H).max())
