import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
import numpy as np
from optimalcontrolmps_amd.native import Engine, MPS
S = dict(np.load('tests/golden/states.npz'))
for (L,p,N,J,U) in [(4,3,4,1.0,2.0),(3,4,3,2.0,2.0),(5,5,5,1.0,2.5),(5,6,5,1.0,2.0)]:
    k=f"L{L}_p{p}_N{N}_J{J:g}_U{U:g}"
    m=MPS(L,p,N,S[k+"/dims"],S[k+"/data"])
    e=Engine(L,p,N,J,0.01,1e-8,0)
    print(k, "lds", e.info.lds_bytes, "cap", e.cap, flush=True)
    r=e.steps(m,[1.0],True)
    print("  roundtrip dims ok", np.array_equal(r.dims,m.dims), "data err", np.abs(r.data-m.data).max(), flush=True)
    print("  <m|m> =", e.overlap(m,m), " <m|dH|m> =", e.overlap(m,m,True), flush=True)
    s=e.step(m,3.0,4.0)
    print("  step dims", s.bond_dims(), "norm via overlap", e.overlap(s,s), flush=True)
