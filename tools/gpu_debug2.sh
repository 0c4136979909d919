cd $GRAFT_REPO_ROOT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DOCG_DEVICE_DEBUG -o /tmp/libdbg.so optimalcontrolmps_amd/csrc/ocmps.hip || exit 3
cp optimalcontrolmps_amd/liboptimalcontrolmps_amd.so /tmp/keep.so
cp /tmp/libdbg.so optimalcontrolmps_amd/liboptimalcontrolmps_amd.so
timeout -k 10 120 python - > gpurun_out/debug2.log 2>&1 <<'PY'
import sys; sys.path.insert(0,'.')
import numpy as np
from optimalcontrolmps_amd.native import Engine, MPS
S = dict(np.load('tests/golden/states.npz'))
for (L,p,N,J,U) in [(4,3,4,1.0,2.0),(3,4,3,2.0,2.0)]:
    k=f"L{L}_p{p}_N{N}_J{J:g}_U{U:g}"
    m=MPS(L,p,N,S[k+"/dims"],S[k+"/data"])
    e=Engine(L,p,N,J,0.01,1e-8,0)
    print(k, "host dims", m.dims.tolist(), flush=True)
    print("  <m|m> =", e.overlap(m,m), flush=True)
PY
echo "exit $?"
