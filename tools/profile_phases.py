"""Diagnostic: per-phase cycle breakdown of the chain engine (OCG_PROFILE build)."""
import os, sys, subprocess, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NT = int(os.environ.get("OCG_PROF_NT", "64"))
lib = os.path.join(ROOT, "tools", "build", f"libocg_prof{NT}.so")
if not os.path.exists(lib) or "--rebuild" in sys.argv:  # build on the CPU side before a GPU call
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-DOCG_PROFILE", f"-DOCG_NT={NT}", "-o", lib,
                           os.path.join(ROOT, "optimalcontrolmps_amd/csrc/ocmps.hip"),
                           os.path.join(ROOT, "optimalcontrolmps_amd/csrc/hbm.hip")])
if "--build-only" in sys.argv:
    sys.exit(0)
print(f"NT = {NT}")
os.environ["OCG_LIB"] = lib
import numpy as np
from optimalcontrolmps_amd import ed
from optimalcontrolmps_amd.native import MPS, Engine
NAMES = {0: "build_theta", 1: "apply_gate", 2: "gram", 3: "jacobi", 4: "rank", 18: "trunc/kept", 19: "ts offsets",
         5: "factor X", 23: "factor Y", 7: "s2theta tabs", 28: "s2theta copy", 24: "gauge BOFFT", 25: "gauge S",
         26: "gauge dims", 27: "gauge wb", 8: "overlap", 9: "phase/norm", 10: "load/store", 11: "dH zip", 12: "other",
         13: "jacobi A", 14: "jacobi B", 15: "theta tabs", 16: "decomp setup", 29: "step phases"}
L, p, Q, J, dt = 5, 5, 5, 1.0, 0.01
ini = MPS(L, p, Q, *ed.mps_from_full(ed.ground_state_full(L, p, Q, J, 2.5)[0], L, p, Q))
tgt = MPS(L, p, Q, *ed.mps_from_full(ed.ground_state_full(L, p, Q, J, 50.0)[0], L, p, Q))
eng = Engine(L, p, Q, J, dt, 1e-8, 80)
u = np.random.default_rng(20261015).uniform(2, 10, 201)
eng.set_states(tgt, ini)
for what in ["trajectory(2 chains x 200 steps)", "div_t+xi_dH", "hessian_rows(199)"]:
    eng.profile(True)
    t0 = time.perf_counter()
    if what.startswith("traj"):
        eng.propagate(u, 3)
    elif what.startswith("div"):
        d = eng.div_t(); F = eng.overlap_factor(); eng.xi_dH()
    else:
        H = eng.hessian_rows(u, list(range(1, 200)), F, d)
    t1 = time.perf_counter()
    pr = eng.profile(True)
    tot = sum(pr[i] for i in NAMES)
    print(f"== {what}: wall {1e3*(t1-t0):.1f} ms, total cycles {tot:.3e}")
    for i, n in sorted(NAMES.items()):
        if pr[i] > 0:
            print(f"   {n:12s} {pr[i]:.3e} ({100*pr[i]/tot:5.1f}%)")
    print(f"   (inside gauge moves: {pr[31]:.3e} = {100*pr[31]/max(tot,1):.1f}% of the cycles)")
    if pr[22] > 0:   # the one-wave padded chain's counters
        nst = 400 if what.startswith("traj") else 1
        print(f"   fast chain: decompositions {pr[22]:.0f} ({pr[22]/nst:.2f} per chain-step), jacobi calls "
              f"{pr[21]:.0f}, sweeps/call {pr[20]/max(pr[21],1):.2f}, rounds/call {pr[30]/max(pr[21],1):.2f}, "
              f"small eigenvalues per decomposition {pr[17]/pr[22]:.1f}")
    elif pr[21] > 0:
        print(f"   jacobi calls {pr[21]:.0f}, sweeps/call {pr[20]/pr[21]:.2f}, rounds/sweep {pr[22]/pr[21]:.2f}, "
              f"rounds executed/call (wave 0 of the first block group) {pr[30]/pr[21]:.2f}")
print("traj kernel ms:", eng.stats(0)["ms"], " rows ms:", eng.stats(3)["ms"])
