"""Diagnose config-3 shard invariance: run the GPU facade driver's config3
scenario for a list of shard counts and report where the Hessians differ."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import facade_build as fb  # noqa: E402

d = "/tmp/c3states"
os.makedirs(d, exist_ok=True)
fb.write_states(d)
gl = sys.argv[1] if len(sys.argv) > 1 else "1,8,8,1"
r = fb.run("gpu", "config3", d, extra=(gl,))
gs = gl.split(",")
for alg in ("grape", "group"):
    H1 = np.asarray(r[f"{alg}_G{gs[0]}"])
    for G in gs[1:]:
        H = np.asarray(r[f"{alg}_G{G}"])
        diff = np.abs(H - H1)
        idx = np.argwhere(diff > 0)
        print(alg, G, "max", diff.max(), "rel", diff.max() / np.abs(H1).max(), "n", len(idx),
              "rows", sorted(set(int(i) for i in idx[:, 0]))[:40], flush=True)
