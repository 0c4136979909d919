"""TEST INFRASTRUCTURE: builds tests/cpp/facade_driver.cpp (the restated
reference C++ tests) against the CPU oracle or the HIP product library, and
writes the golden ED states it reads (tests/golden/states.npz -> <key>.bin)."""
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "cpp", "facade_driver.cpp")
BUILD = os.path.join(HERE, "cpp", "build")
PKG = os.path.join(ROOT, "optimalcontrolmps_amd")


def _deps():
    inc = os.path.join(PKG, "include", "optimalcontrolmps")
    files = [SRC, os.path.join(HERE, "cpp", "oracle_stepper.hpp"), os.path.join(ROOT, "oracle", "tdmrg_oracle.hpp"),
             os.path.join(ROOT, "include", "ocmps.h")]
    files += [os.path.join(inc, f) for f in os.listdir(inc)]
    return max(os.path.getmtime(f) for f in files)


def build_driver(kind):
    """kind: 'oracle' (CPU restatement) or 'gpu' (liboptimalcontrolmps_amd.so)."""
    os.makedirs(BUILD, exist_ok=True)
    out = os.path.join(BUILD, f"facade_{kind}")
    if os.path.exists(out) and os.path.getmtime(out) >= _deps():
        return out
    cmd = ["g++", "-O2", "-std=c++17", "-pthread", "-o", out + ".tmp", SRC]
    if kind == "oracle":
        cmd.insert(1, "-DOCMPS_ORACLE")
    else:
        cmd += [f"-L{PKG}", "-loptimalcontrolmps_amd", f"-Wl,-rpath,{PKG}"]
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


def write_states(directory):
    z = np.load(os.path.join(HERE, "golden", "states.npz"), allow_pickle=False)
    keys = sorted({k.rsplit("/", 1)[0] for k in z.files})
    for k in keys:
        dims = np.ascontiguousarray(z[k + "/dims"], dtype=np.int32)
        data = np.ascontiguousarray(z[k + "/data"], dtype=np.complex128)
        L, p, N = (int(s[1:]) for s in k.split("_")[:3])
        hdr = np.array([L, p, N, dims.size, data.size], dtype=np.int32)
        with open(os.path.join(directory, k + ".bin"), "wb") as f:
            f.write(hdr.tobytes() + dims.tobytes() + data.tobytes())


def run(kind, scenario, directory, timeout=1200, extra=()):
    exe = build_driver(kind)
    r = subprocess.run([exe, scenario, directory, *extra], capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        raise RuntimeError(f"{kind} driver '{scenario}' failed: {r.stderr.strip()}")
    return json.loads(r.stdout)
