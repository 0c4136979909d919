"""CPU-side checking: the oracle built with AddressSanitizer +
UndefinedBehaviorSanitizer and with ThreadSanitizer, and the CPU emulation of
the device bodies (tests/emu) with ASan + UBSan, each running a small
getHessian / step sequence in a child interpreter with the sanitizer runtime
preloaded.  A report fails the test.  Test infrastructure only."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _runtime(name):
    out = subprocess.run(["g++", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    if not out or not os.path.isabs(out) or not os.path.exists(out):
        pytest.skip(f"{name} not available")
    return out


ORACLE_CASE = r"""
import sys, numpy as np
sys.path.insert(0, {tests!r}); sys.path.insert(0, {root!r})
import oracle_ffi as O
from optimalcontrolmps_amd import ed
L, p, Q, J = 5, 5, 5, 1.0
mk = lambda U: O.MPS(L, p, Q, *ed.mps_from_full(ed.ground_state_full(L, p, Q, J, U)[0], L, p, Q))
st = O.Stepper(L, p, Q, J, 0.01, 1e-8, 80)
u = np.random.default_rng(3).uniform(2, 10, 5)
oc = O.OC(st, mk(50.0), mk(2.5), len(u), 1e-6)
H1 = oc.hessian(u, 1)
oc.set_nested(True)
H4 = oc.hessian(u, 4)          # psi || xi, the row pool and the sector threads
assert np.array_equal(H1, H4)
g = oc.gradient(u, True)
print("OK")
"""

EMU_CASE = r"""
import sys, numpy as np
sys.path.insert(0, {tests!r}); sys.path.insert(0, {emu!r}); sys.path.insert(0, {root!r})
import emu_ffi as E
from optimalcontrolmps_amd import ed
L, p, Q, J = 5, 5, 5, 1.0
d, x = ed.mps_from_full(ed.ground_state_full(L, p, Q, J, 2.5)[0], L, p, Q)
u = np.random.default_rng(1).uniform(2, 10, 2)
for fast in (True, False):
    E.Emu(L, p, Q, J, 0.01, 1e-8, 80, fast).steps(d, x, u)
print("OK")
"""


def _child(code, env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    cp = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=900)
    bad = [m for m in ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "ERROR: LeakSanitizer")
           if m in cp.stderr]
    assert cp.returncode == 0 and "OK" in cp.stdout and not bad, (cp.returncode, bad, cp.stderr[-3000:])


def test_oracle_asan_ubsan():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "build/libocmps_oracle_asan.so"])
    _child(ORACLE_CASE.format(tests=HERE, root=ROOT),
           {"LD_PRELOAD": _runtime("libasan.so") + ":" + _runtime("libubsan.so"),
            "ASAN_OPTIONS": "detect_leaks=0", "ORC_LIB": os.path.join(ROOT, "oracle", "build", "libocmps_oracle_asan.so")})


def test_oracle_tsan_row_pool():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "build/libocmps_oracle_tsan.so"])
    _child(ORACLE_CASE.format(tests=HERE, root=ROOT),
           {"LD_PRELOAD": _runtime("libtsan.so"), "TSAN_OPTIONS": "report_signal_unsafe=0",
            "ORC_LIB": os.path.join(ROOT, "oracle", "build", "libocmps_oracle_tsan.so")})


def test_emulated_device_bodies_asan_ubsan():
    emu = os.path.join(HERE, "emu")
    subprocess.check_call(["make", "-s", "-C", emu, "build/libocmps_emu_asan.so"], stdout=subprocess.DEVNULL,
                          stderr=subprocess.DEVNULL)
    _child(EMU_CASE.format(tests=HERE, emu=emu, root=ROOT),
           {"LD_PRELOAD": _runtime("libasan.so") + ":" + _runtime("libubsan.so"),
            "ASAN_OPTIONS": "detect_leaks=0", "EMU_LIB": os.path.join(emu, "build", "libocmps_emu_asan.so")})
