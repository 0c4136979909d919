"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Loads oracle/build/libocmps_oracle.so (built from oracle/ by `make`; the
build is also run by __graft_entry__.build()).  The product package never
imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "build", "libocmps_oracle.so")
# ORC_LIB: another build of the oracle (the sanitizer builds of tests/test_sanitizers.py)
_ALT = os.environ.get("ORC_LIB")

_lib = None

dp = C.POINTER(C.c_double)
ip = C.POINTER(C.c_int)


def lib():
    global _lib
    if _lib is None:
        src_mtime = max(os.path.getmtime(os.path.join(ORACLE_DIR, f))
                        for f in ("tdmrg_oracle.hpp", "oracle_capi.cpp", "Makefile"))
        if _ALT:
            L = C.CDLL(_ALT)
        else:
            if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < src_mtime:
                subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
            L = C.CDLL(LIB_PATH)
        L.orc_new.restype = C.c_void_p
        L.orc_new.argtypes = [C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, C.c_int]
        L.orc_free.argtypes = [C.c_void_p]
        L.orc_gate.argtypes = [C.c_void_p, C.c_int, dp]
        L.orc_step.argtypes = [C.c_void_p, ip, dp, C.c_double, C.c_double, C.c_int, ip, dp, C.c_size_t,
                               C.POINTER(C.c_size_t)]
        L.orc_steps.argtypes = [C.c_void_p, ip, dp, dp, C.c_int, C.c_int, ip, dp, C.c_size_t,
                                C.POINTER(C.c_size_t)]
        L.orc_overlap.argtypes = [C.c_void_p, ip, dp, ip, dp, dp]
        L.orc_overlap_dH.argtypes = [C.c_void_p, ip, dp, ip, dp, dp]
        L.orc_apply_dH.argtypes = [C.c_void_p, ip, dp, ip, dp, C.c_size_t, C.POINTER(C.c_size_t)]
        L.orc_heev.argtypes = [C.c_int, dp, dp, dp]
        L.orc_heev_ql.argtypes = [C.c_int, dp, dp, dp]
        L.orc_truncate.argtypes = [dp, C.c_int, C.c_double, C.c_int]
        L.orc_truncate.restype = C.c_int
        L.orc_oc_new.restype = C.c_void_p
        L.orc_oc_new.argtypes = [C.c_void_p, ip, dp, ip, dp, C.c_int, C.c_double]
        L.orc_oc_free.argtypes = [C.c_void_p]
        L.orc_oc_set_gamma.argtypes = [C.c_void_p, C.c_double]
        L.orc_oc_cost.restype = C.c_double
        L.orc_oc_cost.argtypes = [C.c_void_p, dp]
        L.orc_oc_fidelities.argtypes = [C.c_void_p, dp, dp]
        L.orc_oc_gradient.argtypes = [C.c_void_p, dp, C.c_int, dp]
        L.orc_oc_divT.argtypes = [C.c_void_p, dp, dp]
        L.orc_oc_hessian.argtypes = [C.c_void_p, dp, C.c_int, dp]
        L.orc_oc_rows.argtypes = [C.c_void_p, dp, ip, C.c_int, dp]
        L.orc_oc_state.argtypes = [C.c_void_p, C.c_int, C.c_int, ip, dp, C.c_size_t, C.POINTER(C.c_size_t)]
        L.orc_oc_set_nested.argtypes = [C.c_void_p, C.c_int]
        L.orc_set_sector_threads.argtypes = [C.c_int]
        L.orc_oc_time_hessian.restype = C.c_double
        L.orc_oc_time_hessian.argtypes = [C.c_void_p, dp, C.c_int, dp]
        _lib = L
    return _lib


def _d(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(dp)


def _i(a):
    a = np.ascontiguousarray(a, dtype=np.int32)
    return a, a.ctypes.data_as(ip)


class MPS:
    """compact-format MPS (dims int32[(L+1)*(Q+1)], data complex128)."""

    def __init__(self, L, p, Q, dims, data):
        self.L, self.p, self.Q = L, p, Q
        self.dims = np.ascontiguousarray(np.asarray(dims, dtype=np.int32).reshape(-1))
        self.data = np.ascontiguousarray(np.asarray(data, dtype=np.complex128).reshape(-1))

    def bond_dims(self):
        return self.dims.reshape(self.L + 1, self.Q + 1).sum(axis=1)

    def raw(self):
        return self.data.view(np.float64)


def cap_for(L, p, Q, maxm=5000):
    # generous output capacity for the oracle's output buffers
    return 4 * p * (L + 1) * max(1, min(maxm, 4096)) ** 2 if L > 12 else 1 << 20


class Stepper:
    def __init__(self, L, p, Q, J, dt, cutoff, maxm=5000):
        self.L, self.p, self.Q = L, p, Q
        self.J, self.dt, self.cutoff, self.maxm = J, dt, cutoff, maxm
        self.h = lib().orc_new(L, p, Q, J, dt, cutoff, maxm)
        self.cap = 1 << 21  # complex elements (a saturated chi = 256 config-4 chain has ~5e5)

    def __del__(self):
        try:
            lib().orc_free(self.h)
        except Exception:
            pass

    def _out(self):
        return (np.zeros((self.L + 1) * (self.Q + 1), np.int32), np.zeros(2 * self.cap), C.c_size_t(0))

    def _wrap(self, fd, d, n):
        return MPS(self.L, self.p, self.Q, fd.copy(), d[:2 * n.value].view(np.complex128).copy())

    def step(self, m: MPS, u_from, u_to, forward=True) -> MPS:
        fd, d, n = self._out()
        _, pdims = _i(m.dims)
        raw, praw = _d(m.raw())
        rc = lib().orc_step(self.h, pdims, praw, u_from, u_to, int(forward),
                            fd.ctypes.data_as(ip), d.ctypes.data_as(dp), self.cap, C.byref(n))
        assert rc == 0, rc
        return self._wrap(fd, d, n)

    def steps(self, m: MPS, u, forward=True) -> MPS:
        fd, d, n = self._out()
        _, pdims = _i(m.dims)
        raw, praw = _d(m.raw())
        uu, pu = _d(u)
        rc = lib().orc_steps(self.h, pdims, praw, pu, len(uu) - 1, int(forward),
                             fd.ctypes.data_as(ip), d.ctypes.data_as(dp), self.cap, C.byref(n))
        assert rc == 0, rc
        return self._wrap(fd, d, n)

    def overlap(self, x: MPS, y: MPS) -> complex:
        out = np.zeros(2)
        _, a = _i(x.dims); rx, b = _d(x.raw()); _, c = _i(y.dims); ry, d = _d(y.raw())
        lib().orc_overlap(self.h, a, b, c, d, out.ctypes.data_as(dp))
        return complex(out[0], out[1])

    def overlap_dH(self, x: MPS, y: MPS) -> complex:
        out = np.zeros(2)
        _, a = _i(x.dims); rx, b = _d(x.raw()); _, c = _i(y.dims); ry, d = _d(y.raw())
        lib().orc_overlap_dH(self.h, a, b, c, d, out.ctypes.data_as(dp))
        return complex(out[0], out[1])

    def apply_dH(self, m: MPS) -> MPS:
        fd, d, n = self._out()
        _, pdims = _i(m.dims)
        raw, praw = _d(m.raw())
        rc = lib().orc_apply_dH(self.h, pdims, praw, fd.ctypes.data_as(ip), d.ctypes.data_as(dp),
                                self.cap, C.byref(n))
        assert rc == 0, rc
        return self._wrap(fd, d, n)

    def gate(self, forward=True):
        out = np.zeros(2 * self.p ** 4)
        lib().orc_gate(self.h, int(forward), out.ctypes.data_as(dp))
        return out.view(np.complex128).reshape(self.p ** 2, self.p ** 2)


class OC:
    """Oracle OptimalControl (GRAPE)."""

    def __init__(self, stepper: Stepper, target: MPS, init: MPS, N: int, gamma: float = 0.0):
        self.st = stepper
        self.N = N
        _, a = _i(target.dims); rt, b = _d(target.raw()); _, c = _i(init.dims); ri, d = _d(init.raw())
        self.h = lib().orc_oc_new(stepper.h, a, b, c, d, N, gamma)

    def __del__(self):
        try:
            lib().orc_oc_free(self.h)
        except Exception:
            pass

    def set_gamma(self, g):
        lib().orc_oc_set_gamma(self.h, g)

    def cost(self, u):
        uu, pu = _d(u)
        return lib().orc_oc_cost(self.h, pu)

    def fidelities(self, u):
        uu, pu = _d(u)
        out = np.zeros(self.N)
        lib().orc_oc_fidelities(self.h, pu, out.ctypes.data_as(dp))
        return out

    def gradient(self, u, bfgs=False):
        uu, pu = _d(u)
        out = np.zeros(self.N)
        lib().orc_oc_gradient(self.h, pu, int(bfgs), out.ctypes.data_as(dp))
        return out

    def divT_F(self):
        d = np.zeros(2 * self.N); F = np.zeros(2)
        lib().orc_oc_divT(self.h, d.ctypes.data_as(dp), F.ctypes.data_as(dp))
        return d.view(np.complex128).copy(), complex(F[0], F[1])

    def hessian(self, u, threads=1):
        uu, pu = _d(u)
        out = np.zeros(self.N * self.N)
        lib().orc_oc_hessian(self.h, pu, threads, out.ctypes.data_as(dp))
        return out.reshape(self.N, self.N)

    def rows(self, u, rows):
        """fidelity-Hessian entries of the given rows only (one rank's shard)"""
        uu, pu = _d(u)
        rr = np.ascontiguousarray(rows, dtype=np.int32)
        out = np.zeros(self.N * self.N)
        rc = lib().orc_oc_rows(self.h, pu, rr.ctypes.data_as(ip), len(rr), out.ctypes.data_as(dp))
        assert rc == 0, rc
        return out.reshape(self.N, self.N)

    def set_nested(self, on=True):
        """getHessian's threads also split the U(1) sectors inside each step (CPU
        baseline of the large configs; the same numbers bit for bit)"""
        lib().orc_oc_set_nested(self.h, int(on))

    def time_hessian(self, u, threads=1, out=None):
        """wall seconds of one getHessian; its Hessian into out (N x N float64) if given"""
        uu, pu = _d(u)
        if out is not None:
            assert out.dtype == np.float64 and out.flags.c_contiguous and out.size == self.N * self.N
            return lib().orc_oc_time_hessian(self.h, pu, threads, out.ctypes.data_as(dp))
        return lib().orc_oc_time_hessian(self.h, pu, threads, None)

    def state(self, which, t):
        fd, d, n = self.st._out()
        rc = lib().orc_oc_state(self.h, which, t, fd.ctypes.data_as(ip), d.ctypes.data_as(dp),
                                self.st.cap, C.byref(n))
        assert rc == 0, rc
        return self.st._wrap(fd, d, n)


def set_sector_threads(n):
    """U(1)-sector threads of this (calling) thread's oracle steps (1: serial)"""
    lib().orc_set_sector_threads(int(n))


def heev(A):
    n = A.shape[0]
    a = np.ascontiguousarray(A, dtype=np.complex128)
    w = np.zeros(n); v = np.zeros(2 * n * n)
    lib().orc_heev(n, a.view(np.float64).ctypes.data_as(dp), w.ctypes.data_as(dp), v.ctypes.data_as(dp))
    return w, v.view(np.complex128).reshape(n, n)


def heev_ql(A):
    """the oracle's Householder + QL solver (ORC_HEEV=ql) on one block"""
    n = A.shape[0]
    a = np.ascontiguousarray(A, dtype=np.complex128)
    w = np.zeros(n); v = np.zeros(2 * n * n)
    lib().orc_heev_ql(n, a.view(np.float64).ctypes.data_as(dp), w.ctypes.data_as(dp), v.ctypes.data_as(dp))
    return w, v.view(np.complex128).reshape(n, n)


def truncate(P, cutoff, maxm):
    P = np.ascontiguousarray(P, dtype=np.float64)
    return lib().orc_truncate(P.ctypes.data_as(dp), len(P), cutoff, maxm)
