"""TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU emulation of the device
bodies (tests/emu/emu.cpp, built by `make -C tests/emu`)."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("EMU_LIB") or os.path.join(HERE, "build", "libocmps_emu.so")
dp = C.POINTER(C.c_double)
ip = C.POINTER(C.c_int)
_lib = None


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(LIB)
        L.emu_new_ex.restype = C.c_void_p
        L.emu_new_ex.argtypes = [C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, C.c_int, C.c_int]
        L.emu_free.argtypes = [C.c_void_p]
        L.emu_steps.restype = C.c_size_t
        L.emu_steps.argtypes = [C.c_void_p, ip, dp, dp, C.c_int, C.c_int, ip, dp]
        if hasattr(L, "emu_hessian_fused"):  # absent from the steps-only sanitizer build
            L.emu_hessian_fused.argtypes = [C.c_void_p, ip, dp, ip, dp, dp, C.c_int, dp, dp, dp]
            L.emu_hessian.argtypes = [C.c_void_p, ip, dp, ip, dp, dp, C.c_int, dp, dp, dp, dp, C.c_int]
            L.emu_overlap_pad.argtypes = [C.c_void_p, ip, dp, ip, dp, C.c_int, dp]
        _lib = L
    return _lib


class Emu:
    def __init__(self, L, p, Q, J, dt, cutoff, maxm, fast):
        self.L, self.p, self.Q = L, p, Q
        self.h = lib().emu_new_ex(L, p, Q, J, dt, cutoff, maxm, int(fast))
        if not self.h:
            raise RuntimeError("emulator context not available")
        self.cap = 1 << 16

    def __del__(self):
        if getattr(self, "h", None):
            lib().emu_free(self.h)

    def steps(self, dims, data, u, forward=True):
        d = np.ascontiguousarray(dims, np.int32)
        x = np.ascontiguousarray(data, np.complex128).view(np.float64)
        uu = np.ascontiguousarray(u, np.float64)
        od = np.zeros_like(d)
        ox = np.zeros(2 * self.cap)
        n = lib().emu_steps(self.h, d.ctypes.data_as(ip), x.ctypes.data_as(dp), uu.ctypes.data_as(dp),
                            len(uu) - 1, int(forward), od.ctypes.data_as(ip), ox.ctypes.data_as(dp))
        return od, ox[:2 * n].view(np.complex128).copy()

    def hessian_fused(self, tdims, tdata, idims, idata, u):
        N = len(u)
        H = np.zeros(N * N)
        dv = np.zeros(2 * N)
        F = np.zeros(2)
        a = [np.ascontiguousarray(v, np.int32) for v in (tdims, idims)]
        b = [np.ascontiguousarray(v, np.complex128).view(np.float64) for v in (tdata, idata)]
        uu = np.ascontiguousarray(u, np.float64)
        lib().emu_hessian_fused(self.h, a[0].ctypes.data_as(ip), b[0].ctypes.data_as(dp), a[1].ctypes.data_as(ip),
                                b[1].ctypes.data_as(dp), uu.ctypes.data_as(dp), N, H.ctypes.data_as(dp),
                                dv.ctypes.data_as(dp), F.ctypes.data_as(dp))
        return H.reshape(N, N), dv.view(np.complex128), complex(F[0], F[1])

    def hessian(self, tdims, tdata, idims, idata, u):
        """the unfused path (trajectories, divT / F, exactApplyMPO batches, k_hessian_rows)"""
        N = len(u)
        H = np.zeros(N * N)
        dv = np.zeros(2 * N)
        F = np.zeros(2)
        fid = np.zeros(N)
        a = [np.ascontiguousarray(v, np.int32) for v in (tdims, idims)]
        b = [np.ascontiguousarray(v, np.complex128).view(np.float64) for v in (tdata, idata)]
        uu = np.ascontiguousarray(u, np.float64)
        lib().emu_hessian(self.h, a[0].ctypes.data_as(ip), b[0].ctypes.data_as(dp), a[1].ctypes.data_as(ip),
                          b[1].ctypes.data_as(dp), uu.ctypes.data_as(dp), N, H.ctypes.data_as(dp),
                          dv.ctypes.data_as(dp), F.ctypes.data_as(dp), fid.ctypes.data_as(dp), N)
        return H.reshape(N, N), dv.view(np.complex128), complex(F[0], F[1])

    def overlap_pad(self, dx, x, dy, y, with_dH=False):
        """<x|y> or <x|dH|y> on the padded contraction (csrc/fast_overlap.hpp)"""
        a = [np.ascontiguousarray(v, np.int32) for v in (dx, dy)]
        b = [np.ascontiguousarray(v, np.complex128).view(np.float64) for v in (x, y)]
        out = np.zeros(2)
        rc = lib().emu_overlap_pad(self.h, a[0].ctypes.data_as(ip), b[0].ctypes.data_as(dp), a[1].ctypes.data_as(ip),
                                   b[1].ctypes.data_as(dp), int(with_dH), out.ctypes.data_as(dp))
        if rc != 0:
            raise RuntimeError("no padded overlap plan")
        return complex(out[0], out[1])
