"""ctypes binding of liboptimalcontrolmps_amd.so (include/ocmps.h).

The shared library is built in-tree (``build_native()``, also run by
``__graft_entry__.build()``) with hipcc for gfx950 and lives next to this
file.  There is no fallback: if the library is missing or the HIP runtime has
no GPU, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
LIB_NAME = "liboptimalcontrolmps_amd.so"
LIB_PATH = os.environ.get("OCG_LIB", os.path.join(PKG_DIR, LIB_NAME))
CSRC = os.path.join(PKG_DIR, "csrc")
HEADER = os.path.join(ROOT, "include", "ocmps.h")

OCG_ERRORS = {1: "EINVAL", 2: "ECAP", 3: "EHIP", 4: "ESTATE", 5: "ENUM"}


class OcgError(RuntimeError):
    pass


def sources():
    return [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC))
            if f.endswith((".hip", ".hpp", ".cpp", ".h"))] + [HEADER]


def build_native(force: bool = False, nt: int | None = None, verbose: bool = False) -> str:
    """Compile csrc/ocmps.hip (LDS chain engine + C-ABI) and csrc/hbm.hip (HBM
    engine) for gfx950 into objects (in parallel) and link the in-tree shared
    library.  Each object is rebuilt only when a source it depends on changed."""
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    bdir = os.path.join(PKG_DIR, "build")
    os.makedirs(bdir, exist_ok=True)
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result"]
    if nt:
        flags.append(f"-DOCG_NT={int(nt)}")
    deps = {
        "ocmps": ["ocmps.hip", "engine.hpp", "engine_device.hpp", "kernels.hpp", "params.hpp", "hbm.hpp",
                  "fast.hpp", "fast_plan.hpp", "fast_chain.hpp"],
        "hbm": ["hbm.hip", "hbm.hpp", "hbm_device.hpp", "hbm_eig.hpp"],
    }
    tag = f"nt{int(nt)}" if nt else "prod"
    objs, procs = [], []
    for name, srcs in deps.items():
        obj = os.path.join(bdir, f"{name}.{tag}.o")
        objs.append(obj)
        newest = max([os.path.getmtime(os.path.join(CSRC, f)) for f in srcs] + [os.path.getmtime(HEADER)])
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < newest:
            cmd = [hipcc] + flags + ["-c", os.path.join(CSRC, srcs[0]), "-o", obj + ".tmp"]
            if verbose:
                print(" ".join(cmd))
            procs.append((subprocess.Popen(cmd), obj))
    for pr, obj in procs:
        if pr.wait() != 0:
            raise OcgError(f"hipcc failed building {obj}")
        os.replace(obj + ".tmp", obj)
    if force or procs or not os.path.exists(LIB_PATH) or \
            os.path.getmtime(LIB_PATH) < max(os.path.getmtime(o) for o in objs):
        cmd = [hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", LIB_PATH + ".tmp"] + objs
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
        os.replace(LIB_PATH + ".tmp", LIB_PATH)
    return LIB_PATH


_lib = None
dp = C.POINTER(C.c_double)
ip = C.POINTER(C.c_int)
szp = C.POINTER(C.c_size_t)


class OcgInfo(C.Structure):
    _fields_ = [("L", C.c_int), ("p", C.c_int), ("Q", C.c_int), ("mps_max_nelem", C.c_size_t),
                ("lds_bytes", C.c_int), ("block_threads", C.c_int), ("device", C.c_int), ("fast_chain", C.c_int)]


class OcgPathStats(C.Structure):
    _fields_ = [("size", C.c_size_t), ("pipe_runs", C.c_long), ("pipe_fallbacks", C.c_long),
                ("ckpt_runs", C.c_long), ("ckpt_k", C.c_long), ("coop_launches", C.c_long),
                ("coop_groups", C.c_long), ("coop_fallbacks", C.c_long)]


# (name, restype, argtypes) for every entry point of include/ocmps.h
SIGNATURES = [
    ("ocg_create", C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, C.c_int,
                             C.POINTER(C.c_void_p)]),
    ("ocg_create_ex", C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double, C.c_int,
                                C.c_int, C.POINTER(C.c_void_p)]),
    ("ocg_destroy", C.c_int, [C.c_void_p]),
    ("ocg_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("ocg_last_error", C.c_char_p, [C.c_void_p]),
    ("ocg_get_info", C.c_int, [C.c_void_p, C.POINTER(OcgInfo)]),
    ("ocg_get_info_sz", C.c_int, [C.c_void_p, C.POINTER(OcgInfo), C.c_size_t]),
    ("ocg_abi_version", C.c_int, []),
    ("ocg_get_path_stats", C.c_int, [C.c_void_p, C.POINTER(OcgPathStats)]),
    ("ocg_set_tstep", C.c_int, [C.c_void_p, C.c_double]),
    ("ocg_mps_nelem", C.c_size_t, [C.c_int, C.c_int, C.c_int, ip]),
    ("ocg_step", C.c_int, [C.c_void_p, ip, dp, C.c_double, C.c_double, C.c_int, ip, dp, C.c_size_t, szp]),
    ("ocg_steps", C.c_int, [C.c_void_p, ip, dp, dp, C.c_int, C.c_int, ip, dp, C.c_size_t, szp]),
    ("ocg_imag_steps", C.c_int, [C.c_void_p, ip, dp, C.c_double, C.c_double, C.c_int, ip, dp, C.c_size_t, szp]),
    ("ocg_ground_state", C.c_int, [C.c_void_p, ip, dp, C.c_double, C.c_int, dp, C.c_int, C.c_double, C.c_int, ip, dp,
                                   C.c_size_t, szp, ip]),
    ("ocg_step_batch", C.c_int, [C.c_void_p, C.c_int, ip, C.POINTER(dp), dp, dp, C.c_int, ip, C.POINTER(dp), szp,
                                 szp]),
    ("ocg_overlap", C.c_int, [C.c_void_p, ip, dp, ip, dp, C.c_int, dp]),
    ("ocg_apply_dH", C.c_int, [C.c_void_p, ip, dp, ip, dp, C.c_size_t, szp, dp]),
    ("ocg_set_states", C.c_int, [C.c_void_p, ip, dp, ip, dp]),
    ("ocg_propagate", C.c_int, [C.c_void_p, dp, C.c_int, C.c_int]),
    ("ocg_overlap_factor", C.c_int, [C.c_void_p, dp]),
    ("ocg_fidelities", C.c_int, [C.c_void_p, dp]),
    ("ocg_div_t", C.c_int, [C.c_void_p, dp]),
    ("ocg_xi_dH", C.c_int, [C.c_void_p]),
    ("ocg_hessian_rows", C.c_int, [C.c_void_p, dp, C.c_int, ip, C.c_int, dp, dp, dp]),
    ("ocg_hessian", C.c_int, [C.c_void_p, dp, C.c_int, ip, C.c_int, dp, dp, dp]),
    ("ocg_hessian_multi", C.c_int, [C.c_void_p, C.c_int, dp, C.c_int, ip, C.c_int, dp, dp, dp]),
    ("ocg_gradient_multi", C.c_int, [C.c_void_p, C.c_int, dp, C.c_int, dp, dp]),
    ("ocg_gradient", C.c_int, [C.c_void_p, dp, C.c_int, dp, dp]),
    ("ocg_get_state", C.c_int, [C.c_void_p, C.c_int, C.c_int, ip, dp, C.c_size_t, szp]),
    ("ocg_convert_hessian", C.c_int, [C.c_void_p, dp, C.c_int, dp, C.c_int, dp]),
    ("ocg_denmat_decomp", C.c_int, [C.c_void_p, C.c_int, ip, ip, C.POINTER(dp), C.c_double, C.c_int, ip,
                                    C.POINTER(dp), C.POINTER(dp), C.POINTER(dp)]),
    ("ocg_kernel_stats", C.c_int, [C.c_void_p, C.c_int, dp, C.POINTER(C.c_long), dp, dp, C.POINTER(C.c_long)]),
    ("ocg_reset_stats", C.c_int, [C.c_void_p]),
    ("ocg_profile", C.c_int, [C.c_void_p, dp, C.c_int]),
]


def lib():
    """Load the native library (raises OcgError if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OcgError(f"{LIB_NAME} not built: run optimalcontrolmps_amd.native.build_native() "
                           "or __graft_entry__.build() (no CPU fallback exists)")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _d(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(dp)


def _i(a):
    a = np.ascontiguousarray(a, dtype=np.int32)
    return a, a.ctypes.data_as(ip)


class MPS:
    """Host MPS in the compact U(1)-block interchange format of include/ocmps.h
    (the IQMPS replacement): dims int32[(L+1)*(Q+1)], data complex128."""

    def __init__(self, L, p, Q, dims, data):
        self.L, self.p, self.Q = int(L), int(p), int(Q)
        self.dims = np.ascontiguousarray(np.asarray(dims, dtype=np.int32).reshape(-1))
        self.data = np.ascontiguousarray(np.asarray(data, dtype=np.complex128).reshape(-1))

    def bond_dims(self):
        return self.dims.reshape(self.L + 1, self.Q + 1).sum(axis=1)

    def raw(self):
        return self.data.view(np.float64)

    def copy(self):
        return MPS(self.L, self.p, self.Q, self.dims.copy(), self.data.copy())


class Engine:
    """One device context (ocg_ctx): the BH_tDMRG stepper + device-resident
    trajectories of the OptimalControl hot path."""

    ENGINES = {"auto": 0, "lds": 1, "hbm": 2}

    def __init__(self, L, p, npart, J, tstep, cutoff, maxm=0, device=0, engine="auto"):
        self.L, self.p, self.Q = L, p, npart
        self.J, self.tstep, self.cutoff, self.maxm = J, tstep, cutoff, maxm
        h = C.c_void_p()
        rc = lib().ocg_create_ex(device, L, p, npart, J, tstep, cutoff, maxm, self.ENGINES[engine], C.byref(h))
        if rc != 0:
            raise OcgError(f"ocg_create failed ({OCG_ERRORS.get(rc, rc)}): "
                           f"{lib().ocg_last_error(None).decode()}")
        self.h = h
        info = OcgInfo()
        lib().ocg_get_info(self.h, C.byref(info))
        self.info = info
        self.cap = int(info.mps_max_nelem)
        self.N = 0

    def close(self):
        if getattr(self, "h", None):
            lib().ocg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        if rc != 0:
            raise OcgError(f"{what} failed ({OCG_ERRORS.get(rc, rc)}): {lib().ocg_last_error(self.h).decode()}")

    def _out(self):
        return (np.zeros((self.L + 1) * (self.Q + 1), np.int32), np.zeros(2 * self.cap), C.c_size_t(0))

    def _wrap(self, fd, d, n):
        return MPS(self.L, self.p, self.Q, fd.copy(), d[:2 * n.value].view(np.complex128).copy())

    # ------------------------------------------------ TimeStepper-level
    def step(self, m: MPS, u_from, u_to, forward=True) -> MPS:
        fd, d, n = self._out()
        _, pd = _i(m.dims)
        raw, pr = _d(m.raw())
        self._chk(lib().ocg_step(self.h, pd, pr, u_from, u_to, int(forward), fd.ctypes.data_as(ip),
                                 d.ctypes.data_as(dp), self.cap, C.byref(n)), "ocg_step")
        return self._wrap(fd, d, n)

    def steps(self, m: MPS, u, forward=True) -> MPS:
        fd, d, n = self._out()
        _, pd = _i(m.dims)
        raw, pr = _d(m.raw())
        uu, pu = _d(u)
        self._chk(lib().ocg_steps(self.h, pd, pr, pu, len(uu) - 1, int(forward), fd.ctypes.data_as(ip),
                                  d.ctypes.data_as(dp), self.cap, C.byref(n)), "ocg_steps")
        return self._wrap(fd, d, n)

    def imag_steps(self, m: MPS, U, tau, nsteps) -> MPS:
        """nsteps imaginary-time steps exp(-tau H(J, U)) (ground-state preparation)"""
        fd, d, n = self._out()
        _, pd = _i(m.dims)
        raw, pr = _d(m.raw())
        self._chk(lib().ocg_imag_steps(self.h, pd, pr, float(U), float(tau), int(nsteps), fd.ctypes.data_as(ip),
                                       d.ctypes.data_as(dp), self.cap, C.byref(n)), "ocg_imag_steps")
        return self._wrap(fd, d, n)

    def ground_state(self, m: MPS, U, taus, block=25, tol=1e-13, max_steps=8000):
        """InitializeState's tau schedule on the device in one call (ocg_ground_state):
        returns (state, steps taken)"""
        fd, d, n = self._out()
        _, pd = _i(m.dims)
        raw, pr = _d(m.raw())
        tt, pt = _d(np.asarray(taus, np.float64))
        steps = C.c_int(0)
        self._chk(lib().ocg_ground_state(self.h, pd, pr, float(U), len(tt), pt, int(block), float(tol), int(max_steps),
                                         fd.ctypes.data_as(ip), d.ctypes.data_as(dp), self.cap, C.byref(n),
                                         C.byref(steps)), "ocg_ground_state")
        return self._wrap(fd, d, n), steps.value

    def step_batch(self, states, u_from, u_to, forward=True):
        """one step of every state (own controls each) in a single launch"""
        n = len(states)
        if n == 0:
            return []
        nsq = (self.L + 1) * (self.Q + 1)
        dims = np.ascontiguousarray(np.concatenate([m.dims for m in states]).astype(np.int32))
        raws = [np.ascontiguousarray(m.raw()) for m in states]
        data = (dp * n)(*[r.ctypes.data_as(dp) for r in raws])
        uf, puf = _d(np.asarray(u_from, np.float64).reshape(n))
        ut, put = _d(np.asarray(u_to, np.float64).reshape(n))
        od = np.zeros(n * nsq, np.int32)
        outs = [np.zeros(2 * self.cap) for _ in range(n)]
        odata = (dp * n)(*[o.ctypes.data_as(dp) for o in outs])
        caps = np.full(n, self.cap, dtype=np.uintp)
        nel = np.zeros(n, dtype=np.uintp)
        self._chk(lib().ocg_step_batch(self.h, n, dims.ctypes.data_as(ip), data, puf, put, int(forward),
                                       od.ctypes.data_as(ip), odata, caps.ctypes.data_as(szp),
                                       nel.ctypes.data_as(szp)), "ocg_step_batch")
        return [MPS(self.L, self.p, self.Q, od[i * nsq:(i + 1) * nsq].copy(),
                    outs[i][:2 * int(nel[i])].view(np.complex128).copy()) for i in range(n)]

    def overlap(self, x: MPS, y: MPS, with_dH=False) -> complex:
        out = np.zeros(2)
        _, a = _i(x.dims); rx, b = _d(x.raw()); _, c = _i(y.dims); ry, d = _d(y.raw())
        self._chk(lib().ocg_overlap(self.h, a, b, c, d, int(with_dH), out.ctypes.data_as(dp)), "ocg_overlap")
        return complex(out[0], out[1])

    def apply_dH(self, m: MPS):
        fd, d, n = self._out()
        nrm = C.c_double(0)
        _, pd = _i(m.dims)
        raw, pr = _d(m.raw())
        self._chk(lib().ocg_apply_dH(self.h, pd, pr, fd.ctypes.data_as(ip), d.ctypes.data_as(dp), self.cap,
                                     C.byref(n), C.byref(nrm)), "ocg_apply_dH")
        return self._wrap(fd, d, n), nrm.value

    # ------------------------------------------------ OptimalControl hot path
    def set_states(self, target: MPS, init: MPS):
        _, a = _i(target.dims); rt, b = _d(target.raw()); _, c = _i(init.dims); ri, d = _d(init.raw())
        self._chk(lib().ocg_set_states(self.h, a, b, c, d), "ocg_set_states")

    def propagate(self, u, which=3):
        uu, pu = _d(u)
        self.N = len(uu)
        self._chk(lib().ocg_propagate(self.h, pu, len(uu), which), "ocg_propagate")

    def overlap_factor(self) -> complex:
        out = np.zeros(2)
        self._chk(lib().ocg_overlap_factor(self.h, out.ctypes.data_as(dp)), "ocg_overlap_factor")
        return complex(out[0], out[1])

    def _need_N(self):
        if self.N <= 0:
            raise OcgError("no device trajectories yet: propagate() or hessian() first")

    def fidelities(self):
        self._need_N()
        out = np.zeros(self.N)
        self._chk(lib().ocg_fidelities(self.h, out.ctypes.data_as(dp)), "ocg_fidelities")
        return out

    def div_t(self):
        self._need_N()
        out = np.zeros(2 * self.N)
        self._chk(lib().ocg_div_t(self.h, out.ctypes.data_as(dp)), "ocg_div_t")
        return out.view(np.complex128).copy()

    def xi_dH(self):
        self._chk(lib().ocg_xi_dH(self.h), "ocg_xi_dH")

    def hessian_rows(self, u, rows, F: complex, divT, H=None):
        uu, pu = _d(u)
        N = len(uu)
        r, pr = _i(rows)
        Fa = np.array([F.real, F.imag])
        dv = np.ascontiguousarray(np.asarray(divT, np.complex128)).view(np.float64)
        if H is None:
            H = np.zeros((N, N))
        H = np.ascontiguousarray(H, dtype=np.float64)
        self._chk(lib().ocg_hessian_rows(self.h, pu, N, pr, len(r), Fa.ctypes.data_as(dp), dv.ctypes.data_as(dp),
                                         H.ctypes.data_as(dp)), "ocg_hessian_rows")
        return H

    def hessian(self, u, rows=None, H=None):
        """fused getHessian(u, new_control=true) fidelity part for `rows`
        (default 1..N-2): returns (H, divT, F); device trajectories are left
        as after propagate(u, 3) + xi_dH()"""
        uu, pu = _d(u)
        N = len(uu)
        self.N = N  # the device trajectories now have N states (fidelities / div_t size their outputs by it)
        if rows is None:
            rows = range(1, N - 1)
        r, pr = _i(list(rows))
        if H is None:
            H = np.zeros((N, N))
        H = np.ascontiguousarray(H, dtype=np.float64)
        dv = np.zeros(2 * N)
        Fa = np.zeros(2)
        self._chk(lib().ocg_hessian(self.h, pu, N, pr, len(r), H.ctypes.data_as(dp), dv.ctypes.data_as(dp),
                                    Fa.ctypes.data_as(dp)), "ocg_hessian")
        return H, dv.view(np.complex128).copy(), complex(Fa[0], Fa[1])

    def hessian_multi(self, U, rows=None):
        """K control vectors (rows of U, K x N) in one ocg_hessian_multi call:
        returns (H (K, N, N), divT (K, N), F (K,)); the device keeps control 0's
        trajectories"""
        Um = np.ascontiguousarray(np.atleast_2d(np.asarray(U, dtype=np.float64)))
        K, N = Um.shape
        self.N = N
        if rows is None:
            rows = range(1, N - 1)
        r, pr = _i(list(rows))
        H = np.zeros((K, N, N))
        dv = np.zeros((K, 2 * N))
        Fa = np.zeros((K, 2))
        self._chk(lib().ocg_hessian_multi(self.h, K, Um.ctypes.data_as(dp), N, pr, len(r), H.ctypes.data_as(dp),
                                          dv.ctypes.data_as(dp), Fa.ctypes.data_as(dp)), "ocg_hessian_multi")
        return H, dv.view(np.complex128).copy(), Fa[:, 0] + 1j * Fa[:, 1]

    def gradient(self, u):
        """getAnalyticGradient's device part for one control (ocg_gradient):
        returns (divT (N,), F); on the HBM engine, when the stored trajectories
        would not fit, psi || xi meet in the middle and none are kept"""
        uu, pu = _d(u)
        N = len(uu)
        dv = np.zeros(2 * N)
        Fa = np.zeros(2)
        self._chk(lib().ocg_gradient(self.h, pu, N, dv.ctypes.data_as(dp), Fa.ctypes.data_as(dp)), "ocg_gradient")
        self.N = N
        return dv.view(np.complex128).copy(), complex(Fa[0], Fa[1])

    def gradient_multi(self, U):
        """psi || xi + divT + F for K control vectors (rows of U) in one call:
        returns (divT (K, N), F (K,)); the device keeps control 0's trajectories"""
        Um = np.ascontiguousarray(np.atleast_2d(np.asarray(U, dtype=np.float64)))
        K, N = Um.shape
        self.N = N
        dv = np.zeros((K, 2 * N))
        Fa = np.zeros((K, 2))
        self._chk(lib().ocg_gradient_multi(self.h, K, Um.ctypes.data_as(dp), N, dv.ctypes.data_as(dp),
                                           Fa.ctypes.data_as(dp)), "ocg_gradient_multi")
        return dv.view(np.complex128).copy(), Fa[:, 0] + 1j * Fa[:, 1]

    def convert_hessian(self, Hu, V):
        """ControlBasis::convertHessian on the device: V Hu V^T (V is M x N)"""
        H, ph = _d(Hu)
        Vm, pv = _d(V)
        M, N = Vm.shape
        out = np.zeros((M, M))
        self._chk(lib().ocg_convert_hessian(self.h, ph, N, pv, M, out.ctypes.data_as(dp)), "ocg_convert_hessian")
        return out

    def denmat_decomp(self, mats, cutoff=None, maxm=None):
        """ITensor denmatDecomp (Fromleft) of independent dense complex blocks
        (rows <= cols <= any, rows <= 512) through the HBM engine's batched
        decomposition path (ocg_denmat_decomp): returns [(k, w, A, B)] with A
        (rows x k, orthonormal columns), B = A^H M (k x cols) and the rows Gram
        eigenvalues w as the eigensolver left them."""
        n = len(mats)
        Ms = [np.ascontiguousarray(np.asarray(m, np.complex128)) for m in mats]
        rows, pr = _i([m.shape[0] for m in Ms])
        cols, pc = _i([m.shape[1] for m in Ms])
        ws = [np.zeros(m.shape[0]) for m in Ms]
        As = [np.zeros(2 * m.shape[0] * m.shape[0]) for m in Ms]
        Bs = [np.zeros(2 * m.shape[0] * m.shape[1]) for m in Ms]
        arr = lambda xs: (dp * n)(*[x.view(np.float64).ctypes.data_as(dp) for x in xs])
        kept = np.zeros(n, np.int32)
        self._chk(lib().ocg_denmat_decomp(self.h, n, pr, pc, arr(Ms), self.cutoff if cutoff is None else cutoff,
                                          self.maxm if maxm is None else maxm, kept.ctypes.data_as(ip), arr(ws),
                                          arr(As), arr(Bs)), "ocg_denmat_decomp")
        out = []
        for i, m in enumerate(Ms):
            k, r, c = int(kept[i]), m.shape[0], m.shape[1]
            out.append((k, ws[i], As[i].view(np.complex128)[:r * k].reshape(r, k),
                        Bs[i].view(np.complex128)[:k * c].reshape(k, c)))
        return out

    def state(self, which, t) -> MPS:
        fd, d, n = self._out()
        self._chk(lib().ocg_get_state(self.h, which, t, fd.ctypes.data_as(ip), d.ctypes.data_as(dp), self.cap,
                                      C.byref(n)), "ocg_get_state")
        return self._wrap(fd, d, n)

    def stats(self, kind):
        ms = C.c_double(); n = C.c_long(); b = C.c_double(); f = C.c_double(); s = C.c_long()
        self._chk(lib().ocg_kernel_stats(self.h, kind, C.byref(ms), C.byref(n), C.byref(b), C.byref(f),
                                         C.byref(s)), "ocg_kernel_stats")
        return {"ms": ms.value, "launches": n.value, "alg_bytes": b.value, "alg_flops": f.value,
                "sweep_steps": s.value}

    def path_stats(self):
        """named path counters of the HBM engine (ocg_get_path_stats): pipelined /
        two-phase-fallback / checkpointed getHessians, multi-CU eigenvalue launches,
        blocks and groups re-run on one CU"""
        st = OcgPathStats()
        st.size = C.sizeof(OcgPathStats)
        self._chk(lib().ocg_get_path_stats(self.h, C.byref(st)), "ocg_get_path_stats")
        return {k: getattr(st, k) for k, _ in OcgPathStats._fields_ if k != "size"}

    def profile(self, reset=True):
        out = np.zeros(32)
        self._chk(lib().ocg_profile(self.h, out.ctypes.data_as(dp), int(reset)), "ocg_profile")
        return out

    def reset_stats(self):
        self._chk(lib().ocg_reset_stats(self.h), "ocg_reset_stats")
