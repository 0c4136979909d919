"""The drop-in boundary on CPU (no compute calls): liboptimalcontrolmps_amd.so
builds for gfx950, loads, exports every entry point include/ocmps.h declares,
and fails loudly (OCG_EHIP) instead of falling back when no GPU is present."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from optimalcontrolmps_amd import ed, native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ocmps.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ocg_[A-Za-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def so():
    return native.build_native()


def test_header_declares_the_boundary():
    names = declared()
    for must in ["ocg_create", "ocg_destroy", "ocg_last_error", "ocg_step", "ocg_steps", "ocg_overlap",
                 "ocg_apply_dH", "ocg_set_states", "ocg_propagate", "ocg_div_t", "ocg_xi_dH", "ocg_hessian_rows",
                 "ocg_overlap_factor", "ocg_fidelities", "ocg_get_state", "ocg_kernel_stats"]:
        assert must in names


def test_library_exports_every_declared_symbol(so):
    lib = C.CDLL(so)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (ocg_[A-Za-z_0-9]+)$", out, flags=re.M))
    assert set(declared()) <= exported


def test_python_signatures_cover_the_header(so):
    bound = {s[0] for s in native.SIGNATURES}
    assert set(declared()) <= bound


def test_code_object_is_gfx950(so):
    """the fat binary carries exactly one device target, gfx950"""
    blob = open(so, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", blob))
    assert targets == {b"gfx950"}


def test_mps_nelem_matches_host_count(so):
    lib = native.lib()
    for (L, p, Q) in [(5, 5, 5), (5, 6, 5), (3, 4, 3)]:
        psi, _ = ed.ground_state_full(L, p, Q, 1.0, 3.0)
        dims, data = ed.mps_from_full(psi, L, p, Q)
        d = np.ascontiguousarray(dims, dtype=np.int32).reshape(-1)
        n = lib.ocg_mps_nelem(L, p, Q, d.ctypes.data_as(C.POINTER(C.c_int)))
        assert n == len(data) == ed.nelem(d, L, p, Q)


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK),
                    reason="a GPU is visible: the loud-failure path is for GPU-less hosts")
def test_no_gpu_fails_loudly(so):
    with pytest.raises(native.OcgError):
        native.Engine(5, 5, 5, 1.0, 0.01, 1e-8, 80)
