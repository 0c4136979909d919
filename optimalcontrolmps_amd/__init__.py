"""MI355X-native gradient/Hessian inner loop of fskovbo/OptimalControlMPS.

The hot path (BH_tDMRG time stepping, the <xi|dH|psi> overlaps, dH|psi>
compression and the Hessian-row re-propagations) runs as hand-written HIP
kernels for gfx950 in liboptimalcontrolmps_amd.so behind the C-ABI of
include/ocmps.h; the C++ facade (include/optimalcontrolmps/) keeps the
reference's OptimalControl / TimeStepper / ControlBasis API.
"""
from .native import MPS, Engine, OcgError, build_native  # noqa: F401

__all__ = ["MPS", "Engine", "OcgError", "build_native"]
