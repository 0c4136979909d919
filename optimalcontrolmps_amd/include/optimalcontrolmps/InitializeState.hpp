// Ground-state preparation, the reference's InitializeState
// (include/InitializeState.hpp:18-117), on the MI355X: same signatures and
// starting guess, ITensor's DMRG replaced by imaginary-time evolution on the
// device (ocg_imag_steps: the BH_tDMRG sweep with exp(-tau h) gates and
// exp(-tau U n(n-1)/4) phases, normalised and truncated with the given
// threshold / maxBondDim).
//
//   starting guess  "Occ1" on the Npart right-most sites, "Emp" elsewhere
//                   (:26-40); Npart > N is refused like the reference
//   H               -J sum (a_i a^dag_{i+1} + h.c.) + U/2 sum n(n-1) (:42-51)
//   schedule        tau = 0.05, 0.01, 0.002, 0.001, 0.0005, each run in
//                   blocks of 25 steps until 1 - |<prev|new>| < 1e-13 (the
//                   tau^2 Trotter fixed-point infidelity: 6e-8 at L=5, U=2.5)
//   defaults        maxBondDim 200, threshold 1e-9 (the overload without
//                   them, :18-60: sweeps.maxm() up to 200, cutoff 1e-9)
#pragma once

#include <cmath>
#include <complex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/ocmps.h"
#include "MPS.hpp"

namespace ocmps {

// product state with Npart bosons on the right-most sites, all bonds 1
inline MPS productState(int L, int p, int Npart) {
  if (Npart > L) throw std::invalid_argument("Npart > N not supported");
  const int Q1 = Npart + 1;
  std::vector<int> dims(size_t(L + 1) * Q1, 0);
  int q = 0;
  dims[0] = 1;
  for (int b = 1; b <= L; ++b) {
    if (b > L - Npart) ++q;
    dims[size_t(b) * Q1 + q] = 1;
  }
  return MPS(L, p, Npart, dims, std::vector<Cplx>(size_t(L), Cplx(1.0, 0.0)));
}

namespace detail_gs {
inline void check(int rc, const ocg_ctx* c, const char* what) {
  if (rc != OCG_OK) {
    const char* m = ocg_last_error(c);
    throw std::runtime_error(std::string(what) + ": " + (m ? m : "error"));
  }
}
}  // namespace detail_gs

inline MPS InitializeState(const BoseHubbard& sites, const int Npart, const double J, const double U,
                           const int maxBondDim, const double threshold, bool /*silent*/ = true, int device = 0) {
  const int L = sites.N(), p = sites.localDim();
  MPS psi = productState(L, p, Npart);
  ocg_ctx* c = nullptr;
  detail_gs::check(ocg_create(device, L, p, Npart, J, 0.01, threshold, maxBondDim, &c), nullptr, "ocg_create");
  try {
    ocg_info info;
    detail_gs::check(ocg_get_info(c, &info), c, "ocg_get_info");
    std::vector<int> od(psi.dims.size());
    std::vector<Cplx> out(info.mps_max_nelem);
    const double taus[] = {0.05, 0.01, 0.002, 0.001, 0.0005};
    const int block = 25, max_steps = 8000;
    for (double tau : taus) {
      for (int done = 0; done < max_steps; done += block) {
        size_t n = 0;
        detail_gs::check(ocg_imag_steps(c, psi.dims.data(), psi.raw(), U, tau, block, od.data(),
                                        reinterpret_cast<double*>(out.data()), out.size(), &n),
                         c, "ocg_imag_steps");
        MPS nw(L, p, Npart, od, std::vector<Cplx>(out.begin(), out.begin() + n));
        double ov[2];
        detail_gs::check(ocg_overlap(c, psi.dims.data(), psi.raw(), nw.dims.data(), nw.raw(), 0, ov), c,
                         "ocg_overlap");
        psi = std::move(nw);
        if (1.0 - std::hypot(ov[0], ov[1]) < 1e-13) break;
      }
    }
  } catch (...) {
    ocg_destroy(c);
    throw;
  }
  ocg_destroy(c);
  return psi;
}

inline MPS InitializeState(const BoseHubbard& sites, const int Npart, const double J, const double U,
                           bool silent = true) {
  return InitializeState(sites, Npart, J, U, 200, 1e-9, silent);
}

}  // namespace ocmps
