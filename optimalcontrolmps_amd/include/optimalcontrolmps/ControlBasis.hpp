// GROUP control parameterisation: restatement of the reference's
// ControlBasis (include/ControlBasis.hpp:13-37, src/ControlBasis.cpp:1-124).
//
//   u_i = u0_i + S_i * sum_n f_{i n} c_n          (convertControl, :49-66)
//   dJ/dc_n = sum_i S_i f_{i n} dJ/du_i           (convertGradient, :69-88)
//   H_c = V H_u V^T,  V_{n i} = S_i f_{i n}       (convertHessian, :91-116)
//
// The Hessian projection is evaluated as two dense products (H_u V^T, then
// V (H_u V^T)), each accumulated in the same order as the reference's
// inner products, so the result is bit-identical to its row-by-row form.
#pragma once

#include <cassert>
#include <cstddef>
#include <vector>

#include "MPS.hpp"

class ControlBasis {
 public:
  using stdvec = ocmps::stdvec;
  using rowmat = ocmps::rowmat;

  ControlBasis() = default;
  ControlBasis(stdvec& u0_, stdvec& S_, rowmat& f_)
      : u0(u0_), S(S_), f(f_), N(u0_.size()), M(f_.empty() ? 0 : f_.front().size()) {
    // du_i / dc_n = S_i f_{i n}; V is its transpose
    jac.assign(N, stdvec(M, 0.0));
    V.assign(M, stdvec(N, 0.0));
    for (size_t i = 0; i < N; ++i)
      for (size_t n = 0; n < M; ++n) {
        jac[i][n] = f[i][n] * S[i];
        V[n][i] = jac[i][n];
      }
    ucurrent = u0;  // no coefficients given yet
  }

  size_t getM() const { return M; }
  size_t getN() const { return N; }

  // new_control == false returns the cached u of the last conversion (:49-66)
  stdvec convertControl(const stdvec& c, const bool new_control = true) {
    if (!new_control) return ucurrent;
    assert(c.size() == M);
    stdvec u(u0);
    for (size_t i = 0; i < N; ++i) {
      double fc = 0.0;
      for (size_t n = 0; n < M; ++n) fc += f[i][n] * c[n];
      u[i] += S[i] * fc;
    }
    ucurrent = u;
    return ucurrent;
  }

  stdvec convertGradient(const stdvec& gradu) const {
    assert(gradu.size() == N);
    stdvec gc(M, 0.0);
    for (size_t n = 0; n < M; ++n) {
      double acc = 0.0;
      for (size_t i = 0; i < N; ++i) acc += S[i] * gradu[i] * f[i][n];
      gc[n] = acc;
    }
    return gc;
  }

  rowmat convertHessian(const rowmat& Hu) const {
    assert(Hu.size() == N && (N == 0 || Hu.front().size() == N));
    // HV[j][k] = sum_l Hu[k][l] V[j][l]   (row k of H_u against basis vector j)
    rowmat HV(M, stdvec(N, 0.0));
    for (size_t j = 0; j < M; ++j)
      for (size_t k = 0; k < N; ++k) {
        double acc = 0.0;
        for (size_t l = 0; l < N; ++l) acc += Hu[k][l] * V[j][l];
        HV[j][k] = acc;
      }
    rowmat Hc(M, stdvec(M, 0.0));
    for (size_t i = 0; i < M; ++i)
      for (size_t j = i; j < M; ++j) {
        double acc = 0.0;
        for (size_t k = 0; k < N; ++k) acc += V[i][k] * HV[j][k];
        Hc[i][j] = acc;
        Hc[j][i] = acc;
      }
    return Hc;
  }

  rowmat getControlJacobian() const { return jac; }
  // V (M x N), V[n][i] = S_i f_{i n}: the operand of device projections
  // (GpuTDMRG::Engine::convertHessian, ocg_convert_hessian)
  const rowmat& basisMatrix() const { return V; }

 private:
  stdvec u0, S;
  rowmat f;
  size_t N = 0, M = 0;
  rowmat jac, V;
  stdvec ucurrent;
};
