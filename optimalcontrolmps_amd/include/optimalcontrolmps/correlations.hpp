// Observables of the drivers (reference include/correlations.hpp, used by
// main/ExtendTimeEvolution.cpp, AnalyzeQuench.cpp, AnalyzeBondDim.cpp) over
// ocmps::MPS, with the reference's names, arguments and conventions:
//
//   expectationValue(sites, psi, op, i)            <psi| op_i |psi>          (:100-108)
//   expectationValues(sites, psi, op)              i = 1..N                   (:110-118)
//   correlationFunction(sites, psi, op1, i, op2, j) <psi| op1_i op2_j |psi>   (:9-53);
//                                                  i == j: real part of <op1 op2> on one site
//   correlationMatrix(sites, psi, op1, op2)        rho_ij, rho_ji = conj(rho_ij) (:55-78)
//   correlationTerm(sites, psi, op1, op2)          largest eigenvalue of rho  (:80-98)
//   entanglementEntropy(sites, psi)                von Neumann entropy of every bond,
//                                                  weights below 1e-12 dropped (:120-149)
//
// Site operators as include/BH_sites.h:114-176 defines them: "N", "A", "Adag",
// "N(N-1)", "NN" and "Id" (which, like the reference's, has no n = 0 entry).
//
// Host code (these are analysis calls, not the optimisation's hot path).  The
// contractions are exact and gauge-free: left and right environments are
// both formed, so any MPS the engine returns (trajectory states carry their
// orthogonality centre on site 2) gives the reference's value for a
// normalised state.  Entanglement weights come from the Gram matrices of the
// left and right blocks per U(1) sector (eig(L^1/2 R^T L^1/2)).
#pragma once

#include <algorithm>
#include <cmath>
#include <complex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "MPS.hpp"

namespace ocmps {

namespace obs {

using cmat = std::vector<Cplx>;  // row-major square or rectangular blocks

// p x p matrix O[out][in] of a BosonSite operator (include/BH_sites.h:114-176)
inline std::vector<double> siteOp(const std::string& name, int p) {
  std::vector<double> O(size_t(p) * p, 0.0);
  auto at = [&](int out, int in) -> double& { return O[size_t(out) * p + in]; };
  if (name == "N") {
    for (int j = 0; j < p; ++j) at(j, j) = j;
  } else if (name == "A") {
    for (int j = 1; j < p; ++j) at(j - 1, j) = std::sqrt(double(j));
  } else if (name == "Adag") {
    for (int j = 1; j < p; ++j) at(j, j - 1) = std::sqrt(double(j));
  } else if (name == "N(N-1)") {
    for (int j = 1; j < p; ++j) at(j, j) = double(j) * j - j;
  } else if (name == "NN") {
    for (int j = 1; j < p; ++j) at(j, j) = double(j) * j;
  } else if (name == "Id") {
    for (int j = 1; j < p; ++j) at(j, j) = 1.0;
  } else {
    throw std::invalid_argument("Operator \"" + name + "\" name not recognized");
  }
  return O;
}
inline std::vector<double> identityOp(int p) {
  std::vector<double> O(size_t(p) * p, 0.0);
  for (int j = 0; j < p; ++j) O[size_t(j) * p + j] = 1.0;
  return O;
}
// a * b as operators (b acts first)
inline std::vector<double> opProduct(const std::vector<double>& a, const std::vector<double>& b, int p) {
  std::vector<double> c(size_t(p) * p, 0.0);
  for (int i = 0; i < p; ++i)
    for (int k = 0; k < p; ++k)
      for (int j = 0; j < p; ++j) c[size_t(i) * p + j] += a[size_t(i) * p + k] * b[size_t(k) * p + j];
  return c;
}

// dense site tensors A_k[a][n][c] (bond states ordered by sector) from the
// compact U(1) blocks of include/ocmps.h
struct Dense {
  int L = 0, p = 0;
  std::vector<int> chi;                 // [b] bond dimension
  std::vector<std::vector<int>> off;    // [b][q] first state of sector q
  std::vector<cmat> A;                  // [k], k = 1..L
};
inline Dense dense(const MPS& psi) {
  Dense D;
  D.L = psi.L;
  D.p = psi.p;
  const int Q1 = psi.Q + 1;
  D.chi.assign(psi.L + 1, 0);
  D.off.assign(psi.L + 1, std::vector<int>(Q1 + 1, 0));
  for (int b = 0; b <= psi.L; ++b) {
    for (int q = 0; q < Q1; ++q) D.off[b][q + 1] = D.off[b][q] + psi.dim(b, q);
    D.chi[b] = D.off[b][Q1];
  }
  D.A.assign(psi.L + 1, cmat());
  size_t e = 0;
  for (int k = 1; k <= psi.L; ++k) {
    const int cl = D.chi[k - 1], cr = D.chi[k], p = psi.p;
    cmat& A = D.A[k];
    A.assign(size_t(cl) * p * cr, Cplx(0, 0));
    for (int q = 0; q < Q1; ++q)
      for (int n = 0; n < p && q + n <= psi.Q; ++n) {
        const int r = psi.dim(k - 1, q), c = psi.dim(k, q + n);
        for (int a = 0; a < r; ++a)
          for (int x = 0; x < c; ++x)
            A[(size_t(D.off[k - 1][q] + a) * p + n) * cr + D.off[k][q + n] + x] = psi.data[e++];
      }
  }
  return D;
}

// E'[c'][c] = sum conj(A[a'][n'][c']) O[n'][n] E[a'][a] A[a][n][c]
inline cmat leftStep(const Dense& D, int k, const cmat& E, const std::vector<double>& O) {
  const int cl = D.chi[k - 1], cr = D.chi[k], p = D.p;
  const cmat& A = D.A[k];
  cmat T(size_t(cl) * p * cr, Cplx(0, 0));  // T[a'][n][c] = sum_a E[a'][a] A[a][n][c]
  for (int x = 0; x < cl; ++x)
    for (int a = 0; a < cl; ++a) {
      const Cplx e = E[size_t(x) * cl + a];
      if (e == Cplx(0, 0)) continue;
      const Cplx* src = &A[size_t(a) * p * cr];
      Cplx* dst = &T[size_t(x) * p * cr];
      for (size_t i = 0; i < size_t(p) * cr; ++i) dst[i] += e * src[i];
    }
  cmat U(size_t(cl) * p * cr, Cplx(0, 0));  // U[a'][n'][c] = sum_n O[n'][n] T[a'][n][c]
  for (int x = 0; x < cl; ++x)
    for (int np = 0; np < p; ++np)
      for (int n = 0; n < p; ++n) {
        const double o = O[size_t(np) * p + n];
        if (o == 0.0) continue;
        const Cplx* src = &T[(size_t(x) * p + n) * cr];
        Cplx* dst = &U[(size_t(x) * p + np) * cr];
        for (int c = 0; c < cr; ++c) dst[c] += o * src[c];
      }
  cmat R(size_t(cr) * cr, Cplx(0, 0));
  for (size_t xn = 0; xn < size_t(cl) * p; ++xn) {
    const Cplx* ab = &A[xn * cr];
    const Cplx* u = &U[xn * cr];
    for (int cp = 0; cp < cr; ++cp) {
      const Cplx b = std::conj(ab[cp]);
      if (b == Cplx(0, 0)) continue;
      Cplx* dst = &R[size_t(cp) * cr];
      for (int c = 0; c < cr; ++c) dst[c] += b * u[c];
    }
  }
  return R;
}
// R'[a'][a] = sum conj(A[a'][n'][c']) O[n'][n] A[a][n][c] R[c'][c]
inline cmat rightStep(const Dense& D, int k, const cmat& Rn, const std::vector<double>& O) {
  const int cl = D.chi[k - 1], cr = D.chi[k], p = D.p;
  const cmat& A = D.A[k];
  cmat T(size_t(cl) * p * cr, Cplx(0, 0));  // T[a][n][c'] = sum_c A[a][n][c] R[c'][c]
  for (size_t an = 0; an < size_t(cl) * p; ++an)
    for (int cp = 0; cp < cr; ++cp) {
      Cplx s = 0;
      for (int c = 0; c < cr; ++c) s += A[an * cr + c] * Rn[size_t(cp) * cr + c];
      T[an * cr + cp] = s;
    }
  cmat out(size_t(cl) * cl, Cplx(0, 0));
  for (int ap = 0; ap < cl; ++ap)
    for (int np = 0; np < p; ++np)
      for (int n = 0; n < p; ++n) {
        const double o = O[size_t(np) * p + n];
        if (o == 0.0) continue;
        const Cplx* bra = &A[(size_t(ap) * p + np) * cr];
        for (int a = 0; a < cl; ++a) {
          const Cplx* t = &T[(size_t(a) * p + n) * cr];
          Cplx s = 0;
          for (int cp = 0; cp < cr; ++cp) s += std::conj(bra[cp]) * t[cp];
          out[size_t(ap) * cl + a] += o * s;
        }
      }
  return out;
}
inline Cplx closeEnv(const cmat& E, const cmat& R) {  // sum E[c'][c] R[c'][c]
  Cplx s = 0;
  for (size_t i = 0; i < E.size(); ++i) s += E[i] * R[i];
  return s;
}

// all left / right environments with identity operators: Lenv[b] (bond b,
// b = 0..L), Renv[b] (bond b, from the right)
struct Envs {
  std::vector<cmat> Lenv, Renv;
};
inline Envs envs(const Dense& D) {
  Envs V;
  const std::vector<double> I = identityOp(D.p);
  V.Lenv.assign(D.L + 1, cmat());
  V.Renv.assign(D.L + 1, cmat());
  V.Lenv[0] = cmat(size_t(D.chi[0]) * D.chi[0], Cplx(1, 0));
  for (int k = 1; k <= D.L; ++k) V.Lenv[k] = leftStep(D, k, V.Lenv[k - 1], I);
  V.Renv[D.L] = cmat(size_t(D.chi[D.L]) * D.chi[D.L], Cplx(1, 0));
  for (int k = D.L; k >= 1; --k) V.Renv[k - 1] = rightStep(D, k, V.Renv[k], I);
  return V;
}

// eigenvalues (and vectors, columns of V) of a Hermitian n x n matrix by
// cyclic complex Jacobi
inline std::vector<double> heev(cmat A, int n, cmat* V = nullptr) {
  cmat Z(size_t(n) * n, Cplx(0, 0));
  for (int i = 0; i < n; ++i) Z[size_t(i) * n + i] = 1.0;
  auto a = [&](int i, int j) -> Cplx& { return A[size_t(i) * n + j]; };
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0, tot = 0;
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) (i == j ? tot : off) += std::norm(a(i, j));
    if (off <= 1e-30 * (tot + off) || off == 0) break;
    for (int p = 0; p < n - 1; ++p)
      for (int q = p + 1; q < n; ++q) {
        const Cplx apq = a(p, q);
        const double g = std::abs(apq);
        if (g == 0) continue;
        const double app = a(p, p).real(), aqq = a(q, q).real();
        const double th = 0.5 * std::atan2(2 * g, aqq - app);
        const double c = std::cos(th), s = std::sin(th);
        const Cplx ph = apq / g;  // rotation in the (p, q) plane with phase
        // columns: A <- A G, G = [[c, s ph], [-s conj(ph), c]] applied as unitary similarity
        for (int k = 0; k < n; ++k) {
          const Cplx akp = a(k, p), akq = a(k, q);
          a(k, p) = c * akp - s * std::conj(ph) * akq;
          a(k, q) = s * ph * akp + c * akq;
        }
        for (int k = 0; k < n; ++k) {
          const Cplx apk = a(p, k), aqk = a(q, k);
          a(p, k) = c * apk - s * ph * aqk;
          a(q, k) = s * std::conj(ph) * apk + c * aqk;
        }
        for (int k = 0; k < n; ++k) {
          const Cplx zkp = Z[size_t(k) * n + p], zkq = Z[size_t(k) * n + q];
          Z[size_t(k) * n + p] = c * zkp - s * std::conj(ph) * zkq;
          Z[size_t(k) * n + q] = s * ph * zkp + c * zkq;
        }
      }
  }
  std::vector<double> w(n);
  for (int i = 0; i < n; ++i) w[i] = a(i, i).real();
  if (V) *V = Z;
  return w;
}

inline cmat block(const cmat& M, int ld, int o, int n) {
  cmat B(size_t(n) * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) B[size_t(i) * n + j] = M[size_t(o + i) * ld + o + j];
  return B;
}

}  // namespace obs

inline Cplx expectationValue(const BoseHubbard& sites, const MPS& psi, const std::string& opname, int i) {
  if (i < 1 || i > psi.L) throw std::invalid_argument("expectationValue: site out of range");
  const obs::Dense D = obs::dense(psi);
  const obs::Envs V = obs::envs(D);
  return obs::closeEnv(obs::leftStep(D, i, V.Lenv[i - 1], obs::siteOp(opname, sites.localDim())), V.Renv[i]);
}

inline std::vector<Cplx> expectationValues(const BoseHubbard& sites, const MPS& psi, const std::string& opname) {
  const obs::Dense D = obs::dense(psi);
  const obs::Envs V = obs::envs(D);
  const std::vector<double> O = obs::siteOp(opname, sites.localDim());
  std::vector<Cplx> out;
  for (int i = 1; i <= psi.L; ++i) out.push_back(obs::closeEnv(obs::leftStep(D, i, V.Lenv[i - 1], O), V.Renv[i]));
  return out;
}

namespace obs {
inline Cplx correlation(const Dense& D, const Envs& V, const std::vector<double>& O1, int i,
                        const std::vector<double>& O2, int j) {
  if (i == j) {
    const Cplx v = closeEnv(leftStep(D, i, V.Lenv[i - 1], opProduct(O1, O2, D.p)), V.Renv[i]);
    return Cplx(v.real(), 0.0);  // (bra*ket).real() (:21)
  }
  const std::vector<double>& Oa = i < j ? O1 : O2;
  const std::vector<double>& Ob = i < j ? O2 : O1;
  const int a = std::min(i, j), b = std::max(i, j);
  const std::vector<double> I = identityOp(D.p);
  cmat C = leftStep(D, a, V.Lenv[a - 1], Oa);
  for (int k = a + 1; k < b; ++k) C = leftStep(D, k, C, I);
  return closeEnv(leftStep(D, b, C, Ob), V.Renv[b]);
}
}  // namespace obs

inline Cplx correlationFunction(const BoseHubbard& sites, const MPS& psi, const std::string& opname1, int i,
                                const std::string& opname2, int j) {
  if (i < 1 || i > psi.L || j < 1 || j > psi.L) throw std::invalid_argument("correlationFunction: site out of range");
  const obs::Dense D = obs::dense(psi);
  const obs::Envs V = obs::envs(D);
  const int p = sites.localDim();
  return obs::correlation(D, V, obs::siteOp(opname1, p), i, obs::siteOp(opname2, p), j);
}

// rho[i][j] (i, j = 0..N-1 for sites 1..N), rho[j][i] = conj(rho[i][j])
inline std::vector<std::vector<Cplx>> correlationMatrix(const BoseHubbard& sites, const MPS& psi,
                                                        const std::string& opname1, const std::string& opname2) {
  const obs::Dense D = obs::dense(psi);
  const obs::Envs V = obs::envs(D);
  const int p = sites.localDim(), N = psi.L;
  const std::vector<double> O1 = obs::siteOp(opname1, p), O2 = obs::siteOp(opname2, p);
  std::vector<std::vector<Cplx>> rho(N, std::vector<Cplx>(N, Cplx(0, 0)));
  for (int i = 1; i <= N; ++i) {
    rho[i - 1][i - 1] = obs::correlation(D, V, O1, i, O2, i);
    for (int j = i + 1; j <= N; ++j) {
      const Cplx c = obs::correlation(D, V, O1, i, O2, j);
      rho[i - 1][j - 1] = c;
      rho[j - 1][i - 1] = std::conj(c);
    }
  }
  return rho;
}

// largest eigenvalue of the correlation matrix (diagHermitian, Maxm 1; :80-98)
inline double correlationTerm(const BoseHubbard& sites, const MPS& psi, const std::string& opname1,
                              const std::string& opname2) {
  const auto rho = correlationMatrix(sites, psi, opname1, opname2);
  const int N = int(rho.size());
  obs::cmat A(size_t(N) * N);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) A[size_t(i) * N + j] = rho[i][j];
  const std::vector<double> w = obs::heev(A, N);
  return *std::max_element(w.begin(), w.end());
}

// S_b = -sum p ln p over the Schmidt weights of bond b = 1..N-1 (weights
// normalised to the state's norm, p > 1e-12 kept; :120-149)
inline std::vector<double> entanglementEntropy(const BoseHubbard& /*sites*/, const MPS& psi) {
  const obs::Dense D = obs::dense(psi);
  const obs::Envs V = obs::envs(D);
  std::vector<double> S;
  for (int b = 1; b < psi.L; ++b) {
    const int chi = D.chi[b];
    std::vector<double> wts;
    for (int q = 0; q <= psi.Q; ++q) {
      const int o = D.off[b][q], n = D.off[b][q + 1] - o;
      if (n == 0) continue;
      // weights = eig(L^1/2 R^T L^1/2) of the sector block (L, R Hermitian PSD)
      obs::cmat Vl;
      const std::vector<double> lam = obs::heev(obs::block(V.Lenv[b], chi, o, n), n, &Vl);
      const obs::cmat Rb = obs::block(V.Renv[b], chi, o, n);
      obs::cmat Sm(size_t(n) * n);  // S = V diag(sqrt(lam))
      for (int i = 0; i < n; ++i)
        for (int k = 0; k < n; ++k) Sm[size_t(i) * n + k] = Vl[size_t(i) * n + k] * std::sqrt(std::max(lam[k], 0.0));
      obs::cmat X(size_t(n) * n, Cplx(0, 0));  // X = S^H conj(R) S
      for (int x = 0; x < n; ++x)
        for (int y = 0; y < n; ++y) {
          Cplx s = 0;
          for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j)
              s += std::conj(Sm[size_t(i) * n + x]) * std::conj(Rb[size_t(i) * n + j]) * Sm[size_t(j) * n + y];
          X[size_t(x) * n + y] = s;
        }
      for (double w : obs::heev(X, n)) wts.push_back(w);
    }
    double tot = 0;
    for (double w : wts) tot += std::max(w, 0.0);
    double s = 0;
    for (double w : wts) {
      const double pw = tot > 0 ? w / tot : 0.0;
      if (pw > 1e-12) s += -pw * std::log(pw);
    }
    S.push_back(s);
  }
  return S;
}

}  // namespace ocmps
