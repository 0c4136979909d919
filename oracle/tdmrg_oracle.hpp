// ============================================================================
//  ORACLE — TEST INFRASTRUCTURE ONLY.
//
//  CPU restatement of the reference's gradient/Hessian inner loop
//  (fskovbo/OptimalControlMPS: BH_tDMRG + OptimalControl), written from
//  scratch in plain C++17 with U(1) ("Nb") block-sparse tensors, i.e. the
//  arithmetic ITensor v2's IQTensor/IQMPS performs for this path.
//
//  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
//  load this code, and only as the checker / the CPU baseline.  The product
//  path (optimalcontrolmps_amd/) never links or calls it.
//
//  Reference citations are path:line relative to the reference repository.
//  Parity pins: tests/test_oracle.py (fixtures, exact state-vector
//  cross-check, eigensolver, truncation rule) and tests/test_facade_cpu.py
//  (the reference tests restated: CostTests golden fidelities,
//  FD gradient/Hessian properties, sequencing semantics, exact state-vector
//  cross-check).  ITensor internals that no reference test pins (truncation
//  scale, gauge-move and exactApplyMPO compression rules) are fixed here
//  explicitly and documented in DESIGN.md §Oracle ("parity unpinned" rows).
// ============================================================================
#pragma once

#include <algorithm>
#include <atomic>
#include <cassert>
#include <cmath>
#include <complex>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <mutex>
#include <numeric>
#include <stdexcept>
#include <thread>
#include <tuple>
#include <vector>

namespace oracle {

using cplx = std::complex<double>;

// ---------------------------------------------------------------------------
// Sector parallelism (CPU-baseline speed only).  The U(1) blocks of one
// decomposition / Theta build / gauge move are independent: with a budget of
// T > 1 threads on the calling thread they are dealt over T threads, largest
// first.  Every block is computed by one thread with the same loops, so the
// results are bit-identical to T = 1 (tests/test_oracle.py).  The budget is per
// thread (default 1, or ORC_SECTOR_THREADS); workers run with a budget of 1.
// ---------------------------------------------------------------------------
inline int& sector_threads() {
  static thread_local int t = [] {
    const char* e = std::getenv("ORC_SECTOR_THREADS");
    return e ? std::max(1, std::atoi(e)) : 1;
  }();
  return t;
}
// f(q) for every q in [0, n) with cost[q] > 0, largest cost first
template <class F>
inline void par_sectors(int n, const std::vector<double>& cost, F f) {
  std::vector<int> order;
  for (int q = 0; q < n; ++q)
    if (cost[q] > 0) order.push_back(q);
  const int T = std::min<int>(sector_threads(), int(order.size()));
  if (T <= 1) {
    for (int q : order) f(q);
    return;
  }
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cost[a] > cost[b]; });
  std::atomic<size_t> next(0);
  auto work = [&]() {
    sector_threads() = 1;
    for (size_t i; (i = next.fetch_add(1)) < order.size();) f(order[i]);
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < T; ++t) pool.emplace_back(work);
  const int mine = sector_threads();
  work();
  sector_threads() = mine;
  for (auto& th : pool) th.join();
}

// ---------------------------------------------------------------------------
// Dense helpers
// ---------------------------------------------------------------------------
struct Blk {
  int r = 0, c = 0;
  std::vector<cplx> v;
  Blk() = default;
  Blk(int r_, int c_) : r(r_), c(c_), v(size_t(r_) * c_, cplx(0, 0)) {}
  cplx& at(int i, int j) { return v[size_t(i) * c + j]; }
  const cplx& at(int i, int j) const { return v[size_t(i) * c + j]; }
  bool empty() const { return r == 0 || c == 0; }
};

// Cyclic complex Jacobi eigen-solver for a Hermitian n x n matrix (row-major).
// Returns eigenvalues descending and eigenvectors as columns of V.
// (Stands in for the LAPACK zheev ITensor's diagHermitian calls per QN block.)
inline void heev_jacobi(int n, std::vector<cplx> A, std::vector<double>& w,
                        std::vector<cplx>& V) {
  V.assign(size_t(n) * n, cplx(0, 0));
  for (int i = 0; i < n; ++i) V[size_t(i) * n + i] = 1.0;
  auto a = [&](int i, int j) -> cplx& { return A[size_t(i) * n + j]; };
  double scale = 0;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) scale += std::norm(a(i, j));
  for (int sweep = 0; sweep < 100 && n > 1; ++sweep) {
    double off = 0;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q) off += std::norm(a(p, q));
    if (off <= 1e-32 * scale || off == 0.0) break;
    for (int p = 0; p < n; ++p) {
      for (int q = p + 1; q < n; ++q) {
        cplx b = a(p, q);
        double ab = std::abs(b);
        if (ab == 0.0) continue;
        double app = a(p, p).real(), aqq = a(q, q).real();
        double tau = (aqq - app) / (2.0 * ab);
        double t = (tau >= 0 ? 1.0 : -1.0) / (std::fabs(tau) + std::sqrt(1.0 + tau * tau));
        double c = 1.0 / std::sqrt(1.0 + t * t), s = t * c;
        cplx e = b / ab;             // e^{i phi}
        cplx ec = std::conj(e);      // e^{-i phi}
        // V2 = [[c, s], [-s e^{-i phi}, c e^{-i phi}]];  A <- V2^H A V2
        for (int k = 0; k < n; ++k) {  // columns
          cplx akp = a(k, p), akq = a(k, q);
          a(k, p) = c * akp - s * ec * akq;
          a(k, q) = s * akp + c * ec * akq;
        }
        for (int k = 0; k < n; ++k) {  // rows
          cplx apk = a(p, k), aqk = a(q, k);
          a(p, k) = c * apk - s * e * aqk;
          a(q, k) = s * apk + c * e * aqk;
        }
        a(p, q) = 0; a(q, p) = 0;
        a(p, p) = app - t * ab;
        a(q, q) = aqq + t * ab;
        for (int k = 0; k < n; ++k) {
          cplx vkp = V[size_t(k) * n + p], vkq = V[size_t(k) * n + q];
          V[size_t(k) * n + p] = c * vkp - s * ec * vkq;
          V[size_t(k) * n + q] = s * vkp + c * ec * vkq;
        }
      }
    }
  }
  std::vector<int> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(),
                   [&](int x, int y) { return a(x, x).real() > a(y, y).real(); });
  w.resize(n);
  std::vector<cplx> Vs(size_t(n) * n);
  for (int j = 0; j < n; ++j) {
    w[j] = a(idx[j], idx[j]).real();
    for (int k = 0; k < n; ++k) Vs[size_t(k) * n + j] = V[size_t(k) * n + idx[j]];
  }
  V.swap(Vs);
}

// Householder + implicit QL eigen-solver for a Hermitian n x n matrix
// (row-major): the algorithm of LAPACK's zheev, which ITensor's diagHermitian
// calls per QN block.  A = Q T Q^H with T real symmetric tridiagonal (the
// complex subdiagonal made real by a diagonal phase matrix D), T = Z diag(w) Z^T
// by QL sweeps with implicit Wilkinson shifts, eigenvectors Q D Z.  O(n^3) with
// small constants: the cyclic Jacobi above needs ~50x longer at n ~ 500.
// Eigenvalues descending, eigenvectors as columns of V (gauge differs from
// heev_jacobi's; every quantity the oracle reports is gauge invariant).
inline void heev_ql(int n, std::vector<cplx> A, std::vector<double>& w, std::vector<cplx>& V) {
  w.assign(n, 0.0);
  V.assign(size_t(n) * n, cplx(0, 0));
  if (n == 0) return;
  auto a = [&](int i, int j) -> cplx& { return A[size_t(i) * n + j]; };
  // Q accumulated explicitly (columns = orthonormal basis of the tridiagonal form)
  std::vector<cplx> Q(size_t(n) * n, cplx(0, 0));
  for (int i = 0; i < n; ++i) Q[size_t(i) * n + i] = 1.0;
  std::vector<cplx> sub(n, cplx(0, 0)), v(n), pv(n), wv(n);
  for (int k = 0; k + 2 < n; ++k) {
    // x = A[k+1.., k] -> beta e_1 with H = I - tau v v^H, v_0 = x_0 + e^{i arg x_0} ||x||
    double xn2 = 0;
    for (int i = k + 1; i < n; ++i) xn2 += std::norm(a(i, k));
    const double xn = std::sqrt(xn2);
    const cplx x0 = a(k + 1, k);
    const double ax0 = std::abs(x0);
    if (xn == 0.0) { sub[k] = 0.0; continue; }
    const cplx ph = ax0 > 0 ? x0 / ax0 : cplx(1, 0);
    for (int i = k + 1; i < n; ++i) v[i] = a(i, k);
    v[k + 1] = x0 + ph * xn;
    const double tau = 1.0 / (xn * (xn + ax0));
    sub[k] = -ph * xn;
    // p = tau A v (trailing block), K = tau/2 v^H p, w = p - K v, A -= v w^H + w v^H
    for (int i = k + 1; i < n; ++i) {
      cplx acc = 0;
      for (int j = k + 1; j < n; ++j) acc += a(i, j) * v[j];
      pv[i] = tau * acc;
    }
    cplx K = 0;
    for (int i = k + 1; i < n; ++i) K += std::conj(v[i]) * pv[i];
    K *= 0.5 * tau;
    for (int i = k + 1; i < n; ++i) wv[i] = pv[i] - K * v[i];
    for (int i = k + 1; i < n; ++i)
      for (int j = k + 1; j < n; ++j) a(i, j) -= v[i] * std::conj(wv[j]) + wv[i] * std::conj(v[j]);
    // Q <- Q H (H Hermitian, unitary)
    for (int r = 0; r < n; ++r) {
      cplx acc = 0;
      for (int j = k + 1; j < n; ++j) acc += Q[size_t(r) * n + j] * v[j];
      acc *= tau;
      for (int j = k + 1; j < n; ++j) Q[size_t(r) * n + j] -= acc * std::conj(v[j]);
    }
  }
  if (n >= 2) sub[n - 2] = a(n - 1, n - 2);
  // real tridiagonal: d = diag, e = |sub|, D = diag(phases) with T_c = D T_r D^H
  std::vector<double> d(n), e(n, 0.0);
  std::vector<cplx> dph(n, cplx(1, 0));
  for (int i = 0; i < n; ++i) d[i] = a(i, i).real();
  for (int i = 0; i + 1 < n; ++i) {
    const double ab = std::abs(sub[i]);
    e[i] = ab;
    dph[i + 1] = ab > 0 ? dph[i] * (sub[i] / ab) : dph[i];
  }
  // implicit QL with Wilkinson shifts; Z (row-major n x n) accumulates the rotations
  std::vector<double> Z(size_t(n) * n, 0.0);
  for (int i = 0; i < n; ++i) Z[size_t(i) * n + i] = 1.0;
  const double eps = std::numeric_limits<double>::epsilon();
  double tnorm = 0;
  for (int i = 0; i < n; ++i) tnorm = std::max(tnorm, std::fabs(d[i]) + e[i] + (i ? e[i - 1] : 0.0));
  // deflation: |e_m| negligible next to its diagonal neighbours, or below
  // eps ||T||: zheev's absolute accuracy (eigenvalues to ~eps ||A||), which the
  // truncation (relative cutoffs >= 1e-14 of the total weight) never resolves
  // below; without it graded blocks with tiny trailing eigenvalues stagnate
  const double floor_abs = eps * tnorm;
  for (int l = 0; l < n; ++l) {
    int iter = 0, m;
    for (;;) {
      for (m = l; m + 1 < n; ++m) {
        const double dd = std::fabs(d[m]) + std::fabs(d[m + 1]);
        if (std::fabs(e[m]) <= eps * dd || std::fabs(e[m]) <= floor_abs) break;
      }
      if (m == l) break;
      if (++iter > 300) throw std::runtime_error("heev_ql: no convergence");
      double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
      double r = std::hypot(g, 1.0);
      g = d[m] - d[l] + e[l] / (g + (g >= 0 ? r : -r));
      double s = 1.0, c = 1.0, p = 0.0;
      int i;
      bool deflate = false;
      for (i = m - 1; i >= l; --i) {
        double f = s * e[i];
        const double b = c * e[i];
        r = std::hypot(f, g);
        e[i + 1] = r;
        if (r == 0.0) {
          d[i + 1] -= p;
          e[m] = 0.0;
          deflate = true;
          break;
        }
        s = f / r;
        c = g / r;
        g = d[i + 1] - p;
        r = (d[i] - g) * s + 2.0 * c * b;
        p = s * r;
        d[i + 1] = g + p;
        g = c * r - b;
        for (int k = 0; k < n; ++k) {
          f = Z[size_t(k) * n + i + 1];
          Z[size_t(k) * n + i + 1] = s * Z[size_t(k) * n + i] + c * f;
          Z[size_t(k) * n + i] = c * Z[size_t(k) * n + i] - s * f;
        }
      }
      if (deflate) continue;
      d[l] -= p;
      e[l] = g;
      e[m] = 0.0;
    }
  }
  // descending order; V = Q D Z
  std::vector<int> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](int x, int y) { return d[x] > d[y]; });
  for (int j = 0; j < n; ++j) {
    w[j] = d[idx[j]];
    for (int r = 0; r < n; ++r) {
      cplx acc = 0;
      for (int t = 0; t < n; ++t) acc += Q[size_t(r) * n + t] * dph[t] * Z[size_t(t) * n + idx[j]];
      V[size_t(r) * n + j] = acc;
    }
  }
}

// the per-block eigensolver of denmatDecomp: cyclic Jacobi (default, the
// committed fixtures' solver) or, with ORC_HEEV=ql in the environment, the
// Householder + QL solver (large fixtures: chi = 256 / 512 steps in minutes)
inline bool heev_use_ql() {
  static const bool q = [] {
    const char* e = std::getenv("ORC_HEEV");
    return e && e[0] == 'q';
  }();
  return q;
}
inline void heev(int n, std::vector<cplx> A, std::vector<double>& w, std::vector<cplx>& V) {
  if (heev_use_ql()) {
    try {
      heev_ql(n, A, w, V);
      return;
    } catch (const std::runtime_error&) {  // a block QL cannot deflate: the Jacobi solver takes it
      std::fprintf(stderr, "[oracle] heev_ql did not converge on a block of order %d; cyclic Jacobi instead\n", n);
    }
  }
  heev_jacobi(n, std::move(A), w, V);
}

// ---------------------------------------------------------------------------
// Truncation rule (ITensor v2 `truncate` as used by denmatDecomp; the scale of
// the cutoff is fixed here as relative to the total weight — parity unpinned).
//   P: eigenvalues sorted descending.  Returns the number kept.
// ---------------------------------------------------------------------------
inline int truncate_count(std::vector<double> P, double cutoff, int maxm, int minm = 1) {
  int n = int(P.size());
  if (n == 0) return 0;
  double total = 0;
  for (auto& x : P) { if (x < 0) x = 0; total += x; }
  if (total <= 0) return std::min(std::max(minm, 1), n);
  int last = n - 1;
  double trunc = 0;
  while (last >= maxm) { trunc += P[last]; --last; }
  while (last >= minm && trunc + P[last] < cutoff * total) { trunc += P[last]; --last; }
  return last + 1;
}

// ---------------------------------------------------------------------------
// MPS with U(1) particle-number blocks.
//   Sites k = 1..L (stored at A[k-1]); bond b = 0..L sits between sites b, b+1.
//   Bond b has dims[b][q] states with left particle count q (q = 0..Q).
//   Site k block (q, n): rows dims[k-1][q], cols dims[k][q+n] (QN flow q + n).
//   Canonical form carried by this code: right-orthonormal with the
//   orthogonality centre at site 1 (the reference's psi.position(1) at the end
//   of every doStep, src/BH_tDMRG.cpp:217).
// ---------------------------------------------------------------------------
struct MPS {
  int L = 0, p = 0, Q = 0;
  std::vector<std::vector<int>> dims;      // [L+1][Q+1]
  std::vector<std::vector<Blk>> A;         // [L][(Q+1)*p]

  int d(int b, int q) const { return (q < 0 || q > Q) ? 0 : dims[b][q]; }
  Blk& blk(int k, int q, int n) { return A[k - 1][size_t(q) * p + n]; }
  const Blk& blk(int k, int q, int n) const { return A[k - 1][size_t(q) * p + n]; }

  void init_shape(int L_, int p_, int Q_) {
    L = L_; p = p_; Q = Q_;
    dims.assign(L + 1, std::vector<int>(Q + 1, 0));
    A.assign(L, std::vector<Blk>(size_t(Q + 1) * p));
  }
  // (re)allocate the blocks of site k from the current dims (zeros).
  void alloc_site(int k) {
    for (int q = 0; q <= Q; ++q)
      for (int n = 0; n < p; ++n) {
        int r = d(k - 1, q), c = (q + n <= Q) ? d(k, q + n) : 0;
        blk(k, q, n) = (r > 0 && c > 0) ? Blk(r, c) : Blk();
      }
  }
  int bond_dim(int b) const { int s = 0; for (int q = 0; q <= Q; ++q) s += dims[b][q]; return s; }

  // compact interchange format (shared with the C-ABI of the product):
  // for k=1..L, q=0..Q, n=0..p-1: block rows x cols row-major, complex interleaved.
  size_t nelem() const {
    size_t s = 0;
    for (int k = 1; k <= L; ++k)
      for (int q = 0; q <= Q; ++q)
        for (int n = 0; n < p && q + n <= Q; ++n) s += size_t(d(k - 1, q)) * d(k, q + n);
    return s;
  }
  void to_flat(std::vector<int>& fd, std::vector<double>& data) const {
    fd.clear();
    for (int b = 0; b <= L; ++b)
      for (int q = 0; q <= Q; ++q) fd.push_back(dims[b][q]);
    data.clear();
    for (int k = 1; k <= L; ++k)
      for (int q = 0; q <= Q; ++q)
        for (int n = 0; n < p && q + n <= Q; ++n) {
          const Blk& B = blk(k, q, n);
          for (auto& z : B.v) { data.push_back(z.real()); data.push_back(z.imag()); }
        }
  }
  static MPS from_flat(int L, int p, int Q, const int* fd, const double* data) {
    MPS m;
    m.init_shape(L, p, Q);
    for (int b = 0; b <= L; ++b)
      for (int q = 0; q <= Q; ++q) m.dims[b][q] = fd[b * (Q + 1) + q];
    size_t off = 0;
    for (int k = 1; k <= L; ++k) {
      m.alloc_site(k);
      for (int q = 0; q <= Q; ++q)
        for (int n = 0; n < p && q + n <= Q; ++n) {
          Blk& B = m.blk(k, q, n);
          for (auto& z : B.v) { z = cplx(data[2 * off], data[2 * off + 1]); ++off; }
        }
    }
    return m;
  }
};

// ---------------------------------------------------------------------------
// Block matrix grouped by a QN q:  block q is R_q x C_q; rows are segments of
// (n_row, q_row_bond) and cols segments of (n_col, q_col_bond).
// ---------------------------------------------------------------------------
struct QMat {
  int Q = 0, p = 0;
  std::vector<Blk> blk;                        // [Q+1]
  std::vector<std::vector<int>> rowoff, coloff;  // [Q+1][p]  (-1 = absent)
};

enum Dir { Fromleft, Fromright };

struct Decomp {  // result of a block decomposition M = X * Y
  std::vector<int> kept;       // [Q+1] new bond dims
  std::vector<Blk> X, Y;       // per q: X: R_q x k_q, Y: k_q x C_q
};

// Block denmatDecomp with truncation (ITensor denmatDecomp/diagHermitian per
// QN block, global sort, `truncate`).  Fromleft: X orthonormal columns
// (eigenvectors of M M^H), Y = X^H M.  Fromright: Y orthonormal rows
// (eigenvectors of M^H M, conjugated), X = M Y^H.
inline Decomp decompose(const QMat& M, Dir dir, double cutoff, int maxm) {
  int Q = M.Q;
  std::vector<std::vector<double>> w(Q + 1);
  std::vector<std::vector<cplx>> V(Q + 1);
  struct Ev { double lam; int q, i; };
  std::vector<Ev> all;
  std::vector<double> cost(Q + 1, 0.0);
  for (int q = 0; q <= Q; ++q) {
    const Blk& B = M.blk[q];
    if (B.empty()) continue;
    const double n = (dir == Fromleft) ? B.r : B.c;
    cost[q] = n * n * (n + double(B.r) * B.c / n);
  }
  par_sectors(Q + 1, cost, [&](int q) {
    const Blk& B = M.blk[q];
    int n = (dir == Fromleft) ? B.r : B.c;
    std::vector<cplx> rho(size_t(n) * n, cplx(0, 0));
    if (dir == Fromleft) {
      for (int i = 0; i < B.r; ++i)
        for (int j = 0; j < B.r; ++j) {
          cplx s = 0;
          for (int k = 0; k < B.c; ++k) s += B.at(i, k) * std::conj(B.at(j, k));
          rho[size_t(i) * n + j] = s;
        }
    } else {
      for (int i = 0; i < B.c; ++i)
        for (int j = 0; j < B.c; ++j) {
          cplx s = 0;
          for (int k = 0; k < B.r; ++k) s += std::conj(B.at(k, i)) * B.at(k, j);
          rho[size_t(i) * n + j] = s;
        }
    }
    heev(n, rho, w[q], V[q]);
  });
  for (int q = 0; q <= Q; ++q)
    for (int i = 0; i < int(w[q].size()); ++i) all.push_back({w[q][i], q, i});
  std::stable_sort(all.begin(), all.end(), [](const Ev& a, const Ev& b) {
    if (a.lam != b.lam) return a.lam > b.lam;
    if (a.q != b.q) return a.q < b.q;
    return a.i < b.i;
  });
  std::vector<double> P;
  for (auto& e : all) P.push_back(e.lam);
  int m = truncate_count(P, cutoff, maxm, 1);
  Decomp D;
  D.kept.assign(Q + 1, 0);
  for (int j = 0; j < m; ++j) D.kept[all[j].q]++;  // per block the top-k (block-sorted)
  D.X.assign(Q + 1, Blk());
  D.Y.assign(Q + 1, Blk());
  std::vector<double> fcost(Q + 1, 0.0);
  for (int q = 0; q <= Q; ++q) fcost[q] = double(D.kept[q]) * M.blk[q].r * M.blk[q].c;
  par_sectors(Q + 1, fcost, [&](int q) {
    int k = D.kept[q];
    const Blk& B = M.blk[q];
    if (dir == Fromleft) {
      int n = B.r;
      Blk X(B.r, k), Y(k, B.c);
      for (int i = 0; i < B.r; ++i)
        for (int j = 0; j < k; ++j) X.at(i, j) = V[q][size_t(i) * n + j];
      for (int j = 0; j < k; ++j)
        for (int c = 0; c < B.c; ++c) {
          cplx s = 0;
          for (int i = 0; i < B.r; ++i) s += std::conj(X.at(i, j)) * B.at(i, c);
          Y.at(j, c) = s;
        }
      D.X[q] = std::move(X); D.Y[q] = std::move(Y);
    } else {
      int n = B.c;
      Blk X(B.r, k), Y(k, B.c);
      for (int j = 0; j < k; ++j)
        for (int c = 0; c < B.c; ++c) Y.at(j, c) = std::conj(V[q][size_t(c) * n + j]);
      for (int i = 0; i < B.r; ++i)
        for (int j = 0; j < k; ++j) {
          cplx s = 0;
          for (int c = 0; c < B.c; ++c) s += B.at(i, c) * V[q][size_t(c) * n + j];
          X.at(i, j) = s;
        }
      D.X[q] = std::move(X); D.Y[q] = std::move(Y);
    }
  });
  return D;
}

// Truncation used by gauge moves (ITensor MPS::position) and by the
// left-to-right half of exactApplyMPO's orthogonalisation.  Parity unpinned:
// fixed here as a relative discarded-weight cutoff of 1e-14, no Maxm.
constexpr double kGaugeCutoff = 1e-14;
constexpr int kNoMaxm = 1 << 30;

// ---------------------------------------------------------------------------
// Single-site matricisations of A_k and their write-back.
// ---------------------------------------------------------------------------
// Fromleft grouping: rows (n, a) with qn(a)+n = q, cols c with qn(c) = q.
inline QMat site_as_left(const MPS& m, int k) {
  QMat M; M.Q = m.Q; M.p = m.p;
  M.blk.assign(m.Q + 1, Blk());
  M.rowoff.assign(m.Q + 1, std::vector<int>(m.p, -1));
  M.coloff.assign(m.Q + 1, std::vector<int>(1, -1));
  for (int q = 0; q <= m.Q; ++q) {
    int C = m.d(k, q), R = 0;
    for (int n = 0; n < m.p; ++n) { int ql = q - n; if (m.d(k - 1, ql) > 0) { M.rowoff[q][n] = R; R += m.d(k - 1, ql); } }
    if (R == 0 || C == 0) continue;
    M.coloff[q][0] = 0;
    Blk B(R, C);
    for (int n = 0; n < m.p; ++n) {
      int ql = q - n; if (M.rowoff[q][n] < 0) continue;
      const Blk& S = m.blk(k, ql, n);
      for (int i = 0; i < S.r; ++i)
        for (int j = 0; j < S.c; ++j) B.at(M.rowoff[q][n] + i, j) = S.at(i, j);
    }
    M.blk[q] = std::move(B);
  }
  return M;
}
// Fromright grouping: rows a with qn(a)=q, cols (n, c) with qn(c) = q+n.
inline QMat site_as_right(const MPS& m, int k) {
  QMat M; M.Q = m.Q; M.p = m.p;
  M.blk.assign(m.Q + 1, Blk());
  M.rowoff.assign(m.Q + 1, std::vector<int>(1, -1));
  M.coloff.assign(m.Q + 1, std::vector<int>(m.p, -1));
  for (int q = 0; q <= m.Q; ++q) {
    int R = m.d(k - 1, q), C = 0;
    for (int n = 0; n < m.p; ++n) { int qr = q + n; if (qr <= m.Q && m.d(k, qr) > 0) { M.coloff[q][n] = C; C += m.d(k, qr); } }
    if (R == 0 || C == 0) continue;
    M.rowoff[q][0] = 0;
    Blk B(R, C);
    for (int n = 0; n < m.p; ++n) {
      if (M.coloff[q][n] < 0) continue;
      const Blk& S = m.blk(k, q, n);
      for (int i = 0; i < S.r; ++i)
        for (int j = 0; j < S.c; ++j) B.at(i, M.coloff[q][n] + j) = S.at(i, j);
    }
    M.blk[q] = std::move(B);
  }
  return M;
}

// Move the orthogonality centre one site right (k -> k+1) or left (k -> k-1).
inline void gauge_right(MPS& m, int k) {
  QMat M = site_as_left(m, k);
  Decomp D = decompose(M, Fromleft, kGaugeCutoff, kNoMaxm);
  // new A_k from X
  std::vector<int> old = m.dims[k];
  for (int q = 0; q <= m.Q; ++q) m.dims[k][q] = D.kept[q];
  m.alloc_site(k);
  for (int q = 0; q <= m.Q; ++q) {
    if (D.kept[q] == 0) continue;
    for (int n = 0; n < m.p; ++n) {
      int ql = q - n; if (M.rowoff[q][n] < 0) continue;
      Blk& S = m.blk(k, ql, n);
      for (int i = 0; i < S.r; ++i)
        for (int j = 0; j < S.c; ++j) S.at(i, j) = D.X[q].at(M.rowoff[q][n] + i, j);
    }
  }
  // A_{k+1} <- Y * A_{k+1}
  std::vector<Blk> nb(size_t(m.Q + 1) * m.p);
  std::vector<double> cost(m.Q + 1, 0.0);
  for (int q = 0; q <= m.Q; ++q) cost[q] = double(D.kept[q]) * m.d(k, q) * (m.d(k + 1, q) + 1);
  par_sectors(m.Q + 1, cost, [&](int q) {
    for (int n = 0; n < m.p && q + n <= m.Q; ++n) {
      const Blk& S = m.blk(k + 1, q, n);
      int kq = D.kept[q];
      if (S.empty() || kq == 0) continue;
      Blk T(kq, S.c);
      for (int i = 0; i < kq; ++i)
        for (int j = 0; j < S.c; ++j) {
          cplx s = 0;
          for (int b = 0; b < S.r; ++b) s += D.Y[q].at(i, b) * S.at(b, j);
          T.at(i, j) = s;
        }
      nb[size_t(q) * m.p + n] = std::move(T);
    }
  });
  (void)old;
  m.A[k] = std::move(nb);  // site k+1
}

inline void gauge_left(MPS& m, int k) {
  QMat M = site_as_right(m, k);
  Decomp D = decompose(M, Fromright, kGaugeCutoff, kNoMaxm);
  for (int q = 0; q <= m.Q; ++q) m.dims[k - 1][q] = D.kept[q];
  m.alloc_site(k);
  for (int q = 0; q <= m.Q; ++q) {
    if (D.kept[q] == 0) continue;
    for (int n = 0; n < m.p; ++n) {
      if (M.coloff[q][n] < 0) continue;
      Blk& S = m.blk(k, q, n);
      for (int i = 0; i < S.r; ++i)
        for (int j = 0; j < S.c; ++j) S.at(i, j) = D.Y[q].at(i, M.coloff[q][n] + j);
    }
  }
  // A_{k-1} <- A_{k-1} * X
  std::vector<Blk> nb(size_t(m.Q + 1) * m.p);
  std::vector<double> cost(m.Q + 1, 0.0);
  for (int ql = 0; ql <= m.Q; ++ql) cost[ql] = double(m.d(k - 2, ql) + 1) * m.p * 64.0;
  par_sectors(m.Q + 1, cost, [&](int ql) {
    for (int n = 0; n < m.p && ql + n <= m.Q; ++n) {
      const Blk& S = m.blk(k - 1, ql, n);
      int q = ql + n, kq = D.kept[q];
      if (S.empty() || kq == 0) continue;
      Blk T(S.r, kq);
      for (int i = 0; i < S.r; ++i)
        for (int j = 0; j < kq; ++j) {
          cplx s = 0;
          for (int b = 0; b < S.c; ++b) s += S.at(i, b) * D.X[q].at(b, j);
          T.at(i, j) = s;
        }
      nb[size_t(ql) * m.p + n] = std::move(T);
    }
  });
  m.A[k - 2] = std::move(nb);
}

inline double site_norm(const MPS& m, int k) {
  double s = 0;
  for (auto& b : m.A[k - 1]) for (auto& z : b.v) s += std::norm(z);
  return std::sqrt(s);
}
inline void site_scale(MPS& m, int k, double f) {
  for (auto& b : m.A[k - 1]) for (auto& z : b.v) z *= f;
}

// ---------------------------------------------------------------------------
// Overlaps  <X|Y> (conj on X; ITensor overlapC) and <X|D_k...|Y>.
// ---------------------------------------------------------------------------
inline std::vector<Blk> transfer(const MPS& X, const MPS& Y, int k, const std::vector<Blk>& E,
                                 const double* diag /* nullable, length p */) {
  int Q = X.Q, p = X.p;
  std::vector<Blk> En(Q + 1);
  for (int q = 0; q <= Q; ++q) {
    int rx = X.d(k, q), ry = Y.d(k, q);
    if (rx > 0 && ry > 0) En[q] = Blk(rx, ry);
  }
  for (int q = 0; q <= Q; ++q) {
    const Blk& Eq = E[q];
    if (Eq.empty()) continue;
    for (int n = 0; n < p && q + n <= Q; ++n) {
      const Blk& Xb = X.blk(k, q, n);
      const Blk& Yb = Y.blk(k, q, n);
      if (Xb.empty() || Yb.empty()) continue;
      double f = diag ? diag[n] : 1.0;
      if (f == 0.0) continue;
      // T = E * Yb  (rx_old x cy)
      Blk T(Eq.r, Yb.c);
      for (int i = 0; i < Eq.r; ++i)
        for (int b = 0; b < Eq.c; ++b) {
          cplx e = Eq.at(i, b);
          if (e == cplx(0, 0)) continue;
          for (int j = 0; j < Yb.c; ++j) T.at(i, j) += e * Yb.at(b, j);
        }
      Blk& O = En[q + n];
      for (int a = 0; a < Xb.c; ++a)
        for (int i = 0; i < Xb.r; ++i) {
          cplx x = std::conj(Xb.at(i, a)) * f;
          for (int j = 0; j < Yb.c; ++j) O.at(a, j) += x * T.at(i, j);
        }
    }
  }
  return En;
}

inline cplx overlapC(const MPS& X, const MPS& Y) {
  std::vector<Blk> E(X.Q + 1);
  E[0] = Blk(1, 1); E[0].at(0, 0) = 1.0;
  for (int k = 1; k <= X.L; ++k) E = transfer(X, Y, k, E, nullptr);
  return E[X.Q].empty() ? cplx(0, 0) : E[X.Q].at(0, 0);
}

// <X| sum_k D_k |Y>, D = diag(d) on every site (MPO of bond dimension 2).
inline cplx overlapC_diag(const MPS& X, const std::vector<double>& d, const MPS& Y) {
  std::vector<Blk> E0(X.Q + 1), E1(X.Q + 1);
  E0[0] = Blk(1, 1); E0[0].at(0, 0) = 1.0;
  for (int k = 1; k <= X.L; ++k) {
    auto a = transfer(X, Y, k, E1, nullptr);
    auto b = transfer(X, Y, k, E0, d.data());
    for (int q = 0; q <= X.Q; ++q)
      for (size_t i = 0; i < a[q].v.size(); ++i) a[q].v[i] += b[q].v[i];
    E1 = std::move(a);
    E0 = transfer(X, Y, k, E0, nullptr);
  }
  return E1[X.Q].empty() ? cplx(0, 0) : E1[X.Q].at(0, 0);
}

inline double norm(const MPS& X) { return std::sqrt(std::max(0.0, overlapC(X, X).real())); }

// ---------------------------------------------------------------------------
// The Bose-Hubbard site operators (include/BH_sites.h:114-176) and the
// two-site hopping gate exp(-i tau h), h = -J (a a^dag + a^dag a)
// (src/BH_tDMRG.cpp:28-57), exponentiated by a Taylor series like ITensor's
// BondGate(tReal).  "Id" in BH_sites.h omits |0><0|; the exact exponential is
// used.
// ---------------------------------------------------------------------------
inline std::vector<cplx> hopping_gate(int p, double J, double tau) {
  int D = p * p;
  std::vector<cplx> h(size_t(D) * D, 0.0);
  auto idx = [&](int n1, int n2) { return n1 * p + n2; };
  for (int n1 = 0; n1 < p; ++n1)
    for (int n2 = 0; n2 < p; ++n2) {
      // a_1 a^dag_2 |n1,n2> = sqrt(n1) sqrt(n2+1) |n1-1, n2+1>
      if (n1 >= 1 && n2 + 1 < p)
        h[size_t(idx(n1 - 1, n2 + 1)) * D + idx(n1, n2)] += -J * std::sqrt(double(n1)) * std::sqrt(double(n2 + 1));
      if (n2 >= 1 && n1 + 1 < p)
        h[size_t(idx(n1 + 1, n2 - 1)) * D + idx(n1, n2)] += -J * std::sqrt(double(n1 + 1)) * std::sqrt(double(n2));
    }
  // x = -i tau h ; G = sum_k x^k / k!  (Horner, 60 orders)
  std::vector<cplx> x(h.size());
  for (size_t i = 0; i < h.size(); ++i) x[i] = cplx(0, -tau) * h[i];
  std::vector<cplx> G(size_t(D) * D, 0.0), T(size_t(D) * D);
  for (int i = 0; i < D; ++i) G[size_t(i) * D + i] = 1.0;
  for (int ord = 60; ord >= 1; --ord) {
    // G <- I + (x G)/ord
    for (int i = 0; i < D; ++i)
      for (int j = 0; j < D; ++j) {
        cplx s = 0;
        for (int k = 0; k < D; ++k) s += x[size_t(i) * D + k] * G[size_t(k) * D + j];
        T[size_t(i) * D + j] = s / double(ord) + (i == j ? 1.0 : 0.0);
      }
    G.swap(T);
  }
  return G;
}

// ---------------------------------------------------------------------------
// Bose-Hubbard tDMRG stepper: restatement of BH_tDMRG (src/BH_tDMRG.cpp).
// ---------------------------------------------------------------------------
struct Stepper {
  int L, p, Q;
  double J, dt, cutoff;
  int maxm;
  std::vector<std::pair<int, int>> gates;   // (i1, i2), 1-based
  std::vector<cplx> Gf, Gb;                 // forward / backward gate (p^2 x p^2)
  std::vector<double> dH;                   // 0.5 n(n-1)  (propagatorDeriv, src/BH_tDMRG.cpp:10-14)

  Stepper(int L_, int p_, int Q_, double J_, double dt_, double cutoff_, int maxm_ = 5000)
      : L(L_), p(p_), Q(Q_), J(J_), dt(dt_), cutoff(cutoff_), maxm(maxm_) {
    // initJGates (src/BH_tDMRG.cpp:18-58): even bonds ascending, odd bonds descending
    for (int i = 1; i < L; i += 2) gates.push_back({i, i + 1});
    int offset = (L % 2 == 0) ? 2 : 1;
    for (int i = L - offset; i >= 1; i -= 2) gates.push_back({i, i + 1});
    Gf = hopping_gate(p, J, dt);
    Gb = hopping_gate(p, J, -dt);
    dH.resize(p);
    for (int n = 0; n < p; ++n) dH[n] = 0.5 * n * (n - 1);
  }

  // U-gate phases (src/BH_tDMRG.cpp:74-108): exp(-i 0.25 u tau n(n-1)); the
  // backward step negates u (src/BH_tDMRG.cpp:122), equivalently tau -> -dt.
  std::vector<cplx> uphase(double u, double tau) const {
    std::vector<cplx> ph(p);
    for (int n = 0; n < p; ++n) ph[n] = std::exp(cplx(0, -0.25 * u * tau * n * (n - 1)));
    return ph;
  }

  // Θ for bond (i1, i2), grouped by the middle QN q: rows (n1, a), cols (n2, c).
  QMat build_theta(const MPS& m, int i1) const {
    int l = i1 - 1, mid = i1, r = i1 + 1;
    QMat T; T.Q = Q; T.p = p;
    T.blk.assign(Q + 1, Blk());
    T.rowoff.assign(Q + 1, std::vector<int>(p, -1));
    T.coloff.assign(Q + 1, std::vector<int>(p, -1));
    std::vector<double> cost(Q + 1, 0.0);
    for (int q = 0; q <= Q; ++q) {
      int R = 0, C = 0;
      for (int n1 = 0; n1 < p; ++n1) if (m.d(l, q - n1) > 0) { T.rowoff[q][n1] = R; R += m.d(l, q - n1); }
      for (int n2 = 0; n2 < p; ++n2) if (q + n2 <= Q && m.d(r, q + n2) > 0) { T.coloff[q][n2] = C; C += m.d(r, q + n2); }
      if (R > 0 && C > 0) cost[q] = double(R) * C * (m.d(mid, q) + 1);
    }
    par_sectors(Q + 1, cost, [&](int q) {
      int R = 0, C = 0;
      for (int n1 = 0; n1 < p; ++n1) if (T.rowoff[q][n1] >= 0) R += m.d(l, q - n1);
      for (int n2 = 0; n2 < p; ++n2) if (T.coloff[q][n2] >= 0) C += m.d(r, q + n2);
      Blk B(R, C);
      if (m.d(mid, q) > 0) {
        for (int n1 = 0; n1 < p; ++n1) {
          if (T.rowoff[q][n1] < 0) continue;
          const Blk& X = m.blk(i1, q - n1, n1);
          for (int n2 = 0; n2 < p; ++n2) {
            if (T.coloff[q][n2] < 0) continue;
            const Blk& Y = m.blk(r, q, n2);
            for (int i = 0; i < X.r; ++i)
              for (int j = 0; j < Y.c; ++j) {
                cplx s = 0;
                for (int b = 0; b < X.c; ++b) s += X.at(i, b) * Y.at(b, j);
                B.at(T.rowoff[q][n1] + i, T.coloff[q][n2] + j) = s;
              }
          }
        }
      }
      T.blk[q] = std::move(B);
    });
    return T;
  }

  // apply pre-phase -> J gate -> post-phase on every (a, c) Δ-vector
  void apply_gate(QMat& T, const MPS& m, int i1, const std::vector<cplx>& G,
                  const std::vector<cplx>& pre1, const std::vector<cplx>& pre2,
                  const std::vector<cplx>& post1, const std::vector<cplx>& post2) const {
    int l = i1 - 1, r = i1 + 1;
    std::vector<double> cost(Q + 1, 0.0);
    for (int ql = 0; ql <= Q; ++ql)
      for (int qr = ql; qr <= Q; ++qr) cost[ql] += double(m.d(l, ql)) * m.d(r, qr);
    par_sectors(Q + 1, cost, [&](int ql) {
      std::vector<cplx> v(p), w(p);
      for (int ia = 0; ia < m.d(l, ql); ++ia)
        for (int qr = ql; qr <= Q; ++qr)
          for (int ic = 0; ic < m.d(r, qr); ++ic) {
            int Dl = qr - ql;
            int lo = std::max(0, Dl - (p - 1)), hi = std::min(p - 1, Dl);
            if (lo > hi) continue;
            for (int n1 = lo; n1 <= hi; ++n1) {
              int n2 = Dl - n1, q = ql + n1;
              v[n1] = T.blk[q].at(T.rowoff[q][n1] + ia, T.coloff[q][n2] + ic) * pre1[n1] * pre2[n2];
            }
            for (int a1 = lo; a1 <= hi; ++a1) {
              int a2 = Dl - a1;
              cplx s = 0;
              for (int n1 = lo; n1 <= hi; ++n1) s += G[size_t(a1 * p + a2) * p * p + (n1 * p + (Dl - n1))] * v[n1];
              w[a1] = s * post1[a1] * post2[a2];
            }
            for (int n1 = lo; n1 <= hi; ++n1) {
              int n2 = Dl - n1, q = ql + n1;
              T.blk[q].at(T.rowoff[q][n1] + ia, T.coloff[q][n2] + ic) = w[n1];
            }
          }
    });
  }

  // write a decomposition of Θ back into sites i1, i2 (new middle bond)
  void write_back(MPS& m, int i1, const QMat& T, const Decomp& D) const {
    int r = i1 + 1;
    for (int q = 0; q <= Q; ++q) m.dims[i1][q] = D.kept[q];
    m.alloc_site(i1);
    m.alloc_site(r);
    for (int q = 0; q <= Q; ++q) {
      if (D.kept[q] == 0) continue;
      for (int n1 = 0; n1 < p; ++n1) {
        if (T.rowoff[q][n1] < 0) continue;
        Blk& S = m.blk(i1, q - n1, n1);
        for (int i = 0; i < S.r; ++i)
          for (int j = 0; j < S.c; ++j) S.at(i, j) = D.X[q].at(T.rowoff[q][n1] + i, j);
      }
      for (int n2 = 0; n2 < p; ++n2) {
        if (T.coloff[q][n2] < 0) continue;
        Blk& S = m.blk(r, q, n2);
        for (int i = 0; i < S.r; ++i)
          for (int j = 0; j < S.c; ++j) S.at(i, j) = D.Y[q].at(i, T.coloff[q][n2] + j);
      }
    }
  }

  void position(MPS& m, int& centre, int target) const {
    while (centre < target) { gauge_right(m, centre); ++centre; }
    while (centre > target) { gauge_left(m, centre); --centre; }
  }

  // BH_tDMRG::step + doStep (src/BH_tDMRG.cpp:111-230)
  void step(MPS& psi, double from, double to, bool forward = true) const {
    double tau = forward ? dt : -dt;
    const auto& G = forward ? Gf : Gb;
    auto UF = uphase(from, tau), UT = uphase(to, tau);
    std::vector<cplx> one(p, 1.0);
    int centre = 1;
    if (L % 2 != 0) {  // lonely U_from on site L first (:133-136)
      for (int q = 0; q <= Q; ++q)
        for (int n = 0; n < p; ++n) for (auto& z : psi.blk(L, q, n).v) z *= UF[n];
    }
    bool movingFromLeft = true;
    for (size_t g = 0; g < gates.size(); ++g) {
      int i1 = gates[g].first, i2 = gates[g].second;
      QMat T = build_theta(psi, i1);
      if (movingFromLeft) {
        bool lonely = (i2 == L && L % 2 == 0);  // (:153-155)
        apply_gate(T, psi, i1, G, UF, UF, one, lonely ? UT : one);
      } else {
        apply_gate(T, psi, i1, G, one, one, UT, UT);
      }
      if (g + 1 < gates.size()) {
        int ni1 = gates[g + 1].first, ni2 = gates[g + 1].second;
        if (ni1 >= i2) {
          Decomp D = decompose(T, Fromleft, cutoff, maxm);
          write_back(psi, i1, T, D);
          double nrm = site_norm(psi, i1 + 1);
          if (nrm > 1e-16) site_scale(psi, i1 + 1, 1.0 / nrm);
          centre = i1 + 1;
          position(psi, centre, ni1);
        }
        if (ni1 < i2) {
          Decomp D = decompose(T, Fromright, cutoff, maxm);
          write_back(psi, i1, T, D);
          double nrm = site_norm(psi, i1);
          if (nrm > 1e-16) site_scale(psi, i1, 1.0 / nrm);
          centre = i1;
          position(psi, centre, ni2);
        }
        if (i2 == ni1 || i1 == ni2) movingFromLeft = false;
      } else {
        Decomp D = decompose(T, Fromright, cutoff, maxm);
        write_back(psi, i1, T, D);
        double nrm = site_norm(psi, i1);
        if (nrm > 1e-16) site_scale(psi, i1, 1.0 / nrm);
        centre = i1;
        position(psi, centre, 1);
      }
    }
    for (int q = 0; q <= Q; ++q)  // lonely U_to on site 1 (:222-223)
      for (int n = 0; n < p; ++n) for (auto& z : psi.blk(1, q, n).v) z *= UT[n];
    double nrm = site_norm(psi, 1);  // psi.normalize() (:228)
    if (nrm > 0) site_scale(psi, 1, 1.0 / nrm);
  }

  // exactApplyMPO(propDeriv, psi, args) (src/OptimalControl.cpp:256, :302):
  // exact bond-doubled MPO x MPS, then orthogonalise left->right (gauge cutoff)
  // and truncate right->left with the stepper's Cutoff/Maxm.  Output is
  // right-orthonormal, centre site 1, unnormalised.
  MPS apply_dH(const MPS& psi) const {
    MPS phi;
    phi.init_shape(L, p, Q);
    // bond b of phi: (t, a), t=0 "not yet applied", t=1 "applied"; t-major within each q
    for (int b = 0; b <= L; ++b)
      for (int q = 0; q <= Q; ++q) {
        int d = psi.d(b, q);
        phi.dims[b][q] = (b == 0 || b == L) ? d : 2 * d;
      }
    for (int k = 1; k <= L; ++k) {
      phi.alloc_site(k);
      for (int q = 0; q <= Q; ++q)
        for (int n = 0; n < p && q + n <= Q; ++n) {
          const Blk& S = psi.blk(k, q, n);
          if (S.empty()) continue;
          Blk& O = phi.blk(k, q, n);
          int dl = S.r, dr = S.c;
          // s (row copy) x t (col copy) : (0,0)=1, (0,1)=d(n), (1,1)=1
          auto put = [&](int s, int t, double f) {
            bool lb = (k == 1), rb = (k == L);
            if (lb && s == 1) return;
            if (rb && t == 0) return;
            int ro = lb ? 0 : s * dl, co = rb ? 0 : t * dr;
            for (int i = 0; i < dl; ++i)
              for (int j = 0; j < dr; ++j) O.at(ro + i, co + j) += f * S.at(i, j);
          };
          put(0, 0, 1.0);
          put(0, 1, dH[n]);
          put(1, 1, 1.0);
        }
    }
    for (int k = 1; k < L; ++k) gauge_right(phi, k);
    for (int k = L; k > 1; --k) {
      QMat M = site_as_right(phi, k);
      Decomp D = decompose(M, Fromright, cutoff, maxm);
      for (int q = 0; q <= Q; ++q) phi.dims[k - 1][q] = D.kept[q];
      phi.alloc_site(k);
      for (int q = 0; q <= Q; ++q) {
        if (D.kept[q] == 0) continue;
        for (int n = 0; n < p; ++n) {
          if (M.coloff[q][n] < 0) continue;
          Blk& S = phi.blk(k, q, n);
          for (int i = 0; i < S.r; ++i)
            for (int j = 0; j < S.c; ++j) S.at(i, j) = D.Y[q].at(i, M.coloff[q][n] + j);
        }
      }
      std::vector<Blk> nb(size_t(Q + 1) * p);
      std::vector<double> cost(Q + 1, 0.0);
      for (int ql = 0; ql <= Q; ++ql) cost[ql] = double(phi.d(k - 2, ql) + 1) * p * 64.0;
      par_sectors(Q + 1, cost, [&](int ql) {
        for (int n = 0; n < p && ql + n <= Q; ++n) {
          const Blk& S = phi.blk(k - 1, ql, n);
          int q = ql + n, kq = D.kept[q];
          if (S.empty() || kq == 0) continue;
          Blk T(S.r, kq);
          for (int i = 0; i < S.r; ++i)
            for (int j = 0; j < kq; ++j) {
              cplx s = 0;
              for (int b = 0; b < S.c; ++b) s += S.at(i, b) * D.X[q].at(b, j);
              T.at(i, j) = s;
            }
          nb[size_t(ql) * p + n] = std::move(T);
        }
      });
      phi.A[k - 2] = std::move(nb);
    }
    return phi;
  }
};

// ---------------------------------------------------------------------------
// OptimalControl restatement (src/OptimalControl.cpp), GRAPE parameterisation.
// ---------------------------------------------------------------------------
struct OC {
  Stepper st;
  MPS target, init;
  size_t N;
  double gamma;
  std::vector<MPS> psi_t, xi_t, xiH;
  std::vector<cplx> divT;

  OC(const Stepper& s, const MPS& tgt, const MPS& ini, size_t N_, double gamma_)
      : st(s), target(tgt), init(ini), N(N_), gamma(gamma_) {}

  void calcPsi(const std::vector<double>& u) {  // :375-390
    psi_t.assign(N, MPS());
    MPS psi = init;
    psi_t[0] = psi;
    for (size_t i = 0; i + 1 < N; ++i) { st.step(psi, u[i], u[i + 1], true); psi_t[i + 1] = psi; }
  }
  void calcXi(const std::vector<double>& u) {  // :392-407
    xi_t.assign(N, MPS());
    MPS xi = target;
    xi_t[N - 1] = xi;
    for (size_t i = N - 1; i > 0; --i) { st.step(xi, u[i], u[i - 1], false); xi_t[i - 1] = xi; }
  }
  void calcDivT() {  // :409-419
    divT.assign(N, 0.0);
    for (size_t i = 0; i < N; ++i) divT[i] = overlapC_diag(xi_t[i], st.dH, psi_t[i]);
  }
  // BFGS path: xi propagated inline, divT filled backwards (:217-229)
  void calcDivT_bfgs(const std::vector<double>& u) {
    divT.assign(N, 0.0);
    MPS xi = target;
    divT[N - 1] = overlapC_diag(xi, st.dH, psi_t[N - 1]);
    for (size_t i = N - 1; i > 0; --i) {
      st.step(xi, u[i], u[i - 1], false);
      divT[i - 1] = overlapC_diag(xi, st.dH, psi_t[i - 1]);
    }
  }
  cplx overlapFactor() const { return overlapC(psi_t.back(), target); }

  double regularization(const std::vector<double>& u) const {  // :88-99
    double tmp = 0;
    for (size_t i = 0; i + 1 < N; ++i) { double d = u[i + 1] - u[i]; tmp += d * d / st.dt; }
    return gamma / 2.0 * tmp;
  }
  std::vector<double> regularizationGrad(const std::vector<double>& u) const {  // :102-121
    std::vector<double> del;
    double dt = st.dt;
    del.push_back(-gamma * (-5.0 * u[1] + 4.0 * u[2] - u[3] + 2.0 * u[0]) / dt);
    for (size_t i = 1; i + 1 < N; ++i) del.push_back(-gamma * (u[i + 1] + u[i - 1] - 2.0 * u[i]) / dt);
    del.push_back(-gamma * (-5.0 * u[N - 2] + 4.0 * u[N - 3] - u[N - 4] + 2.0 * u[N - 1]) / dt);
    return del;
  }
  double cost(const std::vector<double>& u) {  // :440-453 (new_control = true)
    calcPsi(u);
    cplx o = overlapC(target, psi_t.back());
    return 0.5 * (1.0 - std::norm(o)) + regularization(u);
  }
  std::vector<double> fidelities() const {  // :548-569
    std::vector<double> f;
    for (auto& s : psi_t) f.push_back(std::norm(overlapC(target, s)));
    return f;
  }
  std::vector<double> gradient(const std::vector<double>& u, bool bfgs) {  // :204-249, :456-467
    calcPsi(u);
    if (bfgs) calcDivT_bfgs(u);
    else { calcXi(u); calcDivT(); }
    cplx F = overlapFactor();
    auto R = regularizationGrad(u);
    std::vector<double> g(N);
    for (size_t i = 0; i < N; ++i) g[i] = st.dt * (divT[i] * F * cplx(0, 1)).real() + R[i];
    return g;
  }

  // calcHessianRow (:251-279): entries (i, j >= i); writes into H (no reg).
  void hessianRow(size_t i, const std::vector<double>& u, cplx F, std::vector<double>& H) const {
    MPS psiH = st.apply_dH(psi_t[i]);
    double normiH = norm(psiH);
    double dt2 = st.dt * st.dt;
    double v1 = (F * overlapC(xiH[i], psiH)).real();
    double v2 = -(divT[i] * std::conj(divT[i])).real();
    H[i * N + i] += dt2 * (v1 + v2);
    for (size_t j = i + 1; j + 1 < N; ++j) {
      st.step(psiH, u[j - 1], u[j], true);
      double a = (F * overlapC(xiH[j], psiH) * normiH).real();
      double b = -(divT[i] * std::conj(divT[j])).real();
      double r = dt2 * (a + b);
      H[i * N + j] += r;
      H[j * N + i] += r;
    }
  }

  // calcHessian_parallel / _sequencial (:281-372), row-major N x N.
  // threads > 1: psi and xi on two threads (calcPsiXiDivT, :424-430) and the
  // xiH list by the worker pool (the reference builds it serially, :300-303;
  // every entry is computed independently, so the result is the same).
  // nested != 0 (CPU baseline of the large configs): the threads also serve the
  // sector parallelism inside each step — psi and xi get threads / 2 each, the
  // row workers threads / workers each (same numbers bit for bit).
  int nested = 0;
  std::vector<double> hessian(const std::vector<double>& u, int threads) {
    const int outer = sector_threads();
    if (threads > 1) {
      const int half = nested ? std::max(1, threads / 2) : 1;
      std::thread tx([&]() { sector_threads() = half; calcXi(u); });
      sector_threads() = half;
      calcPsi(u);
      sector_threads() = outer;
      tx.join();
    } else {
      calcPsi(u);
      calcXi(u);
    }
    calcDivT();
    std::vector<double> H(N * N, 0.0);
    double g = gamma / st.dt;  // calcRegularizationHessian (:124-143)
    for (size_t i = 1; i + 1 < N; ++i) { H[i * N + i - 1] = -g; H[i * N + i + 1] = -g; H[i * N + i] = 2 * g; }
    H[1 * N + 0] = 0; H[(N - 2) * N + N - 1] = 0;
    cplx F = overlapFactor();
    xiH.assign(N, MPS());
    if (threads > 1) {
      std::atomic<size_t> next(0);
      std::vector<std::thread> pool;
      const int workers = nested ? std::min<int>(threads, int(N)) : threads;
      const int per = nested ? std::max(1, threads / std::max(1, workers)) : 1;
      for (int t = 0; t < workers; ++t)
        pool.emplace_back([&]() {
          sector_threads() = per;
          for (size_t i; (i = next.fetch_add(1)) < N;) xiH[i] = st.apply_dH(xi_t[i]);
        });
      for (auto& th : pool) th.join();
    } else {
      for (size_t i = 0; i < N; ++i) xiH[i] = st.apply_dH(xi_t[i]);
    }
    rows(u, F, H, threads);
    return H;
  }
  void rows(const std::vector<double>& u, cplx F, std::vector<double>& H, int threads) const {
    if (threads <= 1) {
      for (size_t i = 1; i + 1 < N; ++i) hessianRow(i, u, F, H);
      return;
    }
    // worker pool with a shared row counter (:306-335); rows write disjoint entries
    std::atomic<size_t> next(1);
    std::vector<std::thread> pool;
    const int workers = nested ? std::min<int>(threads, int(N) - 2) : threads;
    const int per = nested ? std::max(1, threads / std::max(1, workers)) : 1;
    for (int t = 0; t < workers; ++t)
      pool.emplace_back([&]() {
        sector_threads() = per;
        for (;;) {
          size_t i = next.fetch_add(1);
          if (i + 1 >= N) break;
          hessianRow(i, u, F, H);
        }
      });
    for (auto& th : pool) th.join();
  }
};

}  // namespace oracle
