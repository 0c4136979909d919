// Host-side construction of the engine's parameter block (pure C++, no HIP):
// gate tables, per-sector Schmidt-rank bounds and LDS/slot capacities.
#pragma once

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstring>
#include <string>
#include <vector>

#include "engine.hpp"

namespace ocg_host {

// # configurations of m sites (0..p-1 bosons each) holding q bosons, saturating
inline long long hs_count(int m, int p, int q) {
  if (q < 0) return 0;
  std::vector<long long> a(q + 1, 0);
  a[0] = 1;
  for (int s = 0; s < m; ++s) {
    std::vector<long long> b(q + 1, 0);
    for (int x = 0; x <= q; ++x) {
      if (!a[x]) continue;
      for (int n = 0; n < p && x + n <= q; ++n) b[x + n] = std::min<long long>(b[x + n] + a[x], 1LL << 40);
    }
    a.swap(b);
  }
  return a[q];
}

// exp(-i tau h), h = -J (a_1 a^dag_2 + a^dag_1 a_2) on (n1, n2) (p^2 x p^2,
// row = out index n1'*p+n2'), summed by Horner like ITensor's
// BondGate(tReal) Taylor series (reference src/BH_tDMRG.cpp:31-36), 60 orders.
// imag: exp(-tau h) instead (ITensor's BondGate(tImag); ground-state preparation).
inline std::vector<std::complex<double>> hopping_gate(int p, double J, double tau, bool imag = false) {
  int D = p * p;
  std::vector<std::complex<double>> x(size_t(D) * D, 0.0), G(size_t(D) * D, 0.0), T(size_t(D) * D);
  for (int n1 = 0; n1 < p; ++n1)
    for (int n2 = 0; n2 < p; ++n2) {
      int in = n1 * p + n2;
      if (n1 >= 1 && n2 + 1 < p) x[size_t((n1 - 1) * p + n2 + 1) * D + in] += -J * std::sqrt(double(n1) * (n2 + 1));
      if (n2 >= 1 && n1 + 1 < p) x[size_t((n1 + 1) * p + n2 - 1) * D + in] += -J * std::sqrt(double(n1 + 1) * n2);
    }
  for (auto& v : x) v *= imag ? std::complex<double>(-tau, 0) : std::complex<double>(0, -tau);
  for (int i = 0; i < D; ++i) G[size_t(i) * D + i] = 1.0;
  for (int ord = 60; ord >= 1; --ord) {
    for (int i = 0; i < D; ++i)
      for (int j = 0; j < D; ++j) {
        std::complex<double> s = 0;
        for (int k = 0; k < D; ++k) s += x[size_t(i) * D + k] * G[size_t(k) * D + j];
        T[size_t(i) * D + j] = s / double(ord) + (i == j ? 1.0 : 0.0);
      }
    G.swap(T);
  }
  return G;
}

// per-Δ (= n1 + n2) blocks of the forward/backward gates; fills P.glo/gsz/goff/gtotal
inline void gate_tables(OcgParams& P, double J, std::vector<double>& gf, std::vector<double>& gb) {
  const int p = P.p;
  auto Gf = hopping_gate(p, J, P.dt, P.imag != 0), Gb = hopping_gate(p, J, -P.dt, P.imag != 0);
  gf.clear();
  gb.clear();
  int off = 0;
  for (int D = 0; D <= 2 * (p - 1); ++D) {
    int lo = std::max(0, D - (p - 1)), hi = std::min(p - 1, D);
    int sz = hi - lo + 1;
    P.glo[D] = lo;
    P.gsz[D] = sz;
    P.goff[D] = off;
    for (int y = 0; y < sz; ++y)
      for (int x = 0; x < sz; ++x) {
        int a1 = lo + y, a2 = D - a1, n1 = lo + x, n2 = D - n1;
        size_t idx = size_t(a1 * p + a2) * p * p + (n1 * p + n2);
        gf.push_back(Gf[idx].real()); gf.push_back(Gf[idx].imag());
        gb.push_back(Gb[idx].real()); gb.push_back(Gb[idx].imag());
      }
    off += sz * sz;
  }
  P.gtotal = off;
}

// Per-sector Schmidt-rank bounds for the HBM engine (no LDS capacity
// limits): md[b][q] = min(HS_left, HS_right), mdz[b][q] = min(HS_left,
// 2 min(HS_left, HS_right)) (inside the dH zip-up), clamped to 2^30.
inline void rank_bounds(int L, int p, int npart, std::vector<int>& md, std::vector<int>& mdz) {
  const int Q1 = npart + 1;
  md.assign(size_t(L + 1) * Q1, 0);
  mdz.assign(size_t(L + 1) * Q1, 0);
  for (int b = 0; b <= L; ++b)
    for (int q = 0; q < Q1; ++q) {
      const long long a = hs_count(b, p, q), r = hs_count(L - b, p, npart - q);
      md[size_t(b) * Q1 + q] = int(std::min<long long>(std::min(a, r), 1LL << 30));
      mdz[size_t(b) * Q1 + q] = int(std::min<long long>(std::min(a, 2 * std::min(a, r)), 1LL << 30));
    }
}

// gate order of initJGates (src/BH_tDMRG.cpp:18-58): even bonds ascending, odd descending
inline std::vector<int> gate_order(int L) {
  std::vector<int> g;
  for (int i = 1; i < L; i += 2) g.push_back(i);
  const int offset = (L % 2 == 0) ? 2 : 1;
  for (int i = L - offset; i >= 1; i -= 2) g.push_back(i);
  return g;
}

// Decompositions one step performs: one per gate plus the gauge moves of
// MPS::position between gates (the centre walk of doStep,
// src/BH_tDMRG.cpp:173-218, as Chain::step runs it).
inline int step_gauge_moves(const OcgParams& P) {
  int centre = 1, moves = 0;
  for (int g = 0; g < P.ngates; ++g) {
    const int i1 = P.gate_i1[g], i2 = i1 + 1;
    const bool more = g + 1 < P.ngates;
    const int ni1 = more ? P.gate_i1[g + 1] : 0, ni2 = ni1 + 1;
    const bool fromleft = more && ni1 >= i2;
    centre = fromleft ? i2 : i1;
    const int target = !more ? 1 : (fromleft ? ni1 : ni2);
    moves += centre > target ? centre - target : target - centre;
  }
  return moves;
}

// Fills everything in P except lds_bytes and the gate tables.  md receives
// the per-sector rank bound min(HS_left(b,q), HS_right(L-b,Q-q)).  Maxm is
// deliberately not folded in: it caps the TOTAL bond dimension of a gate
// decomposition only (decompose applies it), while the initial/target
// states may carry larger bonds and the gauge moves (ITensor position, no
// Maxm) must keep them.
// Returns an empty string on success, else the error.
inline std::string build_params(OcgParams& P, std::vector<int>& mdv, int L, int p, int npart, double tstep,
                                double cutoff, int maxm) {
  std::memset(&P, 0, sizeof(P));
  if (L < 2 || L > OCG_MAXL) return "L must be in [2, " + std::to_string(OCG_MAXL) + "]";
  if (p < 2 || p > OCG_MAXP) return "p must be in [2, " + std::to_string(OCG_MAXP) + "]";
  if (npart < 0 || npart + 1 > OCG_MAXQ1 || npart > L * (p - 1)) return "bad particle number";
  if (!(tstep == tstep) || !(cutoff >= 0)) return "bad tstep / cutoff";
  P.L = L; P.p = p; P.Q = npart; P.Q1 = npart + 1;
  P.nsq = (L + 1) * P.Q1;
  P.dt = tstep;
  P.cutoff = cutoff;
  P.maxm = maxm > 0 ? maxm : 5000;  // ITensor v2 MAX_M
  for (int n = 0; n < p; ++n) P.dH[n] = 0.5 * n * (n - 1);
  // gate order (initJGates, src/BH_tDMRG.cpp:18-58): even bonds ascending, odd descending
  int g = 0;
  for (int i = 1; i < L; i += 2) P.gate_i1[g++] = i;
  int offset = (L % 2 == 0) ? 2 : 1;
  for (int i = L - offset; i >= 1; i -= 2) P.gate_i1[g++] = i;
  P.ngates = g;
  const int Q1 = P.Q1;
  // mdv[0 .. nsq)     : physical bound min(HS_left(b,q), HS_right(L-b,Q-q))
  // mdv[nsq .. 2 nsq) : bound inside the dH zip-up, whose bonds also carry the
  //                     MPO index: min(HS_left, 2 min(HS_left, HS_right))
  mdv.assign(2 * P.nsq, 0);
  for (int b = 0; b <= L; ++b)
    for (int q = 0; q < Q1; ++q) {
      long long a = hs_count(b, p, q), r = hs_count(L - b, p, P.Q - q);
      mdv[b * Q1 + q] = int(std::min(a, r));
      mdv[P.nsq + b * Q1 + q] = int(std::min<long long>(a, 2 * std::min(a, r)));
    }
  // capacities cover both the physical and the zip-up bond dimensions
  auto md = [&](int b, int q) {
    return (q < 0 || q > P.Q) ? 0 : std::max(mdv[b * Q1 + q], mdv[P.nsq + b * Q1 + q]);
  };
  long long cap = 0, maxsite = 0;
  for (int k = 1; k <= L; ++k) {
    long long s = 0;
    for (int q = 0; q < Q1; ++q)
      for (int n = 0; n < p && q + n <= P.Q; ++n) s += (long long)md(k - 1, q) * md(k, q + n);
    s = std::max<long long>(s, 1);
    P.site_base[k] = int(cap);
    P.site_cap[k] = int(s);
    cap += s;
    maxsite = std::max(maxsite, s);
  }
  long long th = 2 * maxsite, ev = 0, ec = 0, th2 = 0;
  for (int i1 = 1; i1 < L; ++i1) {  // two-site Θ blocks
    long long t = 0, e = 0, t2 = 0;
    for (int q = 0; q < Q1; ++q) {
      long long R = 0, C = 0, R2 = 0, C2 = 0;
      for (int n = 0; n < p; ++n) {
        R += md(i1 - 1, q - n); C += md(i1 + 1, q + n);
        if (q - n >= 0) R2 += mdv[(i1 - 1) * Q1 + q - n];
        if (q + n <= P.Q) C2 += mdv[(i1 + 1) * Q1 + q + n];
      }
      t += R * C;
      t2 += R2 * C2;
      e += std::min(R, C);
    }
    th = std::max(th, t);
    th2 = std::max(th2, t2);
    ev = std::max(ev, e);
  }
  for (int k = 1; k <= L; ++k) {  // single-site and dH zip-up matricisations
    long long e1 = 0, e2 = 0, e3 = 0;
    for (int q = 0; q < Q1; ++q) {
      long long Rl = 0, Cr = 0;
      for (int n = 0; n < p; ++n) { Rl += md(k - 1, q - n); Cr += md(k, q + n); }
      e1 += std::min(Rl, (long long)md(k, q));
      e2 += std::min((long long)md(k - 1, q), Cr);
      e3 += std::min(Rl, 2LL * md(k, q));
    }
    ev = std::max(ev, std::max(e1, std::max(e2, e3)));
  }
  for (int b = 0; b <= L; ++b) {  // overlap environments
    long long e = 0;
    for (int q = 0; q < Q1; ++q) e += (long long)md(b, q) * md(b, q);
    ec = std::max(ec, e);
  }
  th = std::max(th, ec);
  if (cap > (1LL << 28) || th > (1LL << 28)) return "problem too large for the LDS chain engine";
  P.cap = int(cap);
  P.max_site_cap = int(maxsite);
  P.thcap = int(th);
  P.th2cap = int(std::min(th2, th));
  P.ecap = int(ec);
  P.evcap = int(std::max<long long>(ev, 2)) + 2;
  P.nrot = P.evcap + Q1;
  return "";
}

}  // namespace ocg_host
