// Host side of the one-wave padded chain (fast_chain.hpp): the step plan.
//
// Every bond sector is stored at its Schmidt-rank bound D[b][q] =
// min(HS_left, HS_right) (rank_bounds), zero-padded beyond the runtime
// dimension.  The block layout of every site, of every two-site Θ, of every
// single-site matricisation and of every factor is then the same at every
// step, whatever the truncation kept, so all index arithmetic of a step
// (BH_tDMRG::doStep, reference src/BH_tDMRG.cpp:127-230: the gates, the
// denmatDecomp of each, the MPS::position gauge moves between them, the
// closing move to site 1) is computed once here and read by the device as
// plain descriptor tables.  Zero padding is exact: a padded row or column
// contributes nothing to a contraction, a padded Gram index has a zero
// eigenvalue, which the truncation rule always discards, and the factors
// written for it are zeros again.
//
// Used when the chain fits the one-wave design's compile-time bounds
// (fast.hpp: Gram blocks of order <= 4, at most four of order >= 2 per
// decomposition, <= 64 eigenvalues, <= 128 Θ elements, <= 256 elements per
// site / factor list, 16-bit LDS offsets).  Config 1 (L=5, p=5, Npart=5)
// qualifies, and so do the small chains of the reference's tests.
#pragma once

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "engine.hpp"
#include "fast.hpp"

namespace ocg_host {

struct FastPlanBuild {
  std::vector<int> plan;   // the int image copied to the device (fast.hpp layout)
  std::string why_not;     // empty: usable
};

// md: the per-sector Schmidt-rank bound min(HS_left, HS_right) of every bond
// ((L+1) * Q1 ints; build_params' mdv)
inline FastPlanBuild build_fast_plan(const OcgParams& P, const std::vector<int>& md) {
  using namespace ocg::fastp;
  FastPlanBuild out;
  const int L = P.L, p = P.p, Q = P.Q, Q1 = P.Q1;
  auto fail = [&](const std::string& m) {
    out.plan.clear();
    out.why_not = m;
    return out;
  };
  if (P.imag) return fail("imaginary-time steps use the general engine");
  if (p > 6) return fail("local dimension above 6");
  if (Q1 > 64) return fail("more than 64 sectors");
  auto D = [&](int b, int q) { return (b < 0 || b > L || q < 0 || q > Q) ? 0 : md[size_t(b) * Q1 + q]; };
  for (int b = 0; b <= L; ++b)
    for (int q = 0; q <= Q; ++q)
      if (D(b, q) > kMaxDm) return fail("bond sector bound above the unrolled maximum");
  std::vector<int> I(kHdrInts, 0);  // header, filled at the end
  auto pad = [&]() {                // every table starts 16-byte aligned
    while (I.size() & 3) I.push_back(0);
    return int(I.size());
  };
  auto push4 = [&](int a, int b, int c, int d) { I.push_back(a); I.push_back(b); I.push_back(c); I.push_back(d); };
  // ---- padded MPS layout: site k, block (q, n) = D(k-1, q) x D(k, q+n), in the
  // compact (q, n) order
  std::vector<int> poff(size_t(L + 2) * Q1 * p, -1), sbase(L + 2, 0);
  int np = 0;
  std::vector<int> blk_k, blk_q, blk_n;
  for (int k = 1; k <= L; ++k) {
    sbase[k] = np;
    for (int q = 0; q <= Q; ++q)
      for (int n = 0; n < p && q + n <= Q; ++n) {
        const int dl = D(k - 1, q), dr = D(k, q + n);
        if (dl == 0 || dr == 0) continue;
        poff[(size_t(k) * Q1 + q) * p + n] = np;
        blk_k.push_back(k); blk_q.push_back(q); blk_n.push_back(n);
        np += dl * dr;
      }
  }
  sbase[L + 1] = np;
  if (np > 64 * kItMps) return fail("padded MPS above the unrolled maximum");
  auto PO = [&](int k, int q, int n) {
    return (k < 1 || k > L || q < 0 || q > Q || n < 0 || n >= p) ? -1 : poff[(size_t(k) * Q1 + q) * p + n];
  };
  const int nblk = int(blk_k.size());
  if (nblk > 4095) return fail("too many blocks");
  std::vector<int> first(nblk);
  for (int b = 0; b < nblk; ++b) {
    first[b] = b;
    while (first[b] > 0 && blk_k[first[b] - 1] == blk_k[b]) --first[b];
  }
  const int o_blk = pad();
  for (int b = 0; b < nblk; ++b) {
    const int k = blk_k[b], q = blk_q[b], n = blk_n[b];
    push4(k | (q << 8) | (n << 16), (k - 1) * Q1 + q, k * Q1 + q + n, first[b]);
  }
  const int o_ls = pad();
  for (int b = 0; b < nblk; ++b) {
    const int k = blk_k[b], q = blk_q[b], n = blk_n[b];
    for (int a = 0; a < D(k - 1, q); ++a)
      for (int c = 0; c < D(k, q + n); ++c)
        push4(((k - 1) * Q1 + q) | ((k * Q1 + q + n) << 16), b | (first[b] << 16), a | (c << 8), P.site_base[k]);
  }
  const int o_site = pad();
  for (int k = 0; k <= L + 1; ++k) I.push_back(sbase[k]);
  const int o_siten = pad();
  for (int b = 0; b < nblk; ++b)
    if (blk_k[b] == 1)
      for (int x = 0; x < D(0, blk_q[b]) * D(1, blk_q[b] + blk_n[b]); ++x) I.push_back(blk_n[b]);

  // ---- step ops (doStep's sequence as Chain::step runs it)
  struct Op { int kind, k, dir, mode, lonely, closing; };
  std::vector<Op> ops;
  {
    int centre = 1;
    bool mfl = true;
    for (int g = 0; g < P.ngates; ++g) {
      const int i1 = P.gate_i1[g], i2 = i1 + 1;
      const bool more = g + 1 < P.ngates;
      const int ni1 = more ? P.gate_i1[g + 1] : 0, ni2 = ni1 + 1;
      const int dir = (more && ni1 >= i2) ? 0 : 1;
      Op o{kOpGate, i1, dir, mfl ? 0 : 1, 0, 0};
      if (mfl) o.lonely = (i2 == L && L % 2 == 0) ? 1 : 0;
      else o.lonely = (L % 2 != 0 && i2 == L) ? 2 : 0;
      ops.push_back(o);
      centre = dir == 0 ? i2 : i1;
      const int target = !more ? 1 : (dir == 0 ? ni1 : ni2);
      while (centre != target) {
        if (centre < target) { ops.push_back({kOpGaugeR, centre, 0, 0, 0, more ? 0 : 1}); ++centre; }
        else { ops.push_back({kOpGaugeL, centre, 1, 0, 0, more ? 0 : 1}); --centre; }
      }
      if (more && (i2 == ni1 || i1 == ni2)) mfl = false;
    }
  }
  if (int(ops.size()) > kMaxOps) return fail("too many step operations");
  int thmax = 1, xsmax = 1, last_gate = 0;
  std::vector<int> op_off;
  for (const Op& o : ops) {
    if (o.kind == kOpGate) last_gate = o.k;
    // matricisation M: sector q has rows (nr, a in bond bl sector q - nr) for nr in
    // the row physical range, cols (nc, c in bond br sector q + nc)
    int bl, br, prow, pcol;  // prow / pcol: number of physical indices on the side (1 or p)
    if (o.kind == kOpGate) { bl = o.k - 1; br = o.k + 1; prow = p; pcol = p; }
    else if (o.kind == kOpGaugeR) { bl = o.k - 1; br = o.k; prow = p; pcol = 1; }
    else { bl = o.k - 1; br = o.k; prow = 1; pcol = p; }
    const int newb = (o.kind == kOpGaugeL) ? o.k - 1 : o.k;  // the bond the decomposition rewrites
    std::vector<int> R(Q1, 0), C(Q1, 0), THO(Q1 + 1, 0);
    std::vector<std::vector<int>> RS(Q1, std::vector<int>(p, -1)), CS(Q1, std::vector<int>(p, -1));
    for (int q = 0; q <= Q; ++q) {
      for (int n = 0; n < prow; ++n) {
        const int d = D(bl, q - n);
        if (d > 0) { RS[q][n] = R[q]; R[q] += d; }
      }
      for (int n = 0; n < pcol; ++n) {
        const int d = D(br, q + n);
        if (d > 0) { CS[q][n] = C[q]; C[q] += d; }
      }
      if (R[q] == 0 || C[q] == 0) { R[q] = 0; C[q] = 0; }
      THO[q + 1] = THO[q] + R[q] * C[q];
    }
    const int nth = THO[Q1];
    thmax = std::max(thmax, nth);
    if (nth > 64 * kItTh) return fail("matricisation above the unrolled maximum");
    const int hpos = pad();
    op_off.push_back(hpos);
    I.resize(I.size() + kOpHdr, 0);
    auto setH = [&](int f, int v) { I[hpos + f] = v; };
    setH(kOhKind, o.kind); setH(kOhK, o.k); setH(kOhDir, o.dir); setH(kOhMode, o.mode);
    setH(kOhLonely, o.lonely); setH(kOhClosing, o.closing); setH(kOhNth, nth); setH(kOhNewBond, newb);
    // -- M's elements (TH order: sector-major, rows (nr, a), cols (nc, c))
    setH(kOhMat, pad());
    for (int q = 0; q <= Q; ++q) {
      if (R[q] == 0) continue;
      for (int nr = 0; nr < prow; ++nr) {
        if (RS[q][nr] < 0) continue;
        for (int a = 0; a < D(bl, q - nr); ++a)
          for (int nc = 0; nc < pcol; ++nc) {
            if (CS[q][nc] < 0) continue;
            for (int c = 0; c < D(br, q + nc); ++c) {
              if (o.kind == kOpGate) {  // Θ = sum_b A_i1[(q-nr, nr)][a][b] A_i2[(q, nc)][b][c]
                const int dm = D(o.k, q);
                const int x1 = dm > 0 ? PO(o.k, q - nr, nr) + a * dm : 0;
                const int drc = D(o.k + 1, q + nc);
                const int x2 = dm > 0 ? PO(o.k + 1, q, nc) + c : 0;
                I.push_back(x1 | (x2 << 16));
                I.push_back(dm | (drc << 8));
              } else if (o.kind == kOpGaugeR) {  // rows (n, a), col c: A_k[(q-n, n)][a][c]
                I.push_back(PO(o.k, q - nr, nr) + a * D(o.k, q) + c);
              } else {  // row a, cols (n, c): A_k[(q, n)][a][c]
                I.push_back(PO(o.k, q, nc) + a * D(o.k, q + nc) + c);
              }
            }
          }
      }
    }
    // -- gate descriptors (two-site only): output element of sector q, row (a1, a),
    // col (a2, c): int4 {gate row offset | sz << 16 | lo << 20 | a1 << 24 | a2 << 28,
    // then the sz <= 6 input TH offsets as 16-bit pairs}
    if (o.kind == kOpGate) {
      setH(kOhGate, pad());
      for (int q = 0; q <= Q; ++q) {
        if (R[q] == 0) continue;
        for (int a1 = 0; a1 < p; ++a1) {
          if (RS[q][a1] < 0) continue;
          const int ql = q - a1;
          for (int a = 0; a < D(bl, ql); ++a)
            for (int a2 = 0; a2 < p; ++a2) {
              if (CS[q][a2] < 0) continue;
              const int qr = q + a2;
              for (int c = 0; c < D(br, qr); ++c) {
                const int Dl = a1 + a2, lo = P.glo[Dl], sz = P.gsz[Dl];
                int w[4] = {(P.goff[Dl] + (a1 - lo) * sz) | (sz << 16) | (lo << 20) | (a1 << 24) | (a2 << 28), 0, 0, 0};
                for (int x = 0; x < sz; ++x) {
                  const int n1 = lo + x, n2 = Dl - n1, qs = ql + n1;
                  if (qs < 0 || qs > Q || RS[qs][n1] < 0 || CS[qs][n2] < 0 || R[qs] == 0)
                    return fail("internal: gate input outside Θ");
                  const int ad = THO[qs] + (RS[qs][n1] + a) * C[qs] + CS[qs][n2] + c;
                  if (ad > 65535) return fail("Θ offset above 16 bits");
                  w[1 + x / 2] |= ad << (16 * (x & 1));
                }
                push4(w[0], w[1], w[2], w[3]);
              }
            }
        }
      }
    }
    // -- decomposition sectors: order n = min(R, C), Gram on the smaller side
    std::vector<int> sq, secn(Q1, 0), seco(Q1, -1), secside(Q1, 0), secgrp(Q1, -1), seceoff(Q1, 0);
    int ngrp = 0, T = 0, maxn = 0;
    for (int q = 0; q <= Q; ++q) {
      if (R[q] == 0) continue;
      const int n = std::min(R[q], C[q]);
      if (n > kMaxGram) return fail("Gram block above the register Jacobi's order");
      if (std::max(R[q], C[q]) > kMaxDot) return fail("Gram dot product above the unrolled maximum");
      int grp = -1;
      if (n >= 2) {
        if (ngrp >= 4) return fail("more than four Gram blocks of order >= 2");
        grp = ngrp++;
      }
      seco[q] = int(sq.size());
      // Gram on the smaller side; on a tie, a gauge move takes the side of the
      // bond it does not rewrite (cols for a right move, rows for a left move):
      // that bond is already in its Schmidt basis (the previous decomposition of
      // it diagonalised the same reduced density matrix), so the Gram is
      // diagonal up to the truncations since and the Jacobi has nothing to do
      int side = R[q] < C[q] ? 0 : (R[q] > C[q] ? 1 : 0);
      if (R[q] == C[q] && o.kind == kOpGaugeR) side = 1;
      secn[q] = n; secside[q] = side; secgrp[q] = grp; seceoff[q] = T;
      sq.push_back(q);
      T += n;
      maxn = std::max(maxn, n);
    }
    const int nsec = int(sq.size());
    int maxdot = 1;
    for (int q : sq) maxdot = std::max(maxdot, std::max(R[q], C[q]));
    setH(kOhDot, maxdot);
    if (nsec > 15) return fail("more than 15 sectors");
    if (T > 64) return fail("more than 64 eigenvalues per decomposition");
    setH(kOhNsec, nsec); setH(kOhT, T); setH(kOhNgrp, ngrp);
    setH(kOhMaxr, maxn >= 3 ? 3 : (maxn == 2 ? 1 : 0));
    for (int g = 0; g < 4; ++g) I[hpos + kOhGrp + 8 * g] = -1;
    for (int s = 0; s < nsec; ++s) {
      const int q = sq[s], g = secgrp[q];
      if (g < 0) continue;
      int* G = &I[hpos + kOhGrp + 8 * g];
      G[0] = s; G[1] = secn[q]; G[2] = secside[q]; G[3] = THO[q]; G[4] = R[q]; G[5] = C[q]; G[6] = seceoff[q];
    }
    // order-1 sectors: the eigenvalue is the squared norm of the block's one row / column
    setH(kOhO1, pad());
    int no1 = 0;
    for (int s = 0; s < nsec; ++s) {
      const int q = sq[s];
      if (secn[q] != 1) continue;
      const bool rowv = secside[q] == 0;  // R = 1: one row of C entries
      push4(THO[q], rowv ? C[q] : R[q], rowv ? 1 : C[q], seceoff[q]);
      ++no1;
    }
    setH(kOhNo1, no1);
    if (no1 > 64) return fail("too many order-1 sectors");
    setH(kOhEq, pad());
    for (int s = 0; s < nsec; ++s) {
      const int q = sq[s];
      for (int i = 0; i < secn[q]; ++i) push4(s, i, seceoff[q], secn[q] | (D(newb, q) << 8));
    }
    setH(kOhSecQ, pad());
    for (int s = 0; s < nsec; ++s) I.push_back(sq[s] | (seceoff[sq[s]] << 8) | (secn[sq[s]] << 16));
    // -- factor elements, int4:
    //   w0 = dest | s << 16 | j << 20 | isx << 24 | scratch << 25
    //   w1 = exact: W offset of row idx (grp 16 + 4 idx); derived: M offset of the
    //        first term | terms << 16 | M stride << 21
    //   w2 = eigen offset of s | n << 8 | exact << 12
    //   w3 = W offset of the group (grp 16; 64 for an order-1 sector: the unit slot)
    // X rows of the left factor, Y cols of the right one; every destination is a
    // whole padded site (or scratch block): columns / rows j >= kept get zeros
    std::vector<int> XS_off(Q1, 0), YS_off(Q1, 0);
    int xs_tot = 0, ys_tot = 0, nf = 0;
    setH(kOhF, pad());
    bool ok = true;
    auto pushf = [&](int dest, int q, int j, bool isx, bool scratch, int idx) {
      const int s = seco[q], n = secn[q], side = secside[q], g = secgrp[q];
      const bool exact = isx ? side == 0 : side == 1;
      const int wb = g >= 0 ? 16 * g : 64;  // order 1: the unit slot WB[64]
      int w1;
      if (exact) {
        w1 = wb + (g >= 0 ? 4 * idx : 0);
      } else if (isx) {  // X[idx][j] = sum_c M[idx][c] W[c][w], c < C = n
        w1 = (THO[q] + idx * C[q]) | (n << 16) | (1 << 21);
      } else {  // Y[j][idx] = sum_r conj(W[r][w]) M[r][idx], r < R = n
        w1 = (THO[q] + idx) | (n << 16) | (C[q] << 21);
      }
      if (dest > 65535 || j > 15 || C[q] > 255 || THO[q] + idx * C[q] > 65535) ok = false;
      push4(dest | (s << 16) | (j << 20) | (isx ? 1 << 24 : 0) | (scratch ? 1 << 25 : 0), w1,
            seceoff[q] | (n << 8) | (exact ? 1 << 12 : 0), wb);
      ++nf;
    };
    for (int q = 0; q <= Q; ++q) {
      if (R[q] == 0) continue;
      const int jb = D(newb, q);
      if (o.kind == kOpGaugeL) {  // X into scratch, per sector R x D(newb, q)
        XS_off[q] = xs_tot;
        for (int row = 0; row < R[q]; ++row)
          for (int j = 0; j < jb; ++j) pushf(xs_tot + row * jb + j, q, j, true, true, row);
        xs_tot += R[q] * jb;
      } else {  // X into site k: rows (nr, a) of sector q are block (q - nr, nr), row a
        for (int nr = 0; nr < prow; ++nr) {
          if (RS[q][nr] < 0) continue;
          for (int a = 0; a < D(bl, q - nr); ++a)
            for (int j = 0; j < jb; ++j)
              pushf(PO(o.k, q - nr, nr) + a * D(o.k, q) + j, q, j, true, false, RS[q][nr] + a);
        }
      }
      if (o.kind == kOpGaugeR) {  // Y into scratch, per sector D(newb, q) x C
        YS_off[q] = ys_tot;
        for (int j = 0; j < jb; ++j)
          for (int col = 0; col < C[q]; ++col) pushf(ys_tot + j * C[q] + col, q, j, false, true, col);
        ys_tot += jb * C[q];
      } else {  // Y into site k+1 (two-site) / site k (left move): cols (nc, c) are block (q, nc), col c
        const int site = (o.kind == kOpGate) ? o.k + 1 : o.k;
        for (int nc = 0; nc < pcol; ++nc) {
          if (CS[q][nc] < 0) continue;
          for (int j = 0; j < jb; ++j)
            for (int c = 0; c < D(br, q + nc); ++c)
              pushf(PO(site, q, nc) + j * D(site, q + nc) + c, q, j, false, false, CS[q][nc] + c);
        }
      }
    }
    if (!ok) return fail("factor descriptor overflow");
    if (nf > 64 * kItF) return fail("factor list above the unrolled maximum");
    setH(kOhNf, nf);
    xsmax = std::max(xsmax, std::max(xs_tot, ys_tot));
    // -- gauge product: every element of the neighbour site, int4
    //   right move: S[(q, n)][j][c] = sum_b YS_q[j][b] A_{k+1}[(q, n)][b][c]
    //   left move : S[(ql, n)][a][j] = sum_b A_{k-1}[(ql, n)][a][b] XS_q[b][j], q = ql + n
    if (o.kind != kOpGate) {
      setH(kOhS, pad());
      const int nb = (o.kind == kOpGaugeR) ? o.k + 1 : o.k - 1;
      int cnt = 0;
      for (int q = 0; q <= Q; ++q)
        for (int n = 0; n < p && q + n <= Q; ++n) {
          const int po = PO(nb, q, n);
          if (po < 0) continue;
          const int dl = D(nb - 1, q), dr = D(nb, q + n);
          for (int a = 0; a < dl; ++a)
            for (int c = 0; c < dr; ++c) {
              int x1, x2, len, s2;
              if (o.kind == kOpGaugeR) {  // the neighbour's rows: bond k sector q
                len = R[q] == 0 ? 0 : D(o.k, q);
                x1 = YS_off[q] + a * C[q];
                x2 = po + c;
                s2 = dr;
              } else {  // the neighbour's cols: bond k-1 sector q + n
                const int qq = q + n;
                len = R[qq] == 0 ? 0 : D(o.k - 1, qq);
                x1 = po + a * dr;
                x2 = XS_off[qq] + c;
                s2 = D(newb, qq);
              }
              if (x1 > 65535 || x2 > 65535 || len > kMaxDm || s2 > 65535) return fail("product descriptor overflow");
              push4(x1 | (x2 << 16), len | (s2 << 16), po + a * dr + c, 0);
              ++cnt;
            }
        }
      if (cnt > 64 * kItS) return fail("gauge product above the unrolled maximum");
      setH(kOhNs, cnt);
    }
  }
  // ---- capacities and the LDS map of the fast region (complex units)
  int zc_off = 0;
  auto take = [&](int n) { const int o = zc_off; zc_off += (n + 1) & ~1; return o; };
  I[kHNp] = np;
  I[kHNblk] = nblk;
  I[kHBlk] = o_blk;
  I[kHLs] = o_ls;
  I[kHSite] = o_site;
  I[kHSiteN] = o_siten;
  I[kHNops] = int(ops.size());
  for (size_t i = 0; i < ops.size(); ++i) I[kHOps + int(i)] = op_off[i];
  // every operand buffer ends in a zero slot that no phase writes: a clamped
  // index beyond an element's term count points there instead of a select
  I[kHZMps] = take(np + 1);
  I[kHZTh] = take(thmax + 1);
  I[kHZTg] = take(thmax + 1);
  I[kHZW] = take(65);  // 4 groups x 16, then the unit slot
  I[kHZX] = take(xsmax + 1);
  I[kHThZ] = thmax;
  I[kHXsZ] = xsmax;
  I[kHZGt] = take(2 * P.gtotal);
  I[kHZPh] = take(2 * p + 2 * p * p);  // UF, UT, UF UF, UT UT
  I[kHZTot] = zc_off;
  I[kHCentre] = last_gate;
  pad();
  I[kHNint] = int(I.size());
  if (I.size() > 65535) return fail("plan too large");
  if (std::getenv("OCG_FAST_DUMP")) {  // diagnostic: the step's operations
    std::fprintf(stderr, "[fast plan] np %d nblk %d ints %zu zc %d\n", np, nblk, I.size(), zc_off);
    for (size_t i = 0; i < ops.size(); ++i) {
      const int* h = &I[op_off[i]];
      std::fprintf(stderr, "[fast plan] op %zu kind %d k %d nth %d nsec %d T %d ngrp %d maxr %d dot %d no1 %d nf %d ns %d\n",
                   i, h[kOhKind], h[kOhK], h[kOhNth], h[kOhNsec], h[kOhT], h[kOhNgrp], h[kOhMaxr], h[kOhDot],
                   h[kOhNo1], h[kOhNf], h[kOhNs]);
    }
  }
  out.plan = I;
  return out;
}

// ints of the fast region after its complex and double buffers: dims, block
// offsets, kept counts, kept eigenvector index table, flags; then the plan image
constexpr int kFastDbl = 64 + 64 + 64 + 8 + 2 * ocg::fastp::kMaxOps;  // LAM, SIG, 1 / SIG, spare, model cache
inline int fast_int_words(const OcgParams& P, int nblk) {
  auto al = [](int x) { return (x + 3) & ~3; };
  return ocg::fastp::kMaxOps /* model cache epochs */ + al(P.nsq) + al(nblk) + 64 /* KQ */ + 64 /* WIDX */ + 4 /* flags */;
}
inline int fast_lds_bytes(const std::vector<int>& plan, const OcgParams& P) {
  using namespace ocg::fastp;
  return plan[kHZTot] * 16 + kFastDbl * 8 + (fast_int_words(P, plan[kHNblk]) + int(plan.size())) * 4;
}

// The overlap plan of the padded layout (fast.hpp kOv*): the bounds, the
// environment layout per bond, the padded block offsets, per environment
// element its indices, per padded element its compact-format source and its
// stage-1 indices.  Empty (the general overlap runs) when a bound, an
// environment or a site is beyond the packed fields.
inline std::vector<int> build_overlap_plan(const OcgParams& P, const std::vector<int>& md) {
  using namespace ocg::fastp;
  const int L = P.L, p = P.p, Q = P.Q, Q1 = P.Q1;
  auto D = [&](int b, int q) { return (b < 0 || b > L || q < 0 || q > Q) ? 0 : md[size_t(b) * Q1 + q]; };
  if (p > kOvMaxP) return {};
  std::vector<int> eo(size_t(L + 1) * Q1, 0), en(L + 1, 0);
  int maxen = 1;
  for (int b = 0; b <= L; ++b) {
    int o = 0;
    for (int q = 0; q <= Q; ++q) {
      if (D(b, q) > kMaxDm) return {};  // the unrolled sums
      eo[size_t(b) * Q1 + q] = o;
      o += D(b, q) * D(b, q);
    }
    en[b] = o;
    maxen = std::max(maxen, o);
    if (o > kOvMaxE) return {};
  }
  // both ends are one 1 x 1 sector: E_0 = 1 and <X|Y> = E_L
  if (en[0] != 1 || en[L] != 1) return {};
  std::vector<int> po(size_t(L + 2) * Q1 * p, -1), sb(L + 2, 0), ls, blk;
  int np = 0, maxsite = 1;
  for (int k = 1; k <= L; ++k) {
    sb[k] = np;
    const int b0 = int(blk.size());
    for (int q = 0; q <= Q; ++q)
      for (int n = 0; n < p && q + n <= Q; ++n) {
        const int dl = D(k - 1, q), dr = D(k, q + n);
        if (dl == 0 || dr == 0) continue;
        const int b = int(blk.size()), ri = (k - 1) * Q1 + q, ci = k * Q1 + q + n;
        blk.push_back(ri | (ci << 16));
        po[(size_t(k) * Q1 + q) * p + n] = np - sb[k];
        for (int a = 0; a < dl; ++a)
          for (int c = 0; c < dr; ++c) {
            ls.push_back(ri | (ci << 16));
            ls.push_back(b | (b0 << 16));
            ls.push_back(a | (c << 4) | (dl << 8) | (dr << 12) | (eo[size_t(k - 1) * Q1 + q] << 16));
            ls.push_back(P.site_base[k]);
          }
        np += dl * dr;
      }
    maxsite = std::max(maxsite, np - sb[k]);
  }
  sb[L + 1] = np;
  if (np == 0 || np > 4096 || int(blk.size()) > 32767 || (L + 1) * Q1 > 32767) return {};
  std::vector<int> elo(L + 2, 0), el;
  for (int b = 0; b <= L; ++b) {
    elo[b] = int(el.size());
    for (int q = 0; q <= Q; ++q)
      for (int c = 0; c < D(b, q); ++c)
        for (int d = 0; d < D(b, q); ++d) el.push_back(q | (c << 8) | (d << 12) | (D(b, q) << 16));
  }
  elo[L + 1] = int(el.size());
  std::vector<int> Dv(size_t(L + 1) * Q1);
  for (int b = 0; b <= L; ++b)
    for (int q = 0; q <= Q; ++q) Dv[size_t(b) * Q1 + q] = D(b, q);
  std::vector<int> I(kOvHdr, 0);
  auto sec = [&](int slot, const std::vector<int>& v) {
    while (I.size() & 3) I.push_back(0);  // 16-byte aligned tables
    I[slot] = int(I.size());
    I.insert(I.end(), v.begin(), v.end());
  };
  I[kOvL] = L;
  I[kOvQ1] = Q1;
  I[kOvP] = p;
  I[kOvNp] = np;
  I[kOvNblk] = int(blk.size());
  I[kOvMaxSite] = maxsite;
  I[kOvMaxEn] = maxen;
  sec(kOvD, Dv);
  sec(kOvEo, eo);
  sec(kOvEn, en);
  sec(kOvPo, po);
  sec(kOvSb, sb);
  sec(kOvElo, elo);
  sec(kOvEl, el);
  sec(kOvLs, ls);
  sec(kOvBlk, blk);
  while (I.size() & 3) I.push_back(0);
  I[kOvNint] = int(I.size());
  return I;
}
// LDS of the one-wave overlap (fast_overlap.hpp): plan, two dims / block-offset
// arrays, the two padded states and their zero slot, T, two environments
// (with_dH: the <X|dH|Y> buffers too, FastOverlap::contract_dH)
inline int overlap_lds_bytes(const std::vector<int>& I, const OcgParams& P, bool with_dH = false) {
  using namespace ocg::fastp;
  auto al = [](int x) { return (x + 3) & ~3; };
  const int ints = I[kOvNint] + 2 * al(P.nsq) + 2 * al(I[kOvNblk] + 1);
  int zs = 2 * (I[kOvNp] + 2) + (I[kOvMaxSite] + 2) + 2 * (I[kOvMaxEn] + 2);
  if (with_dH) zs += (I[kOvMaxSite] + 2) + 2 * (I[kOvMaxEn] + 2);
  return ints * 4 + zs * 16;
}

}  // namespace ocg_host
