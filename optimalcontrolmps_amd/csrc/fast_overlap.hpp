// MI355X (gfx950) one-wave overlap <X|Y> in the padded layout: calcHessianRow's
// <xiH_j|psiH_i(j)> (reference src/OptimalControl.cpp:259-277) for chains the
// one-wave padded chain runs (fast_chain.hpp, config 1).
//
// The general overlap (Chain::overlap) rebuilds its environment and block
// tables from the two states' runtime bond dimensions at every site, with a
// workgroup barrier between every table scan and contraction: ~38 us per
// overlap on one wave at config 1.  Here both states are expanded into the
// padded layout of the fast plan (every bond sector at its Schmidt-rank bound,
// zero beyond the runtime dimension), so every index of the contraction is a
// host-built table entry (fast_plan.hpp build_overlap_plan), and one wave runs
// two phases per site with a wave fence between them:
//   stage 1  T_(q,n) = E_(k-1)[q] Y_(q,n)          one lane per padded element
//   stage 2  E_k[q'] = sum_n X_(q'-n,n)^H T_(q'-n,n) one lane per environment element
// E_0 = 1 and <X|Y> = E_L (both end bonds are one 1 x 1 sector).  Padded rows
// and columns are exact zeros in both states, so they add exact zeros.
//
// Only wave 0 of the workgroup works; the other waves skip every call, and no
// call contains a workgroup barrier.
#pragma once

#include "engine_device.hpp"
#include "fast.hpp"

namespace ocg {

struct FastOverlap {
  const int lane;
  const bool act;  // wave 0
  LDS int *PL, *DX, *DY, *BX, *BY;
  lzp XP, YP, T, E0, E1;
  lzp T1, F0, F1;  // <X|dH|Y> (contract_dH): T of the dH environment, its two environments
  bool dh = false;
  int L, Q1, p, np, nblk, nsq;
  int zs, ze;  // zero slots of T and of both environments (XP's and YP's: np)
  int o_d, o_eo, o_en, o_po, o_sb, o_elo, o_el, o_ls, o_blk;

  // base: LDS of overlap_lds_bytes(plan) bytes, 16-byte aligned
  // with_dH: the dH buffers after the others (overlap_lds_bytes(plan, P, true))
  __device__ OCG_INLINE FastOverlap(const OcgParams& P, char* base, const int* gplan, bool with_dH = false)
      : lane(threadIdx.x & 63), act(threadIdx.x < 64), dh(with_dH) {
    using namespace fastp;
    if (!gplan) return;
    // the header is read from global memory (uniform scalar loads)
    L = gplan[kOvL]; Q1 = gplan[kOvQ1]; p = gplan[kOvP]; np = gplan[kOvNp]; nblk = gplan[kOvNblk];
    nsq = P.nsq;
    o_d = gplan[kOvD]; o_eo = gplan[kOvEo]; o_en = gplan[kOvEn]; o_po = gplan[kOvPo]; o_sb = gplan[kOvSb];
    o_elo = gplan[kOvElo]; o_el = gplan[kOvEl]; o_ls = gplan[kOvLs]; o_blk = gplan[kOvBlk];
    auto al = [](int x) { return (x + 3) & ~3; };
    LDS int* ib = (LDS int*)base;
    PL = ib; ib += gplan[kOvNint];
    DX = ib; ib += al(nsq);
    DY = ib; ib += al(nsq);
    BX = ib; ib += al(nblk + 1);
    BY = ib; ib += al(nblk + 1);
    zs = gplan[kOvMaxSite];
    ze = gplan[kOvMaxEn];
    XP = lzp{(LDS double*)ib};
    YP = XP + (np + 2);
    T = YP + (np + 2);
    E0 = T + (zs + 2);
    E1 = E0 + (ze + 2);
    T1 = E1 + (ze + 2);
    F0 = T1 + (zs + 2);
    F1 = F0 + (ze + 2);
  }
  __device__ __forceinline__ void wsync() const {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  __device__ __forceinline__ static i4 ld4(const LDS int* p) { return *(const LDS i4*)p; }
  // plan image into LDS (once per launch)
  __device__ OCG_INLINE void init(const int* gplan) {
    if (!act) return;
    const int ni = gplan[fastp::kOvNint];
    for (int i = lane; i < ni; i += 64) PL[i] = gplan[i];
    if (lane == 0) {  // zero slots: a clamped term of an unrolled sum reads one
      XP[np] = c2(0.0, 0.0);
      YP[np] = c2(0.0, 0.0);
      T[zs] = c2(0.0, 0.0);
      E0[ze] = c2(0.0, 0.0);
      E1[ze] = c2(0.0, 0.0);
      if (dh) {
        T1[zs] = c2(0.0, 0.0);
        F0[ze] = c2(0.0, 0.0);
        F1[ze] = c2(0.0, 0.0);
      }
    }
    wsync();
  }

  // compact-format block offsets of the dims in DIMS (site-relative offset of
  // block b: BOF[b] - BOF[first block of its site]); returns the state's
  // compact element count (every site)
  __device__ OCG_INLINE int block_offsets(const LDS int* DIMS, LDS int* BOF) const {
    int carry = 0;
    for (int b0 = 0; b0 < nblk; b0 += 64) {
      const int b = b0 + lane;
      const int t = PL[o_blk + (b < nblk ? b : nblk - 1)];
      const int sz = b < nblk ? DIMS[t & 0xffff] * DIMS[unsigned(t) >> 16] : 0;
      const int inc = wscan(sz);
      if (b < nblk) BOF[b] = carry + inc - sz;
      carry += rdlane(inc, 63);
    }
    return carry;
  }
  // compact state -> padded LDS image (zeros beyond the runtime dims): the
  // source index of padded element x, or -1
  __device__ __forceinline__ int src_index(const LDS int* DIMS, const LDS int* BOF, int x) const {
    const i4 d = ld4(PL + o_ls + 4 * (x < np ? x : np - 1));
    const int dl = DIMS[d[0] & 0xffff], dr = DIMS[unsigned(d[0]) >> 16];
    const int b = d[1] & 0xffff, f = unsigned(d[1]) >> 16, a = d[2] & 15, c = (d[2] >> 4) & 15;
    return (x < np && a < dl && c < dr) ? d[3] + BOF[b] - BOF[f] + a * dr + c : -1;
  }
  // X into XP and (gy set) Y into YP, four elements of each per lane in flight
  __device__ OCG_INLINE void expand(const zc* gx, const zc* gy) const {
    for (int x0 = 0; x0 < np; x0 += 256) {
      zc vx[4], vy[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int x = x0 + lane + 64 * u;
        const int ix = src_index(DX, BX, x);
        vx[u] = c2(0.0, 0.0);
        if (ix >= 0) vx[u] = c2(gx[ix].x, gx[ix].y);
        vy[u] = c2(0.0, 0.0);
        if (gy) {
          const int iy = src_index(DY, BY, x);
          if (iy >= 0) vy[u] = c2(gy[iy].x, gy[iy].y);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int x = x0 + lane + 64 * u;
        if (x < np) {
          XP[x] = vx[u];
          if (gy) YP[x] = vy[u];
        }
      }
    }
  }
  // X (global, compact) into XP; Y (global, compact) into YP when gdy is set.
  // Returns Y's compact element count (the traffic model's), 0 without Y.
  __device__ OCG_INLINE int load(const int* gdx, const zc* gx, const int* gdy, const zc* gy) {
    if (!act) return 0;
    for (int i = lane; i < nsq; i += 64) {
      DX[i] = gdx[i];
      if (gdy) DY[i] = gdy[i];
    }
    wsync();
    block_offsets(DX, BX);
    const int ny = gdy ? block_offsets(DY, BY) : 0;
    wsync();
    expand(gx, gy);
    wsync();
    return ny;
  }
  // the compact element count of a state whose dims are DIMS (LDS)
  __device__ OCG_INLINE int compact_size(const LDS int* DIMS) {
    if (!act) return 0;
    const int n = block_offsets(DIMS, BY);
    wsync();
    return n;
  }

  // <X|Y> with X = XP and Y a padded image (YP, or the one-wave chain's MPS);
  // the value is valid in every lane of wave 0
  __device__ OCG_INLINE zc contract(lzp Y) {
    using fastp::kMaxDm;
    using fastp::kOvMaxP;
    if (!act) return c2(0.0, 0.0);
    if (lane == 0) E0[0] = c2(1.0, 0.0);
    wsync();
    lzp Ep = E0, En = E1;
    for (int k = 1; k <= L; ++k) {
      const int s0 = PL[o_sb + k], ns = PL[o_sb + k + 1] - s0;
      // stage 1: T[(q,n)][a'][c] = sum_a E_(k-1)[q][a'][a] Y_(q,n)[a][c]
      // (a < D(k-1, q) <= kMaxDm, unrolled; a clamped term reads the zero slots)
      for (int e = lane; e < ns; e += 64) {
        const int w = PL[o_ls + 4 * (s0 + e) + 2];
        const int a = w & 15, c = (w >> 4) & 15, dq = (w >> 8) & 15, dr = (w >> 12) & 15, eo = unsigned(w) >> 16;
        const int yb = s0 + e - a * dr, eb = eo + a * dq;  // column c of the block's first row; row a' of E
        zc ev[kMaxDm], yv[kMaxDm];
#pragma unroll
        for (int t = 0; t < kMaxDm; ++t) {
          ev[t] = Ep[t < dq ? eb + t : ze];
          yv[t] = Y[t < dq ? yb + t * dr : np];
        }
        zc acc = c2(0.0, 0.0);
#pragma unroll
        for (int t = 0; t < kMaxDm; ++t) cacc(acc, ev[t], yv[t]);
        T[e] = acc;
      }
      wsync();
      // stage 2: E_k[q'][c'][c] = sum_n sum_a' conj(X_(q'-n,n)[a'][c']) T_(q'-n,n)[a'][c]
      // (n < p <= kOvMaxP, a' < kMaxDm, unrolled and clamped as above)
      const int ne = PL[o_en + k], el0 = PL[o_elo + k];
      for (int x = lane; x < ne; x += 64) {
        const int w = PL[o_el + el0 + x];
        const int qp = w & 255, cp = (w >> 8) & 15, c = (w >> 12) & 15, dr = unsigned(w) >> 16;
        int o[kOvMaxP], dq[kOvMaxP];
#pragma unroll
        for (int n = 0; n < kOvMaxP; ++n) {
          const int q = qp - n;
          const bool in = n < p && q >= 0;
          const int on = PL[in ? o_po + (k * Q1 + q) * p + n : o_po];
          const int dn = PL[in ? o_d + (k - 1) * Q1 + q : o_d];
          o[n] = on;
          dq[n] = (in && on >= 0) ? dn : 0;
        }
        zc acc = c2(0.0, 0.0);
#pragma unroll
        for (int n = 0; n < kOvMaxP; ++n) {
          if (n < p) {  // uniform (no break: it would demote the arrays to scratch)
            zc xv[kMaxDm], tv[kMaxDm];
#pragma unroll
            for (int a = 0; a < kMaxDm; ++a) {
              const bool v = a < dq[n];
              xv[a] = XP[v ? s0 + o[n] + cp + a * dr : np];
              tv[a] = T[v ? o[n] + c + a * dr : zs];
            }
#pragma unroll
            for (int a = 0; a < kMaxDm; ++a) cjacc(acc, xv[a], tv[a]);
          }
        }
        En[x] = acc;
      }
      wsync();
      const lzp t = Ep;
      Ep = En;
      En = t;
    }
    return Ep[0];
  }

  // <X|dH|Y>, dH = sum_k 0.5 n_k (n_k - 1) (propagatorDeriv, src/BH_tDMRG.cpp:10-14;
  // Chain::overlap's with_dH): E carries the identity string, F the strings with
  // dH already applied, F_k = sum_n X^H (F_(k-1) Y + f(n) E_(k-1) Y), f = P.dH.
  // Per n the two partial sums s0, s1 first, as Chain::overlap adds them.
  __device__ OCG_INLINE zc contract_dH(lzp Y, const double* fdh) {
    using fastp::kMaxDm;
    using fastp::kOvMaxP;
    if (!act) return c2(0.0, 0.0);
    if (lane == 0) {
      E0[0] = c2(1.0, 0.0);
      F0[0] = c2(0.0, 0.0);
    }
    wsync();
    lzp Ep = E0, En = E1, Fp = F0, Fn = F1;
    for (int k = 1; k <= L; ++k) {
      const int s0 = PL[o_sb + k], ns = PL[o_sb + k + 1] - s0;
      for (int e = lane; e < ns; e += 64) {
        const int w = PL[o_ls + 4 * (s0 + e) + 2];
        const int a = w & 15, c = (w >> 4) & 15, dq = (w >> 8) & 15, dr = (w >> 12) & 15, eo = unsigned(w) >> 16;
        const int yb = s0 + e - a * dr, eb = eo + a * dq;
        zc ev[kMaxDm], fv[kMaxDm], yv[kMaxDm];
#pragma unroll
        for (int t = 0; t < kMaxDm; ++t) {
          ev[t] = Ep[t < dq ? eb + t : ze];
          fv[t] = Fp[t < dq ? eb + t : ze];
          yv[t] = Y[t < dq ? yb + t * dr : np];
        }
        zc a0 = c2(0.0, 0.0), a1 = c2(0.0, 0.0);
#pragma unroll
        for (int t = 0; t < kMaxDm; ++t) {
          cacc(a0, ev[t], yv[t]);
          cacc(a1, fv[t], yv[t]);
        }
        T[e] = a0;
        T1[e] = a1;
      }
      wsync();
      const int ne = PL[o_en + k], el0 = PL[o_elo + k];
      for (int x = lane; x < ne; x += 64) {
        const int w = PL[o_el + el0 + x];
        const int qp = w & 255, cp = (w >> 8) & 15, c = (w >> 12) & 15, dr = unsigned(w) >> 16;
        int o[kOvMaxP], dq[kOvMaxP];
#pragma unroll
        for (int n = 0; n < kOvMaxP; ++n) {
          const int q = qp - n;
          const bool in = n < p && q >= 0;
          const int on = PL[in ? o_po + (k * Q1 + q) * p + n : o_po];
          const int dn = PL[in ? o_d + (k - 1) * Q1 + q : o_d];
          o[n] = on;
          dq[n] = (in && on >= 0) ? dn : 0;
        }
        zc acc0 = c2(0.0, 0.0), acc1 = c2(0.0, 0.0);
#pragma unroll
        for (int n = 0; n < kOvMaxP; ++n) {
          if (n < p) {  // uniform
            zc xv[kMaxDm], tv[kMaxDm], uv[kMaxDm];
#pragma unroll
            for (int a = 0; a < kMaxDm; ++a) {
              const bool v = a < dq[n];
              xv[a] = XP[v ? s0 + o[n] + cp + a * dr : np];
              tv[a] = T[v ? o[n] + c + a * dr : zs];
              uv[a] = T1[v ? o[n] + c + a * dr : zs];
            }
            zc p0 = c2(0.0, 0.0), p1 = c2(0.0, 0.0);
#pragma unroll
            for (int a = 0; a < kMaxDm; ++a) {
              cjacc(p0, xv[a], tv[a]);
              cjacc(p1, xv[a], uv[a]);
            }
            acc0 = cadd(acc0, p0);
            acc1 = cadd(acc1, cadd(p1, cscale(p0, fdh[n])));
          }
        }
        En[x] = acc0;
        Fn[x] = acc1;
      }
      wsync();
      lzp t = Ep;
      Ep = En;
      En = t;
      t = Fp;
      Fp = Fn;
      Fn = t;
    }
    return Fp[0];
  }
};

}  // namespace ocg
