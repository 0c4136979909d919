// MI355X (gfx950) one-wave padded chain: BH_tDMRG::step for chains whose
// bond sectors all stay small (config 1: L=5, p=5, Npart=5, bonds <= 14).
//
// The generic chain (engine_device.hpp) rebuilds its block tables from the
// runtime bond dimensions and runs every phase on two waves separated by
// workgroup barriers; at config 1 a step costs ~165 k cycles there, most of
// it bookkeeping and barrier / LDS round trips around tiny blocks.  Here every
// bond sector is stored at its Schmidt-rank bound, zero-padded (fast_plan.hpp),
// so the layout of every site, Θ, matricisation and factor is fixed and the
// whole step is a replay of host-built descriptor tables by ONE wave: no
// workgroup barrier, no table scan, a wave-level fence between phases.  Every
// phase is written for instruction-level parallelism: a lane's descriptors for
// all its elements are loaded at once, then all their operands (inner loops
// unrolled to the compile-time bounds of fast.hpp with clamped addresses and
// selects), so a phase costs two or three LDS round trips instead of one per
// loop iteration.
//
// The arithmetic is that of Chain::step (reference src/BH_tDMRG.cpp:111-230
// with ITensor denmatDecomp / position): Θ = A_i1 A_i2, pre-phase -> hopping
// gate -> post-phase, per-sector Gram on the smaller side, register Jacobi
// (16-lane groups, DPP partner exchange), the ITensor truncation rule
// (relative cutoff, Maxm, floor 1e-30, rank bound), factors, gauge moves with
// the 1e-14 gauge cutoff, closing phase and normalisation.  Padded rows /
// columns are exact zeros, their Gram eigenvalues are exact zeros and are
// always discarded, so results agree with the generic chain to rounding
// (tests/test_fast_chain.py, tests/test_emu.py).
//
// Only wave 0 of the workgroup works; the other waves skip every call, and no
// call contains a workgroup barrier.
#pragma once

#include "engine_device.hpp"
#include "fast.hpp"

namespace ocg {

struct FastChain {
  using CH = Chain<64>;  // its static Jacobi helpers (rotation, DPP partners, bpermute)
  const OcgParams& P;
  const int lane;
  const bool act;  // wave 0
  lzp MP, TH, TG, WB, XS, GT, PH;
  LDS double *LAM, *SIG, *SIGI, *MCB, *MCF;
  LDS int* MCE;
  LDS int *DIM, *BOF, *KQ, *WIDX, *PL;
  int np, nblk, o_blk, o_ls, o_site, o_siten, nops, centre_open;
  int thz, xsz;  // zero slots of TH / TG and XS (MP's is np)
  double ph_u = __builtin_nan("");
  int ph_dir = -1;
  // dims_epoch counts bond-dimension changes (block offsets are recomputed
  // only after one)
  int dims_epoch = 0, bof_epoch = -1;
  int trace_op = -1;  // diagnostics: the step operation being run
  // algorithmic-traffic model (the general chain's accounting), per lane
  double m_bytes = 0, m_flops = 0;
  // diagnostic build (-DOCG_PROFILE): shader-clock cycles per phase into the
  // general chain's PROF slots (the same categories as Chain::pf)
  LDS double* PROF = nullptr;
  unsigned long long pf_last = 0;
  int pf_cur = 0;
  __device__ __forceinline__ void pf(int cat) {
#ifdef OCG_PROFILE
    if (threadIdx.x == 0 && PROF) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (pf_last) PROF[pf_cur] += double(t - pf_last);
      pf_last = t;
      pf_cur = cat;
    }
#else
    (void)cat;
#endif
  }
  // diagnostic build: event counts into PROF slots 20..22, 30 (jacobi sweeps,
  // calls, decompositions, rounds)
  __device__ __forceinline__ void cnt(int slot, double v) {
#ifdef OCG_PROFILE
    if (threadIdx.x == 0 && PROF) PROF[slot] += v;
#else
    (void)slot;
    (void)v;
#endif
  }

  // base: the fast region of the dynamic LDS (fast_lds_bytes of the plan)
  __device__ OCG_INLINE FastChain(const OcgParams& P_, char* base, const int* gplan, LDS double* prof = nullptr)
      : P(P_), lane(threadIdx.x & 63), act(threadIdx.x < 64), PROF(prof) {
    using namespace fastp;
    if (!gplan) return;  // not used by this launch
    // the header is read from global memory (uniform scalar loads)
    np = gplan[kHNp]; nblk = gplan[kHNblk]; o_blk = gplan[kHBlk]; o_ls = gplan[kHLs]; o_site = gplan[kHSite];
    o_siten = gplan[kHSiteN]; nops = gplan[kHNops]; centre_open = gplan[kHCentre];
    thz = gplan[kHThZ]; xsz = gplan[kHXsZ];
    lzp cb{(LDS double*)base};
    MP = cb + gplan[kHZMps]; TH = cb + gplan[kHZTh]; TG = cb + gplan[kHZTg]; WB = cb + gplan[kHZW];
    XS = cb + gplan[kHZX]; GT = cb + gplan[kHZGt]; PH = cb + gplan[kHZPh];
    LDS double* db = (cb + gplan[kHZTot]).p;
    LAM = db; SIG = db + 64; SIGI = db + 128;  // then 8 spare doubles
    MCB = db + 200; MCF = db + 200 + fastp::kMaxOps;  // the traffic model's per-op cache
    LDS int* ib = (LDS int*)(db + 200 + 2 * fastp::kMaxOps);
    MCE = ib; ib += fastp::kMaxOps;
    auto al = [](int x) { return (x + 3) & ~3; };  // 16-byte aligned int arrays
    DIM = ib; ib += al(P.nsq);
    BOF = ib; ib += al(nblk);
    KQ = ib; ib += 64;
    WIDX = ib; ib += 64;
    ib += 4;  // flags (spare)
    PL = ib;
  }
  __device__ __forceinline__ void wsync() const {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  __device__ __forceinline__ static i4 ld4(const LDS int* p) { return *(const LDS i4*)p; }
  // op-header fields are wave-uniform: scalar registers, uniform branches
  __device__ __forceinline__ static int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
  // plan image and gate tables into LDS (once per launch)
  __device__ OCG_INLINE void init(const int* gplan, const zc* gf, const zc* gb) {
    if (!act) return;
    const int ni = gplan[fastp::kHNint];
    for (int i = lane; i < ni; i += 64) PL[i] = gplan[i];
    for (int i = lane; i < P.gtotal; i += 64) { GT[i] = gf[i]; GT[P.gtotal + i] = gb[i]; }
    if (lane < fastp::kMaxOps) MCE[lane] = -1;
    if (lane == 0) {
      WB[64] = c2(1.0, 0.0);  // the eigenvector of every order-1 sector
      MP[np] = c2(0.0, 0.0);  // zero slots
      TH[thz] = c2(0.0, 0.0);
      TG[thz] = c2(0.0, 0.0);
      XS[xsz] = c2(0.0, 0.0);
    }
    wsync();
  }
  __device__ __forceinline__ int dim(int b, int q) const { return (q < 0 || q > P.Q) ? 0 : DIM[b * P.Q1 + q]; }

  // ------------------------------------------------------------- I/O
  // compact interchange format (include/ocmps.h): dims[nsq], site k at
  // site_base[k], blocks (q, n) packed row-major in (q, n) order.  BOF[b] =
  // exclusive prefix of the compact block sizes over the block list (the
  // site-relative offset is BOF[b] - BOF[first block of the site]); recomputed
  // only after the dims changed.
  __device__ OCG_INLINE void block_offsets() {
    if (bof_epoch == dims_epoch) return;
    int carry = 0;
    for (int b0 = 0; b0 < nblk; b0 += 64) {
      const int b = b0 + lane, bb = b < nblk ? b : nblk - 1;
      const i4 t = ld4(PL + o_blk + 4 * bb);
      const int sz = b < nblk ? DIM[t[1]] * DIM[t[2]] : 0;
      const int inc = wscan(sz);
      if (b < nblk) BOF[b] = carry + inc - sz;
      carry += rdlane(inc, 63);
    }
    bof_epoch = dims_epoch;
    wsync();
  }
  template <class PI, class PZ>
  __device__ OCG_INLINE void load(const PI* gdims, const PZ* gdata) {
    if (!act) return;
    pf(10);
    for (int i = lane; i < P.nsq; i += 64) DIM[i] = gdims[i];
    ++dims_epoch;
    wsync();
    block_offsets();
    i4 d[fastp::kItMps];
#pragma unroll
    for (int it = 0; it < fastp::kItMps; ++it) {
      const int x = lane + 64 * it;
      d[it] = ld4(PL + o_ls + 4 * (x < np ? x : np - 1));
    }
#pragma unroll
    for (int it = 0; it < fastp::kItMps; ++it) {
      const int x = lane + 64 * it;
      const int dl = DIM[d[it][0] & 0xffff], dr = DIM[unsigned(d[it][0]) >> 16];
      const int b = d[it][1] & 0xffff, f = unsigned(d[it][1]) >> 16, a = d[it][2] & 0xff, c = unsigned(d[it][2]) >> 8;
      const bool ok = x < np && a < dl && c < dr;
      const int idx = d[it][3] + BOF[b] - BOF[f] + a * dr + c;  // no lane-indexed kernel-argument read
      zc v = c2(0.0, 0.0);
      if (ok) v = c2(gdata[idx].x, gdata[idx].y);
      if (x < np) MP[x] = v;
    }
    wsync();
  }
  // wt: write-through stores (agent-scope relaxed stores: the state leaves the
  // XCD's L2 on the store itself, so a consumer on another XCD can read it after
  // a flag without a release fence)
  __device__ OCG_INLINE void store(int* gdims, zc* gdata, bool wt = false) {
    if (!act) return;
    pf(10);
    block_offsets();
    for (int i = lane; i < P.nsq; i += 64) {
      if (wt) __hip_atomic_store(gdims + i, DIM[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else gdims[i] = DIM[i];
    }
    i4 d[fastp::kItMps];
#pragma unroll
    for (int it = 0; it < fastp::kItMps; ++it) {
      const int x = lane + 64 * it;
      d[it] = ld4(PL + o_ls + 4 * (x < np ? x : np - 1));
    }
#pragma unroll
    for (int it = 0; it < fastp::kItMps; ++it) {
      const int x = lane + 64 * it;
      const int dl = DIM[d[it][0] & 0xffff], dr = DIM[unsigned(d[it][0]) >> 16];
      const int b = d[it][1] & 0xffff, f = unsigned(d[it][1]) >> 16, a = d[it][2] & 0xff, c = unsigned(d[it][2]) >> 8;
      const int idx = d[it][3] + BOF[b] - BOF[f] + a * dr + c;  // no lane-indexed kernel-argument read
      const zc v = MP[x < np ? x : 0];
      if (x < np && a < dl && c < dr) {
        if (wt) {
          double* dd = (double*)(gdata + idx);
          __hip_atomic_store(dd, v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(dd + 1, v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          gdata[idx] = v;
        }
      }
    }
  }

  __device__ OCG_INLINE void model_totals(double& b, double& f) const {
    b = wsum(m_bytes);
    f = wsum(m_flops);
  }
  // the traffic model of one two-site update on the current (unpadded) dims:
  // 16 (2 (|A_i1| + |A_i2|) + gate) bytes, 8 (R C m + R C p + n^2 max(R, C) +
  // 2 R C m) flops per middle sector (Chain::build_theta's accounting)
  // The model depends only on the bond dims at the gate, so an op's wave total
  // is cached with the dims epoch it was formed at and reused while no bond
  // dimension has changed since (every step once config 1's dims saturate).
  __device__ OCG_INLINE void model_gate(int o, int i1) {
    using namespace fastp;
    if (uni(MCE[o]) == dims_epoch) {
      if (lane == 0) {
        m_bytes += MCB[o];
        m_flops += MCF[o];
      }
      return;
    }
    // all 3 p bond dims of the three bonds in one wave of loads (clamped
    // addresses, out-of-range sectors selected to 0)
    const int p = P.p, Q = P.Q, Q1 = P.Q1, q = lane < Q1 ? lane : 0;
    const LDS int* d0 = DIM + (i1 - 1) * Q1;
    const LDS int* d1 = DIM + i1 * Q1;
    const LDS int* d2 = DIM + (i1 + 1) * Q1;
    int l[6], a[6], r[6];
#pragma unroll
    for (int n = 0; n < 6; ++n) {
      const int qm = q - n, qp = q + n;
      const bool okm = n < p && qm >= 0, okp = n < p && qp <= Q;
      const int lm = d0[okm ? qm : 0], ap = d1[okp ? qp : 0], rp = d2[okp ? qp : 0];
      l[n] = okm ? lm : 0;
      a[n] = okp ? ap : 0;
      r[n] = okp ? rp : 0;
    }
    int R = 0, C = 0, u = 0;
    const int m = a[0], dl = l[0];
#pragma unroll
    for (int n = 0; n < 6; ++n) {
      R += l[n];
      C += r[n];
      u += dl * a[n] + m * r[n];
    }
    double fl = 0.0, by = 0.0;
    if (lane < Q1) {
      if (R == 0 || C == 0) { R = 0; C = 0; }
      const double Rd = R, Cd = C, nn = R < C ? R : C;
      fl = 8.0 * (Rd * Cd * m + Rd * Cd * p + nn * nn * (R > C ? Rd : Cd) + 2.0 * Rd * Cd * m);
      by = 32.0 * double(u);
    }
    if (lane == 0) by += 16.0 * P.gtotal;
    const double bt = wsum(by), ft = wsum(fl);
    if (lane == 0) {
      m_bytes += bt;
      m_flops += ft;
      MCB[o] = bt;
      MCF[o] = ft;
      MCE[o] = dims_epoch;
    }
  }

  // ------------------------------------------------------------- Θ and gate
  __device__ OCG_INLINE void theta(const LDS int* oh) {
    using namespace fastp;
    pf(0);
    const int nth = uni(oh[kOhNth]);
    if (nth <= 64) theta_it<1>(oh, nth);
    else theta_it<kItTh>(oh, nth);
    wsync();
  }
  // IT: 64-element iterations, unrolled (the op's element count picks the instance)
  template <int IT>
  __device__ OCG_INLINE void theta_it(const LDS int* oh, int nth) {
    using namespace fastp;
    const LDS int* md = PL + uni(oh[kOhMat]);
    int d0[IT], d1[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int e = lane + 64 * it, ee = e < nth ? e : nth - 1;
      d0[it] = md[2 * ee];
      d1[it] = md[2 * ee + 1];
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int e = lane + 64 * it;
      const int x1 = d0[it] & 0xffff, x2 = unsigned(d0[it]) >> 16, dm = d1[it] & 0xff, drc = unsigned(d1[it]) >> 8;
      const int dmc = dm > 0 ? dm - 1 : 0;
      zc acc = c2(0.0, 0.0);
#pragma unroll
      for (int b = 0; b < kMaxDm; ++b) {
        const int bb = b < dmc ? b : dmc;
        const zc a = MP[b < dm ? x1 + b : np], v = MP[x2 + bb * drc];  // beyond dm: the zero slot
        cacc(acc, a, v);
      }
      if (e < nth) TH[e] = acc;
    }
  }
  // pre-phase -> hopping gate (per Δ = n1 + n2 block) -> post-phase (Chain::apply_gate).
  // PH holds UF[p], UT[p], then the pair products UF[n1] UF[n2] and UT[a1] UT[a2] (p^2 each)
  // PRE: 0 none, 1 the pair UF[n1] UF[n2], 2 UF[n2] alone; POST: 0 none, 1 the
  // pair UT[a1] UT[a2], 2 UT[a2] alone (compile-time: no per-element selects)
  __device__ OCG_INLINE void gate(const LDS int* oh, int forward) {
    using namespace fastp;
    pf(1);
    const int mode = uni(oh[kOhMode]), lonely = uni(oh[kOhLonely]);
    if (uni(oh[kOhNth]) <= 64) gate_mode<1>(oh, forward, mode, lonely);
    else gate_mode<kItTh>(oh, forward, mode, lonely);
    wsync();
  }
  template <int IT>
  __device__ OCG_INLINE void gate_mode(const LDS int* oh, int forward, int mode, int lonely) {
    if (mode == 0) {
      if (lonely & 1) gate_body<1, 2, IT>(oh, forward);
      else gate_body<1, 0, IT>(oh, forward);
    } else {
      if (lonely & 2) gate_body<2, 1, IT>(oh, forward);
      else gate_body<0, 1, IT>(oh, forward);
    }
  }
  template <int PRE, int POST, int IT>
  __device__ OCG_INLINE void gate_body(const LDS int* oh, int forward) {
    using namespace fastp;
    const int p = P.p, nth = uni(oh[kOhNth]);
    const LDS int* gd = PL + uni(oh[kOhGate]);
    lzp g0 = GT + (forward ? 0 : P.gtotal);
    lzp UF = PH, UT = PH + p, UFF = PH + 2 * p, UTT = PH + 2 * p + p * p;
    i4 d[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int e = lane + 64 * it;
      d[it] = ld4(gd + 4 * (e < nth ? e : nth - 1));
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int e = lane + 64 * it;
      const unsigned h = d[it][0];
      const int sz = (h >> 16) & 15, lo = (h >> 20) & 15, a1 = (h >> 24) & 15, a2 = h >> 28, D = a1 + a2;
      lzp g = g0 + int(h & 0xffff);
      zc acc = c2(0.0, 0.0);
#pragma unroll
      for (int x = 0; x < 6; ++x) {
        const int xx = x < sz ? x : sz - 1;
        const int n1 = lo + xx, n2 = D - n1;
        const int ad = (unsigned(d[it][1 + (x >> 1)]) >> (16 * (x & 1))) & 0xffff;
        zc z = TH[x < sz ? ad : thz];  // beyond sz: the zero slot
        if (PRE == 1) z = cmul(z, UFF[n1 * p + n2]);
        if (PRE == 2) z = cmul(z, UF[n2]);
        const zc gx = g[xx];
        cacc(acc, gx, z);
      }
      if (POST == 1) acc = cmul(acc, UTT[a1 * p + a2]);
      if (POST == 2) acc = cmul(acc, UT[a2]);
      if (e < nth) TG[e] = acc;
    }
  }
  // single-site matricisation (gauge moves): M[e] = A[src[e]]
  __device__ OCG_INLINE void matcopy(const LDS int* oh) {
    using namespace fastp;
    pf(7);
    const int nth = uni(oh[kOhNth]);
    if (nth <= 64) matcopy_it<1>(oh, nth);
    else matcopy_it<kItTh>(oh, nth);
    wsync();
  }
  template <int IT>
  __device__ OCG_INLINE void matcopy_it(const LDS int* oh, int nth) {
    using namespace fastp;
    const LDS int* src = PL + uni(oh[kOhMat]);
    int s[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int e = lane + 64 * it;
      s[it] = src[e < nth ? e : nth - 1];
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int e = lane + 64 * it;
      const zc v = MP[s[it]];
      if (e < nth) TH[e] = v;
    }
  }

  // ------------------------------------------------------------- decomposition
  // Block decomposition of M (ITensor denmatDecomp per QN block, global
  // truncation): Gram on the smaller side of each block, register Jacobi for
  // orders 2..4, the truncation rule, factors into their destinations; the
  // rewritten bond's dims.  normalize: the norm-carrying factor divided by
  // sqrt(kept weight) (doStep's centre normalisation).
  __device__ OCG_INLINE void decompose(const LDS int* oh, lzp M, int dir, double cutoff, int maxm, bool normalize) {
    using namespace fastp;
    pf(2);
    // the op header in one batch of loads (every field wave-uniform), then every
    // per-lane table entry the decomposition reads, before any arithmetic: the
    // group descriptors, order-1 sectors, eigen slots, the rewritten bond's
    // sectors and their current dims, the factor descriptors
    const i4 h2 = ld4(oh + 8), h3 = ld4(oh + 12), h4 = ld4(oh + 16), h5 = ld4(oh + 20);
    const int newb = uni(oh[kOhNewBond]);
    const int nsec = uni(h2[kOhNsec - 8]), T = uni(h2[kOhT - 8]), maxr = uni(h3[kOhMaxr - 12]),
              no1 = uni(h3[kOhNo1 - 12]), o_o1 = uni(h3[kOhO1 - 12]), o_eq = uni(h4[kOhEq - 16]),
              o_secq = uni(h4[kOhSecQ - 16]), o_f = uni(h4[kOhF - 16]), nf = uni(h4[kOhNf - 16]),
              dot = uni(h5[kOhDot - 20]);
    const int g = lane >> 4, i = (lane >> 2) & 3, j = lane & 3, rb = lane & ~15;
    const i4 ga = ld4(oh + kOhGrp + 8 * g), gb = ld4(oh + kOhGrp + 8 * g + 4);
    const i4 o1 = ld4(PL + o_o1 + 4 * (lane < no1 ? lane : 0));
    const bool ae = lane < T;
    const i4 eq = ld4(PL + o_eq + 4 * (ae ? lane : 0));
    const int sqe = PL[o_secq + (lane < nsec ? lane : 0)];  // q | eigen offset << 8 | n << 16
    const int at_q = newb * P.Q1 + (sqe & 255);
    const int dold = DIM[at_q];
    // ---- Gram of the Jacobi groups: lane 16 g + 4 i + j holds G[i][j]
    const bool used = ga[0] >= 0;
    const int n = used ? ga[1] : 0, side = ga[2], tho = ga[3], R = gb[0], C = gb[1], eoff = gb[2];
    const bool valid = i < n && j < n;
    // order-1 sectors (lanes < no1): the block's one row / column squared norm
    // G[i][j] = sum_c a_c conj(b_c) on either side (cols side: the conjugate of
    // that sum); the loop is unrolled to the op's longest dot product (header,
    // uniform), indices beyond a block's length read the zero slot
    zc gv = c2(0.0, 0.0);
    double lam1 = 0.0;
    {
      const int len = used ? (side == 0 ? C : R) : 0, st = side == 0 ? 1 : C;
      const int bi = side == 0 ? tho + (i < n ? i : 0) * C : tho + (i < n ? i : 0);
      const int bj = side == 0 ? tho + (j < n ? j : 0) * C : tho + (j < n ? j : 0);
      const int len1 = lane < no1 ? o1[1] : 0, b1 = o1[0], s1 = o1[2];
      switch ((dot + 1) >> 1) {  // unrolled to the even bound above the op's longest dot
        case 0: case 1: gram_dots<2>(M, len, st, bi, bj, len1, b1, s1, gv, lam1); break;
        case 2: gram_dots<4>(M, len, st, bi, bj, len1, b1, s1, gv, lam1); break;
        case 3: gram_dots<6>(M, len, st, bi, bj, len1, b1, s1, gv, lam1); break;
        case 4: gram_dots<8>(M, len, st, bi, bj, len1, b1, s1, gv, lam1); break;
        case 5: gram_dots<10>(M, len, st, bi, bj, len1, b1, s1, gv, lam1); break;
        case 6: gram_dots<12>(M, len, st, bi, bj, len1, b1, s1, gv, lam1); break;
        case 7: gram_dots<14>(M, len, st, bi, bj, len1, b1, s1, gv, lam1); break;
        default: gram_dots<kMaxDot>(M, len, st, bi, bj, len1, b1, s1, gv, lam1); break;
      }
      if (side == 1) gv.y = -gv.y;
    }
    if (!valid) gv = c2(0.0, 0.0);
    zc w = c2(i == j ? 1.0 : 0.0, 0.0);
    pf(3);
    if (maxr > 0) jacobi(gv, w, valid, i, j, rb, n, maxr);
    cnt(22, 1.0);
    pf(4);
    // eigenvectors and eigenvalues (clamped at 0) to LDS
    if (used) WB[16 * g + 4 * i + j] = w;
    if (valid && i == j) LAM[eoff + i] = gv.x > 0 ? gv.x : 0.0;
    if (lane < no1) LAM[o1[3]] = lam1;
    wsync();
    // ---- truncation (Chain::decompose, one-wave form): eigen slot e = lane
    const double lam = ae ? LAM[lane] : 0.0;
    const int i_e = eq[1], eo_e = eq[2], n_e = eq[3] & 255, bound = unsigned(eq[3]) >> 8;
    // rank inside the block (descending, ties by index)
    // (all partner values fetched first; non-short-circuit predicates keep the
    // compares free of branches, so the four exchanges are in flight together)
    double lt[kMaxGram];
#pragma unroll
    for (int t = 0; t < kMaxGram; ++t) lt[t] = CH::bperm(lam, ((eo_e + t) & 63) << 2);
    int jb = 0;
#pragma unroll
    for (int t = 0; t < kMaxGram; ++t)
      jb += (ae & (t < n_e) & (t != i_e) & ((lt[t] > lam) | ((lt[t] == lam) & (t < i_e)))) ? 1 : 0;
    const double total = wsum(lam);
    const double cut = cutoff * total, floor_ = 1e-30 * total;
    bool disc = false;
    if (T <= maxm) {
      // Maxm cannot bind: only eigenvalues below max(cut, floor) can be discarded
      const double thr = fmax(cut, floor_);
      const bool small = ae && (lam < thr || lam <= floor_);
      unsigned long long Mk = __ballot(small);
      pf(18);
      cnt(17, __popcll(Mk));
      if (Mk) {
        const int nbig = T - __popcll(Mk);
        double S = lam;
        int rs = 0;
        while (Mk) {
          const int f = __ffsll((long long)Mk) - 1;
          Mk &= Mk - 1;
          const double lf = rdlane(lam, f);
          rs += (lf > lam || (lf == lam && f < lane)) ? 1 : 0;
          if (f != lane && (lf < lam || (lf == lam && f > lane))) S += lf;
        }
        disc = small && nbig + rs >= 1 && (S < cut || lam <= floor_);
      }
    } else {
      // global rank (descending; ties by slot), then the sorted spectrum's suffix sums
      int rk = 0;
      for (int f = 0; f < T; ++f) {
        const double lf = rdlane(lam, f);
        rk += (lf > lam || (lf == lam && f < lane)) ? 1 : 0;
      }
      // lane T-1-rk receives lam: lanes ascend from the smallest
      const int dst = ((T - 1 - rk) & 63) << 2;
      const long long lb = __double_as_longlong(lam);
      const unsigned lo = unsigned(__builtin_amdgcn_ds_permute(dst, int(lb)));
      const unsigned hi = unsigned(__builtin_amdgcn_ds_permute(dst, int(lb >> 32)));
      const double v = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
      const int jpos = T - 1 - lane;  // sorted position of the value lane holds
      const double vv = lane < T ? v : 0.0;
      const double suf = wscan(vv);
      const bool d2 = lane < T && jpos >= 1 && (jpos >= maxm || suf < cut || vv <= floor_);
      // discarded positions are a suffix of the sorted order: m = kept count
      const int m = T - __popcll(__ballot(d2));
      disc = ae && rk >= m;
    }
    pf(16);
    const bool kept = ae && !disc && jb < bound;
    if (kept) {
      const double sq = sqrt(lam);
      WIDX[eo_e + jb] = i_e;
      SIG[eo_e + jb] = sq;
      SIGI[eo_e + jb] = sq > 0 ? 1.0 / sq : 0.0;  // the factors' 1 / sigma, once per eigenvalue
    }
    const double kw = wsum(kept ? lam : 0.0);
    {
      // kept count of sector s = lane: the kept bits of its eigen slots
      // [eoff, eoff + n) (consecutive, in sector order)
      const unsigned long long K = __ballot(kept);
      const int eo = (sqe >> 8) & 255, ns = (sqe >> 16) & 15;
      const int kq = __popcll((K >> eo) & ((1ull << ns) - 1));
      bool changed = false;
      if (lane < nsec) {
        changed = dold != kq;
        KQ[lane] = kq;
        DIM[at_q] = kq;
      }
      if (__ballot(changed)) ++dims_epoch;
    }
    wsync();
    pf(5);
    // ---- factors (Chain::decompose's materialisation): X rows, Y cols
    const double inv = (normalize && kw > 1e-32) ? 1.0 / sqrt(kw) : 1.0;
    if (nf <= 64) factors<1>(o_f, nf, M, dir, inv);
    else if (nf <= 128) factors<2>(o_f, nf, M, dir, inv);
    else if (nf <= 192) factors<3>(o_f, nf, M, dir, inv);
    else factors<kItF>(o_f, nf, M, dir, inv);
  }

  // factor elements (IF 64-element iterations; the op's count picks the instance)
  template <int IF>
  __device__ OCG_INLINE void factors(int o_f, int nf, lzp M, int dir, double inv) {
    using namespace fastp;
    i4 fd[IF];
#pragma unroll
    for (int it = 0; it < IF; ++it) {
      const int e = lane + 64 * it;
      fd[it] = ld4(PL + o_f + 4 * (e < nf ? e : nf - 1));
    }
    // operands in two dependent waves of loads, all elements at once: (KQ, WIDX,
    // SIG, the M terms), then the eigenvector entries W[., wv]; branch-free
    // (an exact factor is a selected entry of W, a derived one sum_x M W)
    int kqs[IF], wvv[IF];
    double sg[IF], isg[IF];
    zc mv[IF][kMaxGram];
#pragma unroll
    for (int it = 0; it < IF; ++it) {
      const int w0 = fd[it][0], w1 = fd[it][1], w2 = fd[it][2];
      const int s = (w0 >> 16) & 15, jj = (w0 >> 20) & 15, eo = w2 & 255;
      const bool exact = (w2 >> 12) & 1;
      const int mb = w1 & 0xffff, terms = (w1 >> 16) & 31, ms = unsigned(w1) >> 21;
      kqs[it] = KQ[s];
      wvv[it] = WIDX[eo + jj];
      sg[it] = SIG[eo + jj];
      isg[it] = SIGI[eo + jj];
#pragma unroll
      for (int x = 0; x < kMaxGram; ++x) mv[it][x] = M[(exact || x >= terms) ? thz : mb + x * ms];
    }
    zc out[IF];
    int dst[IF];
#pragma unroll
    for (int it = 0; it < IF; ++it) {
      const int e = lane + 64 * it;
      const int w0 = fd[it][0], w1 = fd[it][1], w2 = fd[it][2], wbse = fd[it][3];
      const int dest = w0 & 0xffff, jj = (w0 >> 20) & 15;
      const bool isx = (w0 >> 24) & 1, scr = (w0 >> 25) & 1;
      const bool exact = (w2 >> 12) & 1;
      const int terms = exact ? 1 : (w1 >> 16) & 31;
      const int tc = terms > 0 ? terms - 1 : 0;
      const bool live = jj < kqs[it] && e < nf;
      const int wvc = live ? wvv[it] : 0;
      const int base = exact ? w1 : wbse;  // an order-1 sector points at the unit slot WB[64]
      const double cs = isx ? 1.0 : -1.0;  // w (Θ w) or conj(w) (w^H Θ)
      zc wp[kMaxGram];
#pragma unroll
      for (int x = 0; x < kMaxGram; ++x) {
        const zc t = WB[base + 4 * (x < tc ? x : tc) + wvc];
        wp[x] = c2(t.x, cs * t.y);
      }
      zc acc = c2(0.0, 0.0);
#pragma unroll
      for (int x = 0; x < kMaxGram; ++x) cacc(acc, mv[it][x], wp[x]);  // beyond terms: the zero slot
      // exact: the selected entry of W, times sigma / sqrt(kept weight) on the
      // norm-carrying side; derived: divided by sigma on the orthonormal side
      const double sig = sg[it];
      const zc we = wp[0];
      const bool scl = isx ? dir == kFromright : dir == kFromleft;
      const bool orth = isx ? dir == kFromleft : dir == kFromright;
      const double f = exact ? (scl ? sig * inv : 1.0) : (orth ? (sig > 0 ? isg[it] : 0.0) : inv);
      const zc r = cscale(exact ? we : acc, f);
      out[it] = live ? r : c2(0.0, 0.0);
      dst[it] = e < nf ? (dest | (scr ? 0x10000 : 0)) : -1;
    }
    pf(23);
#pragma unroll
    for (int it = 0; it < IF; ++it)
      if (dst[it] >= 0) ((dst[it] >> 16) ? XS : MP)[dst[it] & 0xffff] = out[it];
    wsync();
  }

  template <int K>
  __device__ __forceinline__ void gram_dots(lzp M, int len, int st, int bi, int bj, int len1, int b1, int s1, zc& gv,
                                            double& lam1) const {
    zc a[K], b[K], z[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
      const bool in = c < len, in1 = c < len1;
      a[c] = M[in ? bi + c * st : thz];
      b[c] = M[in ? bj + c * st : thz];
      z[c] = M[in1 ? b1 + c * s1 : thz];
    }
#pragma unroll
    for (int c = 0; c < K; ++c) {
      cacc(gv, a[c], cconj(b[c]));
      lam1 += cabs2(z[c]);
    }
  }

  // The rotation of the pair this lane holds (CH::jrot_fast's formulas, the
  // identity when !live), returned as this lane's role coefficients: index p
  // (up): J[p][p] = c, J[q][p] = -s e*, shift -sh; index q: J[q][q] = c e*,
  // J[p][q] = s, shift +sh.  The rare power-of-two rescale runs only when some
  // lane needs it (sc = 1 otherwise: the same bits as without it).
  __device__ __forceinline__ void jrot_role(zc bv, double app, double aqq, bool live, bool up, zc& jd, zc& jo,
                                            double& ds) const {
    const double mb = fmax(fabs(bv.x), fabs(bv.y)), sz = fabs(app) + fabs(aqq);
    const bool resc = live && (mb < 1e-120 || mb > 1e120 || sz > 1e120);
    double sc = 1.0;
    if (__ballot(resc)) {
      sc = resc ? ldexp(1.0, -ilogb(fmax(mb, sz))) : 1.0;
      bv = cscale(bv, sc);
      app *= sc;
      aqq *= sc;
    }
    const double r2 = live ? bv.x * bv.x + bv.y * bv.y : 1.0;
    const double rinv = CH::rsq_ref(r2), r = r2 * rinv;
    const double D = aqq - app, sg = D >= 0 ? 1.0 : -1.0;
    const double x = fma(D, D, 4.0 * r2);
    const double E = fabs(D) + x * CH::rsq_ref(x);
    const double h = CH::rsq_ref(fma(E, E, 4.0 * r2));
    const double c = E * h, s = sg * 2.0 * r * h;
    const double ex = bv.x * rinv, ey = bv.y * rinv;
    const double sh = sg * 2.0 * r2 * CH::rcp_ref(E * sc);
    jd = up ? c2(c, 0.0) : c2(ex * c, -ey * c);
    jo = up ? c2(ex * -s, -ey * -s) : c2(s, 0.0);
    ds = up ? -sh : sh;
    jd = live ? jd : c2(1.0, 0.0);
    jo = live ? jo : c2(0.0, 0.0);
    ds = live ? ds : 0.0;
  }

  // register Jacobi on up to four Gram blocks of order <= 4 (Chain::jacobi_reg<4>):
  // lane 16 g + 4 i + j holds G[i][j] and W[i][j] of group g; round r pairs
  // x with x ^ (r + 1), partner elements by DPP, rotations by bpermute.  The
  // lane also carries the diagonal entries of its row and column (di, dj),
  // updated by the rotations' shifts, so a round needs no diagonal gather.
  __device__ OCG_INLINE void jacobi(zc& g, zc& w, bool valid, int i, int j, int rb, int n, int maxr) {
    auto at = [&](int r, int c) { return (rb + r * 4 + c) << 2; };
    double di = CH::bperm(g.x, at(i, i)), dj = CH::bperm(g.x, at(j, j));
    // Lane (x, y) publishes the rotation coefficients of index x in the pair
    // (x, y): J[x][x] and J[y][x].  A reader takes its column's from lane
    // (j, pj) and its row's from lane (i, pi) -- the pivot (p, q) for p, its
    // mirror (q, p) for q, a diagonal lane (identity) for an unpaired index.  The
    // mirror evaluates the pivot's rotation from the pivot's own element (the
    // DPP partner g11 = g[p][q] of this round) and the same diagonal pair, so
    // both roles use one rotation, bit for bit; no reader selects a role.
    int arow[3], acol[3];
    bool zp[3];
#pragma unroll
    for (int rnd = 0; rnd < 3; ++rnd) {
      const int k = rnd + 1;
      int pi = i, pj = j;
      if (rnd < maxr && valid) {
        if ((i ^ k) < n) pi = i ^ k;
        if ((j ^ k) < n) pj = j ^ k;
      }
      arow[rnd] = at(i, pi);
      acol[rnd] = at(j, pj);
      zp[rnd] = pi == j && i != j;  // the lane holds its own pair's off-diagonal
    }
    const bool up = i < j, dg = i == j;
    int sweep = 0, nr = 0;
    bool done = false;
    for (; sweep < 40; ++sweep) {
      bool flag = false;
#pragma unroll
      for (int rnd = 0; rnd < 3; ++rnd) {
        if (rnd >= maxr) break;
        if (__ballot(valid && up && CH::jneed(cabs2(g), di, dj)) == 0) {
          done = true;
          break;
        }
        ++nr;
        const zc g01 = CH::xcol(g, rnd), g10 = CH::xrow(g, rnd);
        const zc g11 = CH::xrow(g01, rnd), w1 = CH::xcol(w, rnd);
        const zc bv = up ? g : g11;  // the pivot element g[p][q] (for the mirror: its DPP partner)
        const double app = up ? di : dj, aqq = up ? dj : di;
        const bool need = CH::jneed(cabs2(bv), app, aqq);
        zc jd, jo;
        double ds;
        jrot_role(bv, app, aqq, need && !dg, up, jd, jo, ds);
        const zc jdc = CH::bpermz(jd, acol[rnd]), joc = CH::bpermz(jo, acol[rnd]);
        const zc jdr = CH::bpermz(jd, arow[rnd]), jor = CH::bpermz(jo, arow[rnd]);
        const double dsc = CH::bperm(ds, acol[rnd]), dsr = CH::bperm(ds, arow[rnd]);
        // W' = W J, G' = J^H G J on the 2 x 2 super-block of (i, pi) x (j, pj)
        zc wn = cmul(w, jdc);
        cacc(wn, w1, joc);
        zc r0 = cmul(g, jdc);
        cacc(r0, g01, joc);
        zc r1 = cmul(g10, jdc);
        cacc(r1, g11, joc);
        zc out = cjmul(jdr, r0);
        cjacc(out, jor, r1);
        // the diagonal entries of this lane's row and column after the rotation
        const double dj2 = dj + dsc, di2 = di + dsr;
        out = (zp[rnd] && need) ? c2(0.0, 0.0) : out;  // the rotated pair: exact zero
        out = dg ? c2(dj2, 0.0) : out;                  // a diagonal entry: the shifted value
        if (rnd == maxr - 1) flag = valid && up && CH::jneed(cabs2(out), di2, dj2);
        g = out;
        w = wn;
        di = di2;
        dj = dj2;
      }
      if (done || __ballot(flag) == 0) break;
    }
    if (sweep == 40 && lane == 0 && P.err) atomicOr(P.err, OCG_ERR_JACOBI);
    cnt(21, 1.0);
    cnt(20, double(sweep + 1));
    cnt(30, double(nr));
#ifdef OCG_FAST_TRACE  // CPU emulation diagnostics (tests/emu, EXTRA=-DOCG_FAST_TRACE)
    if (lane == 0) printf("[jacobi] op %d sweeps %d rounds %d\n", trace_op, sweep + 1, nr);
#endif
  }

  // ------------------------------------------------------------- gauge neighbour
  // right move: A_{k+1} <- Y A_{k+1}; left move: A_{k-1} <- A_{k-1} X (XS holds the factor)
  __device__ OCG_INLINE void neighbour(const LDS int* oh) {
    using namespace fastp;
    pf(25);
    const int ns = uni(oh[kOhNs]), kind = uni(oh[kOhKind]);
    if (ns <= 64) neighbour_it<1>(oh, ns, kind);
    else if (ns <= 128) neighbour_it<2>(oh, ns, kind);
    else neighbour_it<kItS>(oh, ns, kind);
  }
  template <int IT>
  __device__ OCG_INLINE void neighbour_it(const LDS int* oh, int ns, int kind) {
    using namespace fastp;
    const LDS int* sl = PL + uni(oh[kOhS]);
    i4 d[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int e = lane + 64 * it;
      d[it] = ld4(sl + 4 * (e < ns ? e : ns - 1));
    }
    zc acc[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int x1 = d[it][0] & 0xffff, x2 = unsigned(d[it][0]) >> 16, len = d[it][1] & 0xffff,
                s2 = unsigned(d[it][1]) >> 16;
      const int lc = len > 0 ? len - 1 : 0;
      acc[it] = c2(0.0, 0.0);
#pragma unroll
      for (int b = 0; b < kMaxDm; ++b) {
        const int bb = b < lc ? b : lc;
        const bool in = b < len;  // beyond len: the zero slot of the first operand's buffer
        const zc a = (kind == kOpGaugeR) ? zc(XS[in ? x1 + b : xsz]) : zc(MP[in ? x1 + b : np]);
        const zc v = (kind == kOpGaugeR) ? zc(MP[x2 + bb * s2]) : zc(XS[x2 + bb * s2]);
        cacc(acc[it], a, v);
      }
    }
    wsync();
#pragma unroll
    for (int it = 0; it < IT; ++it)
      if (lane + 64 * it < ns) MP[d[it][2]] = acc[it];
    wsync();
  }

  // sin / cos of |x| <= pi/4 by their Taylor series through x^17 / x^16 (the
  // next terms are below 1e-17): the step's phase arguments |u dt n(n-1)/4| are
  // far inside that for the controls of the reference's drivers; larger ones take
  // libm's sincos (uniform branch in step)
  __device__ __forceinline__ static void sincos_q(double x, double& s, double& c) {
    constexpr double s3 = -1.0 / 6.0, s5 = 1.0 / 120.0, s7 = -1.0 / 5040.0, s9 = 1.0 / 362880.0,
                     s11 = -1.0 / 39916800.0, s13 = 1.0 / 6227020800.0, s15 = -1.0 / 1307674368000.0,
                     s17 = 1.0 / 355687428096000.0;
    constexpr double c2_ = -0.5, c4 = 1.0 / 24.0, c6 = -1.0 / 720.0, c8 = 1.0 / 40320.0, c10 = -1.0 / 3628800.0,
                     c12 = 1.0 / 479001600.0, c14 = -1.0 / 87178291200.0, c16 = 1.0 / 20922789888000.0;
    const double z = x * x;
    const double ps = fma(z, fma(z, fma(z, fma(z, fma(z, fma(z, fma(z, s17, s15), s13), s11), s9), s7), s5), s3);
    const double pc = fma(z, fma(z, fma(z, fma(z, fma(z, fma(z, fma(z, c16, c14), c12), c10), c8), c6), c4), c2_);
    s = fma(x * z, ps, x);
    c = fma(z, pc, 1.0);
  }

  // ------------------------------------------------------------- step
  // BH_tDMRG::step (src/BH_tDMRG.cpp:111-125) + doStep (:127-230), as Chain::step
  // (final_gauge = false: the closing position(1) is skipped, the centre stays on
  // the last gate's left site, which is normalised instead of site 1).
  __device__ OCG_INLINE void step(double ufrom, double uto, int forward, bool final_gauge = true) {
    using namespace fastp;
    if (!act) return;
    pf(29);
    const int p = P.p;
    const double tau = forward ? P.dt : -P.dt;
    // U phases exp(-i u tau n(n-1) / 4) (initUGates, :74-108): lane < p the
    // single-site UF[n], UT[n]; lane < p^2 the pair products UF[n1] UF[n2],
    // UT[a1] UT[a2] as the phase of the summed argument -- all in registers, one
    // LDS write and one wave fence
    {
      const double ta = -0.25 * tau;
      const int a = lane / p, b = lane - a * p;
      const double n1 = lane < p ? double(lane) * double(lane - 1) : 0.0;
      const double n2 = lane < p * p ? double(a) * double(a - 1) + double(b) * double(b - 1) : 0.0;
      const double xf1 = ta * ufrom * n1, xt1 = ta * uto * n1, xf2 = ta * ufrom * n2, xt2 = ta * uto * n2;
      const bool big = fmax(fmax(fabs(xf1), fabs(xt1)), fmax(fabs(xf2), fabs(xt2))) > 0.78;
      double sf1, cf1, st1, ct1, sf2, cf2, st2, ct2;
      if (__ballot(big) == 0) {
        sincos_q(xf1, sf1, cf1);
        sincos_q(xt1, st1, ct1);
        sincos_q(xf2, sf2, cf2);
        sincos_q(xt2, st2, ct2);
      } else {
        sincos(xf1, &sf1, &cf1);
        sincos(xt1, &st1, &ct1);
        sincos(xf2, &sf2, &cf2);
        sincos(xt2, &st2, &ct2);
      }
      if (lane < p) {
        PH[lane] = c2(cf1, sf1);
        PH[p + lane] = c2(ct1, st1);
      }
      if (lane < p * p) {
        PH[2 * p + lane] = c2(cf2, sf2);
        PH[2 * p + p * p + lane] = c2(ct2, st2);
      }
    }
    ph_u = uto;
    ph_dir = forward;
    wsync();
    for (int o = 0; o < nops; ++o) {
      const LDS int* oh = PL + PL[kHOps + o];
      const i4 h0 = ld4(oh), h1 = ld4(oh + 4);
      if (uni(h1[1]) && !final_gauge) continue;  // closing move
      const int kind = uni(h0[0]), dir = uni(h0[2]);
      trace_op = o;
      if (kind == kOpGate) {
        pf(12);
        model_gate(o, uni(h0[1]));
        theta(oh);
        gate(oh, forward);
        decompose(oh, TG, dir, P.cutoff, P.maxm, true);
      } else {
        matcopy(oh);
        decompose(oh, TH, dir, OCG_GAUGE_CUTOFF, 1 << 30, false);
        neighbour(oh);
      }
    }
    // lonely U_to on site 1 (:222-223), then psi.normalize() (:228): the norm of
    // the MPS is the norm of the centre site
    pf(9);
    const int centre = final_gauge ? 1 : centre_open;
    const int s1a = PL[o_site + 1], s1b = PL[o_site + 2];
    for (int x = s1a + lane; x < s1b; x += 64) MP[x] = cmul(MP[x], PH[p + PL[o_siten + x - s1a]]);
    wsync();
    const int ca = PL[o_site + centre], cb = PL[o_site + centre + 1];
    double acc = 0.0;
    zc v[kItMps];
#pragma unroll
    for (int it = 0; it < kItMps; ++it) {
      const int x = ca + lane + 64 * it;
      v[it] = MP[x < cb ? x : ca];
      if (x < cb) acc += cabs2(v[it]);
    }
    const double n2 = wsum(acc);
    if (n2 > 0) {
      const double f = 1.0 / sqrt(n2);
#pragma unroll
      for (int it = 0; it < kItMps; ++it) {
        const int x = ca + lane + 64 * it;
        if (x < cb) MP[x] = cscale(v[it], f);
      }
    }
    wsync();
  }
};

}  // namespace ocg
