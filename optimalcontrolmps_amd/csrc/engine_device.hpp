// MI355X (gfx950) device side of the tDMRG chain engine.
//
// Restates, per workgroup and entirely in LDS, the arithmetic of
//   BH_tDMRG::step / doStep           (reference src/BH_tDMRG.cpp:111-230)
//   ITensor denmatDecomp per QN block (called at src/BH_tDMRG.cpp:178,191,209)
//   MPS::position / normalize         (src/BH_tDMRG.cpp:187,198,217,228)
//   exactApplyMPO(propDeriv, psi)     (src/OptimalControl.cpp:256,302)
//   overlapC(psi, phi) / overlapC(psi, H, phi)  (src/OptimalControl.cpp:242,261,272,412)
// on U(1) ("Nb") block-sparse tensors stored compactly per site.
//
// Layout of one MPS (HBM slot and LDS copy alike):
//   dims[b*Q1 + q]  (int)   bond b = 0..L, sector q = left particle count
//   data            (zc) site k occupies [site_base[k], +site_cap[k]);
//                   inside it blocks (q, n) (rows dims[k-1][q], cols
//                   dims[k][q+n]) are packed row-major in (q, n) order.
#pragma once

#include <hip/hip_runtime.h>

#include "engine.hpp"

#ifndef OCG_INLINE
#define OCG_INLINE __attribute__((always_inline))
#endif

namespace ocg {

// ---------------------------------------------------------------- complex
// POD complex double (same layout as HIP double2) so it can live behind
// address-space-3 (LDS) pointers: 32-bit addresses and ds_* instructions.
struct __attribute__((aligned(16))) zc {
  double x, y;
};
#define LDS __attribute__((address_space(3)))
__host__ __device__ __forceinline__ zc c2(double x, double y) { zc r; r.x = x; r.y = y; return r; }

// LDS complex buffers: an address-space-3 double* (32-bit addresses, ds_*
// instructions) with complex element access through a converting reference
// (clang does not let struct copy/assign operate through AS3 pointers).
struct lref {
  LDS double* p;
  __device__ __forceinline__ operator zc() const { return c2(p[0], p[1]); }
  __device__ __forceinline__ const lref& operator=(const zc& v) const { p[0] = v.x; p[1] = v.y; return *this; }
  __device__ __forceinline__ const lref& operator=(const lref& o) const {
    double a = o.p[0], b = o.p[1];
    p[0] = a; p[1] = b;
    return *this;
  }
};
struct lzp {
  LDS double* p;
  __device__ __forceinline__ lref operator[](int i) const { return lref{p + 2 * i}; }
  __device__ __forceinline__ lzp operator+(int i) const { return lzp{p + 2 * i}; }
  __device__ __forceinline__ bool operator==(const lzp& o) const { return p == o.p; }
};
__device__ __forceinline__ zc cadd(zc a, zc b) { return c2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ zc csub(zc a, zc b) { return c2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ zc cmul(zc a, zc b) {
  return c2(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}
// conj(a) * b
__device__ __forceinline__ zc cjmul(zc a, zc b) {
  return c2(fma(a.x, b.x, a.y * b.y), fma(a.x, b.y, -a.y * b.x));
}
__device__ __forceinline__ zc cscale(zc a, double s) { return c2(a.x * s, a.y * s); }
__device__ __forceinline__ zc cconj(zc a) { return c2(a.x, -a.y); }
__device__ __forceinline__ void cacc(zc& acc, zc a, zc b) {  // acc += a*b
  acc.x = fma(a.x, b.x, fma(-a.y, b.y, acc.x));
  acc.y = fma(a.x, b.y, fma(a.y, b.x, acc.y));
}
__device__ __forceinline__ void cjacc(zc& acc, zc a, zc b) {  // acc += conj(a)*b
  acc.x = fma(a.x, b.x, fma(a.y, b.y, acc.x));
  acc.y = fma(a.x, b.y, fma(-a.y, b.x, acc.y));
}
__device__ __forceinline__ double cabs2(zc a) { return a.x * a.x + a.y * a.y; }

// ---------------------------------------------------------------- LDS map
struct LdsLayout {
  // complex buffers (offsets in zc units)
  int A, TH, G, G2, W, W2, X, Y, CR, S, GT, PH, ROT;
  int ncplx;
  // double buffers (offsets in doubles, after the complex region)
  int LAM, PP, RED, SCAL, PROF;
  int ndbl;
  // int buffers (offsets in ints, after the double region)
  int DIMS, MD, BOFF, BOFFT, THR, THC, THO, THRO, THCO, NQ, SIDE, GOFF, EOFF, MQ, POFF, KEPT, XOFF, YOFF, RANK,
      KIDX, PART, ROLE, PAIR, CDIM, COLD, COFF, ISCAL;
  int nint;
  int bytes;
};

__host__ __device__ inline LdsLayout lds_layout(const OcgParams& P, int nt) {
  LdsLayout l;
  int c = 0;
  l.A = c; c += P.cap;
  l.TH = c; c += P.thcap;
  l.G = c; c += P.thcap;
  l.G2 = c; c += P.thcap;
  l.W = c; c += P.thcap;
  l.W2 = c; c += P.thcap;
  l.X = c; c += P.thcap;
  l.Y = c; c += P.thcap;
  l.CR = c; c += P.thcap;
  l.S = c; c += P.max_site_cap;
  l.GT = c; c += 2 * P.gtotal;
  l.PH = c; c += 2 * P.p;
  l.ROT = c; c += 2 * P.nrot + 2;
  l.ncplx = c;
  int d = 0;
  l.LAM = d; d += P.evcap;
  l.PP = d; d += P.evcap;
  l.RED = d; d += nt;
  l.SCAL = d; d += 16;
  l.PROF = d; d += 32;
  l.ndbl = d;
  int i = 0;
  int Q1 = P.Q1, p = P.p;
  l.DIMS = i; i += P.nsq;
  l.MD = i; i += 2 * P.nsq;
  l.BOFF = i; i += P.L * Q1 * p;
  l.BOFFT = i; i += Q1 * p;
  l.THR = i; i += Q1;
  l.THC = i; i += Q1;
  l.THO = i; i += Q1 + 1;
  l.THRO = i; i += Q1 * p;
  l.THCO = i; i += Q1 * p;
  l.NQ = i; i += Q1;
  l.SIDE = i; i += Q1;
  l.GOFF = i; i += Q1 + 1;
  l.EOFF = i; i += Q1 + 1;
  l.MQ = i; i += Q1;
  l.POFF = i; i += Q1 + 1;
  l.KEPT = i; i += Q1;
  l.XOFF = i; i += Q1 + 1;
  l.YOFF = i; i += Q1 + 1;
  l.RANK = i; i += P.evcap;
  l.KIDX = i; i += P.evcap;
  l.PART = i; i += P.evcap;
  l.ROLE = i; i += P.evcap;
  l.PAIR = i; i += P.evcap;
  l.CDIM = i; i += Q1 + 1;
  l.COLD = i; i += Q1 + 1;
  l.COFF = i; i += Q1 + 1;
  l.ISCAL = i; i += 16;
  l.nint = i;
  l.bytes = l.ncplx * 16 + l.ndbl * 8 + l.nint * 4;
  return l;
}

enum { kFromleft = 0, kFromright = 1 };

// scalar slots
enum { S_TOTAL = 0, S_KEPTW = 1, S_NORM = 2, S_OVRE = 3, S_OVIM = 4, S_FACT = 5 };
enum { I_M = 0, I_MAXROUNDS = 1, I_FLAG0 = 2, I_FLAG1 = 3, I_NBLK = 4, I_EVT = 5, I_XT = 6, I_YT = 7, I_THT = 8,
       I_NPAIR = 9 };

template <int NT>
struct Chain {
  const OcgParams& P;
  int tid;
  lzp A, TH, G, G2, W, W2, X, Y, CR, S, GT, PH, ROT;
  LDS double *LAM, *PP, *RED, *SCAL, *PROF;
  unsigned long long pf_last = 0;
  int pf_cur = 0;
  LDS int *DIMS, *MD, *BOFF, *BOFFT, *THR, *THC, *THO, *THRO, *THCO, *NQ, *SIDE, *GOFF, *EOFF, *MQ, *POFF, *KEPT, *XOFF,
      *YOFF, *RANK, *KIDX, *PART, *ROLE, *PAIR, *CDIM, *COLD, *COFF, *ISCAL;

  __device__ Chain(const OcgParams& P_, char* smem) : P(P_), tid(threadIdx.x) {
    LdsLayout l = lds_layout(P, NT);
    lzp cb{(LDS double*)smem};
    A = cb + l.A; TH = cb + l.TH; G = cb + l.G; G2 = cb + l.G2; W = cb + l.W; W2 = cb + l.W2; X = cb + l.X;
    Y = cb + l.Y; CR = cb + l.CR; S = cb + l.S; GT = cb + l.GT; PH = cb + l.PH; ROT = cb + l.ROT;
    LDS double* db = (cb + l.ncplx).p;
    LAM = db + l.LAM; PP = db + l.PP; RED = db + l.RED; SCAL = db + l.SCAL; PROF = db + l.PROF;
    LDS int* ib = (LDS int*)(db + l.ndbl);
    DIMS = ib + l.DIMS; MD = ib + l.MD; BOFF = ib + l.BOFF; BOFFT = ib + l.BOFFT; THR = ib + l.THR; THC = ib + l.THC;
    THO = ib + l.THO; THRO = ib + l.THRO; THCO = ib + l.THCO; NQ = ib + l.NQ; SIDE = ib + l.SIDE;
    GOFF = ib + l.GOFF; EOFF = ib + l.EOFF; MQ = ib + l.MQ; POFF = ib + l.POFF; KEPT = ib + l.KEPT;
    XOFF = ib + l.XOFF; YOFF = ib + l.YOFF; RANK = ib + l.RANK; KIDX = ib + l.KIDX; PART = ib + l.PART;
    ROLE = ib + l.ROLE; PAIR = ib + l.PAIR; CDIM = ib + l.CDIM; COLD = ib + l.COLD; COFF = ib + l.COFF;
    ISCAL = ib + l.ISCAL;
  }

  __device__ __forceinline__ void sync() { __syncthreads(); }
  // Diagnostic build only (-DOCG_PROFILE): thread 0 charges the shader-clock
  // cycles since the previous stamp to the category that was running.
  // Categories: 0 build_theta 1 apply_gate 2 gram 3 jacobi 4 rank/truncate
  // 5 factors X/Y 6 scatter 7 gauge write-back 8 overlap 9 phases/norms
  // 10 load/store 11 apply_dH zip 12 other.
  __device__ __forceinline__ void pf(int cat) {
#ifdef OCG_PROFILE
    if (tid == 0) {
      unsigned long long t = __builtin_amdgcn_s_memtime();
      if (pf_last) PROF[pf_cur] += double(t - pf_last);
      pf_last = t;
      pf_cur = cat;
    }
#else
    (void)cat;
#endif
  }
  __device__ __forceinline__ int d(int b, int q) const { return (q < 0 || q > P.Q) ? 0 : DIMS[b * P.Q1 + q]; }
  __device__ __forceinline__ int bo(int k, int q, int n) const { return BOFF[((k - 1) * P.Q1 + q) * P.p + n]; }
  __device__ __forceinline__ lzp site(int k) { return A + P.site_base[k]; }

  // ------------------------------------------------------------- tables
  // block offsets of site k from the current dims (single thread)
  __device__ OCG_INLINE int site_offsets_serial(int k, LDS int* out) const {
    int off = 0;
    for (int q = 0; q < P.Q1; ++q)
      for (int n = 0; n < P.p; ++n) {
        int r = d(k - 1, q), c = (q + n <= P.Q) ? d(k, q + n) : 0;
        if (r > 0 && c > 0) { out[q * P.p + n] = off; off += r * c; }
        else out[q * P.p + n] = -1;
      }
    return off;
  }
  __device__ OCG_INLINE void all_offsets() {  // parallel over sites
    for (int k = 1 + tid; k <= P.L; k += NT) site_offsets_serial(k, BOFF + (k - 1) * P.Q1 * P.p);
  }
  // (q, local) of the idx-th state of bond b
  __device__ __forceinline__ void bond_split(int b, int idx, int& q, int& loc) const {
    int acc = 0;
    for (q = 0; q < P.Q1; ++q) {
      int dq = DIMS[b * P.Q1 + q];
      if (idx < acc + dq) { loc = idx - acc; return; }
      acc += dq;
    }
    q = -1; loc = -1;
  }
  __device__ __forceinline__ int bond_dim(int b) const {
    int s = 0;
    for (int q = 0; q < P.Q1; ++q) s += DIMS[b * P.Q1 + q];
    return s;
  }
  // segment lookup in a (Q1 x p) offset table: find n with off[n] <= r < off[n] + len(n)
  __device__ __forceinline__ int seg_find(const LDS int* offs, int r) const {
    int best = -1, bo = -1;
    for (int n = 0; n < P.p; ++n) {
      int o = offs[n];
      if (o >= 0 && o <= r && o > bo) { bo = o; best = n; }
    }
    return best;
  }
  // flat element -> block q using prefix table off[0..Q1]
  __device__ __forceinline__ int blk_find(const LDS int* off, int e) const {
    int q = 0;
    while (q + 1 < P.Q1 && off[q + 1] <= e) ++q;
    return q;
  }

  // ------------------------------------------------------------- I/O
  __device__ OCG_INLINE void load(const int* gdims, const zc* gdata) {
    pf(10);
    for (int i = tid; i < P.nsq; i += NT) DIMS[i] = gdims[i];
    for (int i = tid; i < P.cap; i += NT) A[i] = gdata[i];
    sync();
    all_offsets();
    sync();
  }
  __device__ OCG_INLINE void store(int* gdims, zc* gdata) {
    pf(10);
    for (int i = tid; i < P.nsq; i += NT) gdims[i] = DIMS[i];
    for (int k = 1; k <= P.L; ++k) {
      // number of used elements of site k
      int last = 0;
      for (int q = 0; q < P.Q1; ++q)
        for (int n = 0; n < P.p; ++n) {
          int o = bo(k, q, n);
          if (o >= 0) { int e = o + d(k - 1, q) * d(k, q + n); if (e > last) last = e; }
        }
      for (int i = tid; i < last; i += NT) gdata[P.site_base[k] + i] = A[P.site_base[k] + i];
    }
  }
  // gate tables and the per-sector rank bound md[b][q] (Hilbert-space
  // Schmidt-rank bound, capped by Maxm) used to clamp numerically-zero
  // directions out of every decomposition (guards the LDS capacities).
  __device__ OCG_INLINE void load_tables(const zc* gf, const zc* gb, const int* md) {
    for (int i = tid; i < 32; i += NT) PROF[i] = 0.0;
    for (int i = tid; i < P.gtotal; i += NT) { GT[i] = gf[i]; GT[P.gtotal + i] = gb[i]; }
    for (int i = tid; i < 2 * P.nsq; i += NT) MD[i] = md[i];
  }

  // ------------------------------------------------------------- norms
  __device__ OCG_INLINE double block_reduce_sum(double v) {
    RED[tid] = v;
    sync();
    for (int s = NT / 2; s > 0; s >>= 1) {
      if (tid < s) RED[tid] += RED[tid + s];
      sync();
    }
    double r = RED[0];
    sync();
    return r;
  }
  __device__ OCG_INLINE double site_norm2(int k) {
    pf(9);
    int n = P.site_cap[k];
    // sum over used blocks only (unused tail may hold stale data)
    double acc = 0;
    for (int q = 0; q < P.Q1; ++q)
      for (int nn = 0; nn < P.p; ++nn) {
        int o = bo(k, q, nn);
        if (o < 0) continue;
        int sz = d(k - 1, q) * d(k, q + nn);
        for (int i = tid; i < sz; i += NT) acc += cabs2(site(k)[o + i]);
      }
    (void)n;
    return block_reduce_sum(acc);
  }
  __device__ OCG_INLINE void site_scale(int k, double f) {
    for (int i = tid; i < P.site_cap[k]; i += NT) site(k)[i] = cscale(site(k)[i], f);
    sync();
  }
  // multiply site k by a per-physical-index phase table ph[n]
  __device__ OCG_INLINE void site_phase(int k, lzp ph) {
    pf(9);
    for (int q = 0; q < P.Q1; ++q)
      for (int n = 0; n < P.p; ++n) {
        int o = bo(k, q, n);
        if (o < 0) continue;
        int sz = d(k - 1, q) * d(k, q + n);
        zc f = ph[n];
        for (int i = tid; i < sz; i += NT) site(k)[o + i] = cmul(site(k)[o + i], f);
      }
    sync();
  }

  // ------------------------------------------------------------- Θ
  // Two-site tensor for bond (i1, i1+1), blocks by middle QN q:
  //   rows (n1, a in bond i1-1 sector q-n1), cols (n2, c in bond i1+1 sector q+n2)
  __device__ OCG_INLINE void build_theta(int i1) {
    pf(0);
    const int l = i1 - 1, mid = i1, r = i1 + 1, p = P.p;
    if (tid == 0) {
      int off = 0;
      for (int q = 0; q < P.Q1; ++q) {
        int R = 0, C = 0;
        for (int n1 = 0; n1 < p; ++n1) {
          int dl = d(l, q - n1);
          THRO[q * p + n1] = dl > 0 ? R : -1;
          R += dl;
        }
        for (int n2 = 0; n2 < p; ++n2) {
          int dr = (q + n2 <= P.Q) ? d(r, q + n2) : 0;
          THCO[q * p + n2] = dr > 0 ? C : -1;
          C += dr;
        }
        if (R == 0 || C == 0) { R = 0; C = 0; }
        THR[q] = R; THC[q] = C; THO[q] = off;
        off += R * C;
      }
      THO[P.Q1] = off;
      ISCAL[I_THT] = off;
    }
    sync();
    const int tot = ISCAL[I_THT];
    for (int e = tid; e < tot; e += NT) {
      int q = blk_find(THO, e);
      int loc = e - THO[q], C = THC[q];
      int row = loc / C, col = loc - row * C;
      int n1 = seg_find(THRO + q * p, row), n2 = seg_find(THCO + q * p, col);
      int ia = row - THRO[q * p + n1], ic = col - THCO[q * p + n2];
      int dm = d(mid, q);
      zc acc = c2(0, 0);
      if (dm > 0) {
        lzp X1 = site(i1) + bo(i1, q - n1, n1) + ia * dm;
        int drc = d(r, q + n2);
        lzp X2 = site(r) + bo(r, q, n2) + ic;
        for (int b = 0; b < dm; ++b) cacc(acc, X1[b], X2[b * drc]);
      }
      TH[e] = acc;
    }
    sync();
  }

  // pre-phase -> hopping gate (per Δ = n1+n2 block) -> post-phase, on every
  // (a, c) vector of Θ.  mode 0: left-moving (UF both, optional lonely UT on
  // n2); mode 1: right-moving (UT both after the gate).  One thread per
  // output element (no runtime-indexed private arrays); the result goes to X
  // and the TH/X buffers are swapped.
  __device__ OCG_INLINE void apply_gate(int i1, int forward, int mode, int lonely) {
    pf(1);
    const int p = P.p;
    lzp gt = GT + (forward ? 0 : P.gtotal);
    lzp UF = PH;
    lzp UT = PH + p;
    const int tot = ISCAL[I_THT];
    for (int e = tid; e < tot; e += NT) {
      int q = blk_find(THO, e);
      int loc = e - THO[q], C = THC[q];
      int row = loc / C, col = loc - row * C;
      int a1 = seg_find(THRO + q * p, row), a2 = seg_find(THCO + q * p, col);
      int ia = row - THRO[q * p + a1], ic = col - THCO[q * p + a2];
      int D = a1 + a2, ql = q - a1;
      int lo = P.glo[D], sz = P.gsz[D], y = a1 - lo;
      lzp g = gt + P.goff[D] + y * sz;
      zc acc = c2(0, 0);
      for (int x = 0; x < sz; ++x) {
        int n1 = lo + x, n2 = D - n1, qs = ql + n1;
        zc z = TH[THO[qs] + (THRO[qs * p + n1] + ia) * THC[qs] + THCO[qs * p + n2] + ic];
        if (mode == 0) z = cmul(z, cmul(UF[n1], UF[n2]));
        cacc(acc, g[x], z);
      }
      if (mode == 1) acc = cmul(acc, cmul(UT[a1], UT[a2]));
      else if (lonely) acc = cmul(acc, UT[a2]);
      X[e] = acc;
    }
    sync();
    lzp t = TH; TH = X; X = t;
  }

  // ------------------------------------------------------------- Jacobi
  // Parallel (round-robin) complex Jacobi on all Gram blocks at once.
  // Block q: n = NQ[q] at G + GOFF[q]; eigenvectors accumulated in W.
  // On exit G/W point at the converged buffers (diag = eigenvalues).
  __device__ OCG_INLINE void jacobi(lzp& Gc, lzp& Wc) {
    lzp Gn = (Gc == G) ? G2 : G;
    lzp Wn = (Wc == W) ? W2 : W;
    const int maxr = ISCAL[I_MAXROUNDS];
    if (maxr <= 0) return;
    const int npair = ISCAL[I_NPAIR];
    const int nel = GOFF[P.Q1];
    for (int sweep = 0; sweep < 40; ++sweep) {
      for (int rnd = 0; rnd < maxr; ++rnd) {
        // Phase A: rotation parameters for every (block, pair)
        for (int t = tid; t < npair; t += NT) {
          int q = blk_find(POFF, t);
          int k = t - POFF[q], m = MQ[q], n = NQ[q];
          int pp_, qq_;
          bool active = rnd < m - 1;
          if (k == 0) { pp_ = m - 1; qq_ = rnd; }
          else { pp_ = (rnd + k) % (m - 1); qq_ = (rnd - k + m - 1) % (m - 1); }
          if (pp_ > qq_) { int tmp = pp_; pp_ = qq_; qq_ = tmp; }
          zc cs = c2(1.0, 0.0), e = c2(1.0, 0.0);
          double shift = 0.0;
          bool rot = false;
          if (active && qq_ < n) {
            lzp g = Gc + GOFF[q];
            zc b = g[pp_ * n + qq_];
            double ab = hypot(b.x, b.y);  // no underflow: e = b/|b| must stay unit-modulus
            double app = zc(g[pp_ * n + pp_]).x, aqq = zc(g[qq_ * n + qq_]).x;
            // skip rotations whose off-diagonal is below working precision of the diagonal
            if (ab > 1e-300 && ab > 1e-18 * (fabs(app) + fabs(aqq))) {
              double tau = (aqq - app) / (2.0 * ab);
              double tt = (tau >= 0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
              double c = 1.0 / sqrt(1.0 + tt * tt);
              cs = c2(c, tt * c);
              e = c2(b.x / ab, b.y / ab);
              shift = tt * ab;
              rot = true;
            }
          }
          ROT[2 * t] = cs;
          ROT[2 * t + 1] = e;
          if (active && qq_ < n) {
            int base = EOFF[q];
            PART[base + pp_] = qq_; ROLE[base + pp_] = rot ? 0 : 2; PAIR[base + pp_] = t;
            PART[base + qq_] = pp_; ROLE[base + qq_] = rot ? 1 : 2; PAIR[base + qq_] = t;
            LAM[base + pp_] = shift;  // reuse LAM as per-index shift scratch
          } else if (active && pp_ < n) {
            int base = EOFF[q];
            ROLE[base + pp_] = 2; PART[base + pp_] = pp_; PAIR[base + pp_] = t;
          }
          if (!active) {
            // block idle this round: all its indices unrotated (written by pair 0 only)
            if (k == 0) {
              int base = EOFF[q];
              for (int i = 0; i < n; ++i) { ROLE[base + i] = 2; PART[base + i] = i; }
            }
          }
        }
        sync();
        // Phase B: G' = J^H G J, W' = W J (double-buffered)
        for (int t = tid; t < 2 * nel; t += NT) {
          bool isW = t >= nel;
          int e = isW ? t - nel : t;
          int q = blk_find(GOFF, e);
          int n = NQ[q];
          int loc = e - GOFF[q];
          int i = loc / n, j = loc - i * n;
          int base = EOFF[q];
          lzp g = (isW ? Wc : Gc) + GOFF[q];
          if (MQ[q] == 0) {  // 1x1 block: nothing to rotate
            (isW ? Wn : Gn)[GOFF[q] + loc] = g[loc];
            continue;
          }
          // column-j coefficients of J: J[j][j], J[j'][j]
          int rj = ROLE[base + j], pj = PART[base + j];
          zc jjj, jpj;
          if (rj == 2) { jjj = c2(1, 0); jpj = c2(0, 0); pj = j; }
          else {
            zc cs = ROT[2 * PAIR[base + j]], ee = ROT[2 * PAIR[base + j] + 1];
            if (rj == 0) { jjj = c2(cs.x, 0); jpj = cscale(cconj(ee), -cs.y); }  // J[p][p]=c, J[q][p]=-s e*
            else { jjj = cscale(cconj(ee), cs.x); jpj = c2(cs.y, 0); }          // J[q][q]=c e*, J[p][q]=s
          }
          zc out;
          if (isW) {
            // W'[i][j] = W[i][j] J[j][j] + W[i][j'] J[j'][j]
            out = cmul(g[i * n + j], jjj);
            if (rj != 2) cacc(out, g[i * n + pj], jpj);
            Wn[GOFF[q] + loc] = out;
          } else {
            int ri = ROLE[base + i], pi = PART[base + i];
            if (ri != 2 && pi == j) {
              // the rotated 2x2 block: exact zero off-diagonal
              out = c2(0, 0);
            } else if (ri != 2 && i == j) {
              double sh = LAM[base + (ri == 0 ? i : pi)];
              out = c2(zc(g[i * n + i]).x + (ri == 0 ? -sh : sh), 0);
            } else {
              zc jii, jpi;
              if (ri == 2) { jii = c2(1, 0); jpi = c2(0, 0); pi = i; }
              else {
                zc cs = ROT[2 * PAIR[base + i]], ee = ROT[2 * PAIR[base + i] + 1];
                if (ri == 0) { jii = c2(cs.x, 0); jpi = cscale(cconj(ee), -cs.y); }
                else { jii = cscale(cconj(ee), cs.x); jpi = c2(cs.y, 0); }
              }
              // sum_{k in {i,i'}} sum_{l in {j,j'}} conj(J[k][i]) G[k][l] J[l][j]
              zc r0 = cmul(g[i * n + j], jjj);
              if (rj != 2) cacc(r0, g[i * n + pj], jpj);
              out = cjmul(jii, r0);
              if (ri != 2) {
                zc r1 = cmul(g[pi * n + j], jjj);
                if (rj != 2) cacc(r1, g[pi * n + pj], jpj);
                cjacc(out, jpi, r1);
              }
            }
            Gn[GOFF[q] + loc] = out;
          }
        }
        sync();
        lzp tg = Gc; Gc = Gn; Gn = tg;
        lzp tw = Wc; Wc = Wn; Wn = tw;
      }
      // convergence check: per block off-diagonal weight vs diagonal weight
      int fl = (sweep & 1) ? I_FLAG1 : I_FLAG0;
      int fo = (sweep & 1) ? I_FLAG0 : I_FLAG1;
      if (tid == 0) ISCAL[fo] = 0;
      for (int q = tid; q < P.Q1; q += NT) {
        int n = NQ[q];
        if (n < 2) continue;
        lzp g = Gc + GOFF[q];
        double off = 0, dia = 0;
        for (int i = 0; i < n; ++i)
          for (int j = 0; j < n; ++j) {
            double a = cabs2(g[i * n + j]);
            if (i == j) dia += a; else off += a;
          }
        if (off > 1e-30 * dia) atomicOr((int*)&ISCAL[fl], 1);
      }
      sync();
      int more = ISCAL[fl];
      sync();
      if (tid == 0) ISCAL[fl] = 0;
      if (!more) break;
    }
  }

  // ------------------------------------------------------------- decomposition
  // Block decomposition of TH (blocks THR x THC at THO) with truncation:
  //   Fromleft : TH = X Y, X orthonormal columns (left factor), Y carries norm
  //   Fromright: TH = X Y, Y orthonormal rows, X carries norm
  // The Gram matrix is formed on the smaller side of each block; the factor
  // on the other side is derived from TH.
  // If `normalize`, the norm-carrying factor is divided by sqrt(kept weight).
  // `bound` = per-sector rank bound of the new bond (MD row, or MDZ row in
  // the dH zip-up); vectors beyond it are numerically zero and dropped.
  __device__ OCG_INLINE void decompose(int dir, double cutoff, int maxm, bool normalize, const LDS int* bound) {
    pf(2);
    if (tid == 0) {
      int go = 0, eo = 0, po = 0, maxr = 0;
      for (int q = 0; q < P.Q1; ++q) {
        int R = THR[q], C = THC[q];
        int n = (R == 0 || C == 0) ? 0 : (R <= C ? R : C);
        NQ[q] = n;
        SIDE[q] = (R <= C) ? 0 : 1;  // 0: rows side (TH TH^H), 1: cols side (TH^H TH)
        GOFF[q] = go; go += n * n;
        EOFF[q] = eo; eo += n;
        int m = (n >= 2) ? (n + (n & 1)) : 0;
        MQ[q] = m;
        POFF[q] = po; po += m / 2;
        if (m - 1 > maxr) maxr = m - 1;
      }
      GOFF[P.Q1] = go; EOFF[P.Q1] = eo; POFF[P.Q1] = po;
      ISCAL[I_MAXROUNDS] = maxr;
      ISCAL[I_NPAIR] = po;
      ISCAL[I_EVT] = eo;
      ISCAL[I_FLAG0] = 0; ISCAL[I_FLAG1] = 0;
    }
    sync();
    // Gram matrices and identity eigenvectors
    const int nel = GOFF[P.Q1];
    for (int e = tid; e < nel; e += NT) {
      int q = blk_find(GOFF, e);
      int n = NQ[q], loc = e - GOFF[q];
      int i = loc / n, j = loc - i * n;
      lzp T = TH + THO[q];
      int R = THR[q], C = THC[q];
      zc acc = c2(0, 0);
      if (SIDE[q] == 0) {
        for (int c = 0; c < C; ++c) cacc(acc, T[i * C + c], cconj(T[j * C + c]));
      } else {
        for (int r = 0; r < R; ++r) cjacc(acc, T[r * C + i], T[r * C + j]);
      }
      G[e] = acc;
      W[e] = (i == j) ? c2(1, 0) : c2(0, 0);
    }
    sync();
    lzp Gc = G;
    lzp Wc = W;
    pf(3);
    jacobi(Gc, Wc);
    pf(4);
    // eigenvalues + global ranking (descending; ties by flat index)
    const int T = ISCAL[I_EVT];
    for (int e = tid; e < T; e += NT) {
      int q = blk_find(EOFF, e);
      int i = e - EOFF[q], n = NQ[q];
      double lam = zc(Gc[GOFF[q] + i * n + i]).x;
      LAM[e] = lam > 0 ? lam : 0.0;
    }
    sync();
    for (int e = tid; e < T; e += NT) {
      double le = LAM[e];
      int rk = 0;
      for (int f = 0; f < T; ++f) {
        double lf = LAM[f];
        rk += (lf > le) || (lf == le && f < e);
      }
      RANK[e] = rk;
      PP[rk] = le;
    }
    sync();
    // truncation (ITensor truncate; relative cutoff; floor 1e-30)
    if (tid == 0) {
      double total = 0;
      for (int i = 0; i < T; ++i) total += PP[i];
      int last = T - 1;
      double trunc = 0;
      while (last >= maxm) { trunc += PP[last]; --last; }
      while (last >= 1 && (trunc + PP[last] < cutoff * total || PP[last] <= 1e-30 * total)) {
        trunc += PP[last];
        --last;
      }
      int m = last + 1;
      double kw = 0;
      for (int i = 0; i < m; ++i) kw += PP[i];
      ISCAL[I_M] = m;
      SCAL[S_TOTAL] = total;
      SCAL[S_KEPTW] = kw;
      // kept per block + output offsets
      int xo = 0, yo = 0;
      for (int q = 0; q < P.Q1; ++q) {
        int k = 0;
        for (int i = 0; i < NQ[q]; ++i) k += RANK[EOFF[q] + i] < m;
        int cap = bound[q];
        if (k > cap) {  // beyond the sector's Schmidt-rank bound: numerical noise
          for (int r = 0; r < m && k > cap; ++r) {
            // drop this block's lowest-ranked kept vectors first
            int worst = -1, wr = -1;
            for (int i = 0; i < NQ[q]; ++i) {
              int rk = RANK[EOFF[q] + i];
              if (rk < m && rk > wr) { wr = rk; worst = i; }
            }
            kw -= PP[wr];
            RANK[EOFF[q] + worst] = 1 << 30;
            --k;
          }
          SCAL[S_KEPTW] = kw;
        }
        KEPT[q] = k;
        XOFF[q] = xo; xo += THR[q] * k;
        YOFF[q] = yo; yo += k * THC[q];
      }
      XOFF[P.Q1] = xo; YOFF[P.Q1] = yo;
    }
    // kept eigenvector order within each block (by global rank)
    sync();
    const int m = ISCAL[I_M];
    for (int e = tid; e < T; e += NT) {
      int rk = RANK[e];
      if (rk >= m) continue;
      int q = blk_find(EOFF, e);
      int j = 0;
      for (int f = EOFF[q]; f < EOFF[q + 1]; ++f) j += RANK[f] < rk;
      KIDX[EOFF[q] + j] = e - EOFF[q];
    }
    sync();
    pf(5);
    // materialise X (R x k) and Y (k x C) per block
    const double inv = (normalize && SCAL[S_KEPTW] > 1e-32) ? 1.0 / sqrt(SCAL[S_KEPTW]) : 1.0;
    const int xt = XOFF[P.Q1], yt = YOFF[P.Q1];
    for (int t = tid; t < xt + yt; t += NT) {
      bool isX = t < xt;
      int e = isX ? t : t - xt;
      int q = blk_find(isX ? XOFF : YOFF, e);
      int k = KEPT[q], R = THR[q], C = THC[q], n = NQ[q];
      int loc = e - (isX ? XOFF[q] : YOFF[q]);
      lzp Tq = TH + THO[q];
      lzp Wq = Wc + GOFF[q];
      if (isX) {
        int row = loc / k, j = loc - row * k;
        int w = KIDX[EOFF[q] + j];
        double lam = LAM[EOFF[q] + w];
        double sig = sqrt(lam);
        zc out;
        if (SIDE[q] == 0) {
          out = Wq[row * n + w];                       // u exact
          if (dir == kFromright) out = cscale(out, sig * inv);
        } else {
          zc acc = c2(0, 0);                      // Θ w
          for (int c = 0; c < C; ++c) cacc(acc, Tq[row * C + c], Wq[c * n + w]);
          if (dir == kFromleft) out = (sig > 0) ? cscale(acc, 1.0 / sig) : c2(0, 0);
          else out = cscale(acc, inv);
        }
        X[XOFF[q] + loc] = out;
      } else {
        int j = loc / C, col = loc - j * C;
        int w = KIDX[EOFF[q] + j];
        double lam = LAM[EOFF[q] + w];
        double sig = sqrt(lam);
        zc out;
        if (SIDE[q] == 1) {
          out = cconj(Wq[col * n + w]);                // v^H exact
          if (dir == kFromleft) out = cscale(out, sig * inv);
        } else {
          zc acc = c2(0, 0);                      // w^H Θ
          for (int r = 0; r < R; ++r) cjacc(acc, Wq[r * n + w], Tq[r * C + col]);
          if (dir == kFromright) out = (sig > 0) ? cscale(acc, 1.0 / sig) : c2(0, 0);
          else out = cscale(acc, inv);
        }
        Y[YOFF[q] + loc] = out;
      }
    }
    sync();
  }

  // write X (rows (n1,a)) into site i1 and Y (cols (n2,c)) into site i1+1
  __device__ OCG_INLINE void scatter_two_site(int i1) {
    pf(6);
    const int r = i1 + 1, p = P.p;
    if (tid == 0) {
      for (int q = 0; q < P.Q1; ++q) DIMS[i1 * P.Q1 + q] = KEPT[q];
    }
    sync();
    if (tid == 0) site_offsets_serial(i1, BOFF + (i1 - 1) * P.Q1 * p);
    if (tid == NT - 1 || NT == 1) site_offsets_serial(r, BOFF + (r - 1) * P.Q1 * p);
    sync();
    const int xt = XOFF[P.Q1], yt = YOFF[P.Q1];
    for (int t = tid; t < xt + yt; t += NT) {
      bool isX = t < xt;
      int e = isX ? t : t - xt;
      int q = blk_find(isX ? XOFF : YOFF, e);
      int k = KEPT[q];
      int loc = e - (isX ? XOFF[q] : YOFF[q]);
      if (isX) {
        int row = loc / k, j = loc - row * k;
        int n1 = seg_find(THRO + q * p, row);
        int ia = row - THRO[q * p + n1];
        site(i1)[bo(i1, q - n1, n1) + ia * k + j] = X[e];
      } else {
        int C = THC[q];
        int j = loc / C, col = loc - j * C;
        int n2 = seg_find(THCO + q * p, col);
        int ic = col - THCO[q * p + n2];
        site(r)[bo(r, q, n2) + j * d(r, q + n2) + ic] = Y[e];
      }
    }
    sync();
  }

  // single-site matricisation of site k into TH
  //   left (Fromleft grouping): rows (n, a in bond k-1 sector q-n), cols c in bond k sector q
  //   right (Fromright grouping): rows a in bond k-1 sector q, cols (n, c in bond k sector q+n)
  __device__ OCG_INLINE void site_to_theta(int k, bool left) {
    pf(7);
    const int p = P.p;
    if (tid == 0) {
      int off = 0;
      for (int q = 0; q < P.Q1; ++q) {
        int R = 0, C = 0;
        if (left) {
          for (int n = 0; n < p; ++n) { int dl = d(k - 1, q - n); THRO[q * p + n] = dl > 0 ? R : -1; R += dl; }
          C = d(k, q);
          for (int n = 0; n < p; ++n) THCO[q * p + n] = -1;
          THCO[q * p] = C > 0 ? 0 : -1;
        } else {
          R = d(k - 1, q);
          for (int n = 0; n < p; ++n) THRO[q * p + n] = -1;
          THRO[q * p] = R > 0 ? 0 : -1;
          for (int n = 0; n < p; ++n) {
            int dr = (q + n <= P.Q) ? d(k, q + n) : 0;
            THCO[q * p + n] = dr > 0 ? C : -1;
            C += dr;
          }
        }
        if (R == 0 || C == 0) { R = 0; C = 0; }
        THR[q] = R; THC[q] = C; THO[q] = off;
        off += R * C;
      }
      THO[P.Q1] = off;
      ISCAL[I_THT] = off;
    }
    sync();
    const int tot = ISCAL[I_THT];
    for (int e = tid; e < tot; e += NT) {
      int q = blk_find(THO, e);
      int loc = e - THO[q], C = THC[q];
      int row = loc / C, col = loc - row * C;
      zc v;
      if (left) {
        int n = seg_find(THRO + q * p, row);
        int ia = row - THRO[q * p + n];
        v = site(k)[bo(k, q - n, n) + ia * C + col];
      } else {
        int n = seg_find(THCO + q * p, col);
        int ic = col - THCO[q * p + n];
        v = site(k)[bo(k, q, n) + row * d(k, q + n) + ic];
      }
      TH[e] = v;
    }
    sync();
  }

  // move the orthogonality centre k -> k+1 (ITensor position, one bond)
  __device__ OCG_INLINE void gauge_right(int k, double cutoff, int maxm) {
    const int p = P.p;
    site_to_theta(k, true);
    decompose(kFromleft, cutoff, maxm, false, MD + k * P.Q1);
    pf(7);
    // new offsets of site k+1 with new bond-k dims (into BOFFT)
    if (tid == 0) {
      int off = 0;
      for (int q = 0; q < P.Q1; ++q)
        for (int n = 0; n < p; ++n) {
          int rr = KEPT[q], cc = (q + n <= P.Q) ? d(k + 1, q + n) : 0;
          if (rr > 0 && cc > 0) { BOFFT[q * p + n] = off; off += rr * cc; }
          else BOFFT[q * p + n] = -1;
        }
    }
    sync();
    // S = Y * A_{k+1}   (per (q, n): k_q x d(k+1, q+n))
    for (int q = 0; q < P.Q1; ++q)
      for (int n = 0; n < p; ++n) {
        int o = BOFFT[q * p + n];
        if (o < 0) continue;
        int kq = KEPT[q], cc = d(k + 1, q + n), dold = d(k, q);
        int oo = bo(k + 1, q, n);
        lzp Yq = Y + YOFF[q];
        for (int e = tid; e < kq * cc; e += NT) {
          int i = e / cc, j = e - i * cc;
          zc acc = c2(0, 0);
          if (oo >= 0)
            for (int b = 0; b < dold; ++b) cacc(acc, Yq[i * dold + b], site(k + 1)[oo + b * cc + j]);
          S[o + e] = acc;
        }
      }
    sync();
    if (tid == 0) {
      for (int q = 0; q < P.Q1; ++q) DIMS[k * P.Q1 + q] = KEPT[q];
      site_offsets_serial(k, BOFF + (k - 1) * P.Q1 * p);
      site_offsets_serial(k + 1, BOFF + k * P.Q1 * p);
    }
    sync();
    // A_k <- X ; A_{k+1} <- S
    const int xt = XOFF[P.Q1];
    for (int e = tid; e < xt; e += NT) {
      int q = blk_find(XOFF, e);
      int kq = KEPT[q], loc = e - XOFF[q];
      int row = loc / kq, j = loc - row * kq;
      int n = seg_find(THRO + q * p, row);
      int ia = row - THRO[q * p + n];
      site(k)[bo(k, q - n, n) + ia * kq + j] = X[e];
    }
    int ns = 0;
    for (int q = 0; q < P.Q1; ++q)
      for (int n = 0; n < p; ++n) {
        int o = bo(k + 1, q, n);
        if (o >= 0) { int e = o + d(k, q) * d(k + 1, q + n); if (e > ns) ns = e; }
      }
    for (int e = tid; e < ns; e += NT) site(k + 1)[e] = S[e];
    sync();
  }

  // move the orthogonality centre k -> k-1
  __device__ OCG_INLINE void gauge_left(int k, double cutoff, int maxm) {
    const int p = P.p;
    site_to_theta(k, false);
    decompose(kFromright, cutoff, maxm, false, MD + (k - 1) * P.Q1);
    pf(7);
    if (tid == 0) {
      int off = 0;
      for (int ql = 0; ql < P.Q1; ++ql)
        for (int n = 0; n < p; ++n) {
          int rr = d(k - 2, ql), cc = (ql + n <= P.Q) ? KEPT[ql + n] : 0;
          if (rr > 0 && cc > 0) { BOFFT[ql * p + n] = off; off += rr * cc; }
          else BOFFT[ql * p + n] = -1;
        }
    }
    sync();
    // S = A_{k-1} * X   (per (ql, n): d(k-2, ql) x k_{ql+n})
    for (int ql = 0; ql < P.Q1; ++ql)
      for (int n = 0; n < p; ++n) {
        int o = BOFFT[ql * p + n];
        if (o < 0) continue;
        int q = ql + n, kq = KEPT[q], rr = d(k - 2, ql), dold = d(k - 1, q);
        int oo = bo(k - 1, ql, n);
        lzp Xq = X + XOFF[q];
        for (int e = tid; e < rr * kq; e += NT) {
          int i = e / kq, j = e - i * kq;
          zc acc = c2(0, 0);
          if (oo >= 0)
            for (int b = 0; b < dold; ++b) cacc(acc, site(k - 1)[oo + i * dold + b], Xq[b * kq + j]);
          S[o + e] = acc;
        }
      }
    sync();
    if (tid == 0) {
      for (int q = 0; q < P.Q1; ++q) DIMS[(k - 1) * P.Q1 + q] = KEPT[q];
      site_offsets_serial(k, BOFF + (k - 1) * P.Q1 * p);
      site_offsets_serial(k - 1, BOFF + (k - 2) * P.Q1 * p);
    }
    sync();
    const int yt = YOFF[P.Q1];
    for (int e = tid; e < yt; e += NT) {
      int q = blk_find(YOFF, e);
      int C = THC[q], loc = e - YOFF[q];
      int j = loc / C, col = loc - j * C;
      int n = seg_find(THCO + q * p, col);
      int ic = col - THCO[q * p + n];
      site(k)[bo(k, q, n) + j * d(k, q + n) + ic] = Y[e];
    }
    int ns = 0;
    for (int q = 0; q < P.Q1; ++q)
      for (int n = 0; n < p; ++n) {
        int o = bo(k - 1, q, n);
        if (o >= 0) { int e = o + d(k - 2, q) * d(k - 1, q + n); if (e > ns) ns = e; }
      }
    for (int e = tid; e < ns; e += NT) site(k - 1)[e] = S[e];
    sync();
  }

  __device__ OCG_INLINE void position(int& centre, int target) {
    while (centre != target) {
      if (centre < target) { gauge_right(centre, OCG_GAUGE_CUTOFF, 1 << 30); ++centre; }
      else { gauge_left(centre, OCG_GAUGE_CUTOFF, 1 << 30); --centre; }
    }
  }

  // ------------------------------------------------------------- step
  // BH_tDMRG::step (src/BH_tDMRG.cpp:111-125) + doStep (:127-230).
  // The gate loop is written with one decompose call site and one gauge-move
  // call site so the (large) decomposition is inlined only twice.
  __device__ OCG_INLINE void step(double ufrom, double uto, int forward) {
    const int L = P.L, p = P.p;
    const double tau = forward ? P.dt : -P.dt;
    if (tid < p) {
      double nn = double(tid) * double(tid - 1);
      double af = -0.25 * ufrom * tau * nn, at = -0.25 * uto * tau * nn;
      PH[tid] = c2(cos(af), sin(af));
      PH[p + tid] = c2(cos(at), sin(at));
    }
    sync();
    if (L % 2 != 0) site_phase(L, PH);  // lonely U_from on site L (:133-136)
    int centre = 1;
    bool movingFromLeft = true;
    for (int g = 0; g < P.ngates; ++g) {
      const int i1 = P.gate_i1[g], i2 = i1 + 1;
      build_theta(i1);
      if (movingFromLeft) apply_gate(i1, forward, 0, (i2 == L && L % 2 == 0) ? 1 : 0);
      else apply_gate(i1, forward, 1, 0);
      // next gate: right of this one -> Fromleft, centre i2, move to ni1;
      //            left of it / last -> Fromright, centre i1, move to ni2 / 1
      const bool more = g + 1 < P.ngates;
      const int ni1 = more ? P.gate_i1[g + 1] : 0, ni2 = ni1 + 1;
      const int dir = (more && ni1 >= i2) ? kFromleft : kFromright;
      decompose(dir, P.cutoff, P.maxm, true, MD + i1 * P.Q1);
      scatter_two_site(i1);
      centre = (dir == kFromleft) ? i2 : i1;
      const int target = !more ? 1 : (dir == kFromleft ? ni1 : ni2);
      position(centre, target);
      if (more && (i2 == ni1 || i1 == ni2)) movingFromLeft = false;
    }
    site_phase(1, PH + p);  // lonely U_to on site 1 (:222-223)
    double n2 = site_norm2(1);
    if (n2 > 0) site_scale(1, 1.0 / sqrt(n2));  // psi.normalize() (:228)
  }

  // ------------------------------------------------------------- overlaps
  // <X|Y> (with_dH = 0) or <X| sum_k 0.5 n_k(n_k-1) |Y> (with_dH = 1);
  // X: an MPS in global memory (slot dims gd, data gx); Y: this chain's MPS.
  // Environments are block-diagonal in q: E_q is dX[b][q] x dY[b][q].
  // E0 carries the identity string, E1 the strings with dH already applied
  // (the bond-dimension-2 MPO of propagatorDeriv, src/BH_tDMRG.cpp:10-14).
  // Scratch: G/G2/W/W2 (environments), X (transfer temp), int tables
  // XOFF/YOFF (env offsets), BOFFT (temp offsets), THRO (X block offsets).
  __device__ OCG_INLINE zc overlap(const int* gd, const zc* gx, int with_dH) {
    pf(8);
    const int p = P.p, Q1 = P.Q1;
    lzp E0 = G;  lzp E1 = G2;
    lzp N0 = W;  lzp N1 = W2;
    LDS int* eo = XOFF;
    LDS int* no = YOFF;
    LDS int* to = BOFFT;
    LDS int* xo = THRO;
    if (tid == 0) {
      eo[0] = 0;
      for (int q = 1; q <= Q1; ++q) eo[q] = 1;  // prefix table: block q=0 is 1x1
      E0[0] = c2(1, 0);
      E1[0] = c2(0, 0);
    }
    sync();
    for (int k = 1; k <= P.L; ++k) {
      if (tid == 0) {
        // X block offsets of site k, temp offsets, next-env offsets
        int ox = 0, ot = 0, oe = 0;
        for (int q = 0; q < Q1; ++q)
          for (int n = 0; n < p; ++n) {
            int rx = gd[(k - 1) * Q1 + q];
            int cx = (q + n <= P.Q) ? gd[k * Q1 + q + n] : 0;
            xo[q * p + n] = (rx > 0 && cx > 0) ? ox : -1;
            if (rx > 0 && cx > 0) ox += rx * cx;
            int cy = (q + n <= P.Q) ? d(k, q + n) : 0;
            bool ok = rx > 0 && cx > 0 && d(k - 1, q) > 0 && bo(k, q, n) >= 0;
            to[q * p + n] = ok ? ot : -1;
            if (ok) ot += rx * cy;
          }
        for (int q = 0; q < Q1; ++q) {  // prefix table (empty blocks have size 0)
          no[q] = oe;
          oe += gd[k * Q1 + q] * d(k, q);
        }
        no[Q1] = oe;
      }
      sync();
      const int nenv = with_dH ? 2 : 1;
      // T_(q,n) = E_q * Y_(q,n)   for E0 (and E1): rows dX[k-1][q], cols dY[k][q+n]
      for (int ev = 0; ev < nenv; ++ev) {
        lzp E = ev == 0 ? E0 : E1;
        lzp T = X + ev * (P.thcap / 2);
        for (int q = 0; q < Q1; ++q)
          for (int n = 0; n < p; ++n) {
            int ot = to[q * p + n];
            if (ot < 0) continue;
            int rx = gd[(k - 1) * Q1 + q], ry = d(k - 1, q), cy = d(k, q + n);
            lzp Eq = E + eo[q];
            lzp Yb = site(k) + bo(k, q, n);
            for (int e = tid; e < rx * cy; e += NT) {
              int i = e / cy, j = e - i * cy;
              zc acc = c2(0, 0);
              for (int b = 0; b < ry; ++b) cacc(acc, Eq[i * ry + b], Yb[b * cy + j]);
              T[ot + e] = acc;
            }
          }
      }
      sync();
      // En_q' = sum_n f(n) X_(q'-n, n)^H T_(q'-n, n)
      const zc* sx = gx + P.site_base[k];
      const int ne = no[Q1];
      for (int t = tid; t < nenv * ne; t += NT) {
        int ev = t >= ne;
        int e = t - ev * ne;
        int qq = blk_find(no, e);
        int cy = d(k, qq);
        int loc = e - no[qq];
        int a = loc / cy, j = loc - a * cy;
        zc acc = c2(0, 0);
        for (int n = 0; n < p && n <= qq; ++n) {
          int q = qq - n;
          int ot = to[q * p + n];
          if (ot < 0) continue;
          int rx = gd[(k - 1) * Q1 + q], cx = gd[k * Q1 + qq];
          const zc* Xb = sx + xo[q * p + n];
          if (ev == 0) {
            lzp Tb = X + ot;
            zc s = c2(0, 0);
            for (int i = 0; i < rx; ++i) cjacc(s, Xb[i * cx + a], Tb[i * cy + j]);
            acc = cadd(acc, s);
          } else {
            // E1' = X^H (E1 Y) + f(n) X^H (E0 Y)
            lzp T0 = X + ot;
            lzp T1 = X + P.thcap / 2 + ot;
            zc s0 = c2(0, 0), s1 = c2(0, 0);
            for (int i = 0; i < rx; ++i) {
              cjacc(s1, Xb[i * cx + a], T1[i * cy + j]);
              cjacc(s0, Xb[i * cx + a], T0[i * cy + j]);
            }
            acc = cadd(acc, cadd(s1, cscale(s0, P.dH[n])));
          }
        }
        (ev == 0 ? N0 : N1)[e] = acc;
      }
      sync();
      lzp t0 = E0; E0 = N0; N0 = t0;
      lzp t1 = E1; E1 = N1; N1 = t1;
      if (tid == 0)
        for (int q = 0; q <= Q1; ++q) eo[q] = no[q];
      sync();
    }
    zc res = c2(0, 0);
    int oq = eo[P.Q];
    if (eo[P.Q1] > oq) res = with_dH ? E1[oq] : E0[oq];
    sync();
    return res;
  }

  // ------------------------------------------------------------- dH |psi>
  // exactApplyMPO(propDeriv, psi, args) (src/OptimalControl.cpp:256,:302):
  // exact bond-doubled MPO x MPS, zipped left->right through gauge-cutoff
  // decompositions (the orthogonalisation half-sweep), then truncated
  // right->left with the stepper's Cutoff/Maxm.  In place; the result is
  // right-orthonormal with the (unnormalised) centre at site 1.
  // Carry C_q (new bond k-1 x (s, old bond k-1)) lives in CR at COFF[q].
  __device__ OCG_INLINE void apply_dH(bool truncate_sweep = true) {
    pf(11);
    const int L = P.L, p = P.p, Q1 = P.Q1;
    LDS int* coff = COFF;   // carry offsets   (Q1+1)
    LDS int* cdim = CDIM;   // carry rows   = new dims of bond k-1
    LDS int* cold = COLD;   // carry cols/2 = old dims of bond k-1
    if (tid == 0) {
      for (int q = 0; q < Q1; ++q) { cdim[q] = d(0, q); cold[q] = d(0, q); coff[q] = 0; }
      coff[Q1] = 2;
      CR[0] = c2(1, 0);  // left boundary of the MPO: s = 0
      CR[1] = c2(0, 0);
    }
    sync();
    for (int k = 1; k <= L; ++k) {
      const bool last = (k == L);
      // ---- M_k: rows (n, a' in new bond k-1, sector q-n), cols (t, c in old bond k, sector q)
      if (tid == 0) {
        int off = 0;
        for (int q = 0; q < Q1; ++q) {
          int R = 0;
          for (int n = 0; n < p; ++n) {
            int dl = (q - n >= 0) ? cdim[q - n] : 0;
            THRO[q * p + n] = dl > 0 ? R : -1;
            R += dl;
          }
          int dc = d(k, q);
          int C = last ? dc : 2 * dc;
          for (int n = 0; n < p; ++n) THCO[q * p + n] = -1;
          THCO[q * p] = C > 0 ? 0 : -1;
          if (R == 0 || C == 0) { R = 0; C = 0; }
          THR[q] = R; THC[q] = C; THO[q] = off;
          off += R * C;
        }
        THO[Q1] = off;
        ISCAL[I_THT] = off;
      }
      sync();
      const int tot = ISCAL[I_THT];
      for (int e = tid; e < tot; e += NT) {
        int q = blk_find(THO, e);
        int loc = e - THO[q], C = THC[q];
        int row = loc / C, col = loc - row * C;
        int n = seg_find(THRO + q * p, row);
        int ap = row - THRO[q * p + n];
        int ql = q - n;
        int dc = d(k, q);
        int t = last ? 1 : (col >= dc ? 1 : 0);
        int c = last ? col : col - t * dc;
        int dl = cold[ql];                          // old rows of A_k blocks
        lzp Ab = site(k) + bo(k, ql, n);  // dl x dc (old layout)
        lzp Cq = CR + coff[ql];
        int w = 2 * cold[ql];
        zc v0 = c2(0, 0), v1 = c2(0, 0);
        for (int a = 0; a < dl; ++a) {
          zc av = Ab[a * dc + c];
          cacc(v0, Cq[ap * w + a], av);
          cacc(v1, Cq[ap * w + cold[ql] + a], av);
        }
        TH[e] = (t == 0) ? v0 : c2(P.dH[n] * v0.x + v1.x, P.dH[n] * v0.y + v1.y);
      }
      sync();
      if (last) {
        if (tid == 0) {
          for (int q = 0; q < Q1; ++q) DIMS[(L - 1) * Q1 + q] = cdim[q];
          site_offsets_serial(L, BOFF + (L - 1) * Q1 * p);
        }
        sync();
        for (int e = tid; e < tot; e += NT) {
          int q = blk_find(THO, e);
          int loc = e - THO[q], C = THC[q];
          int row = loc / C, col = loc - row * C;
          int n = seg_find(THRO + q * p, row);
          int ap = row - THRO[q * p + n];
          site(L)[bo(L, q - n, n) + ap * C + col] = TH[e];
        }
        sync();
        break;
      }
      decompose(kFromleft, OCG_GAUGE_CUTOFF, 1 << 30, false, MD + P.nsq + k * P.Q1);
      pf(11);
      if (tid == 0) {
        // new layout of site k: rows = new bond k-1 (cdim), cols = KEPT
        int o2 = 0;
        for (int q = 0; q < Q1; ++q)
          for (int n = 0; n < p; ++n) {
            int r = cdim[q], c = (q + n <= P.Q) ? KEPT[q + n] : 0;
            if (r > 0 && c > 0) { BOFFT[q * p + n] = o2; o2 += r * c; }
            else BOFFT[q * p + n] = -1;
          }
        ISCAL[12] = o2;
      }
      sync();
      // S <- X in the new layout of site k; CR <- Y (next carry)
      const int xt = XOFF[Q1], yt = YOFF[Q1];
      for (int e = tid; e < xt; e += NT) {
        int q = blk_find(XOFF, e);
        int kq = KEPT[q], loc = e - XOFF[q];
        int row = loc / kq, j = loc - row * kq;
        int n = seg_find(THRO + q * p, row);
        int ap = row - THRO[q * p + n];
        S[BOFFT[(q - n) * p + n] + ap * kq + j] = X[e];
      }
      for (int e = tid; e < yt; e += NT) CR[e] = Y[e];
      sync();
      const int ns = ISCAL[12];
      for (int e = tid; e < ns; e += NT) site(k)[e] = S[e];
      if (tid == 0) {
        // commit: bond k-1 gets its new dims; bond k keeps the OLD dims
        // (A_{k+1} is still laid out with them) until site k+1 is rebuilt.
        if (k > 1)
          for (int q = 0; q < Q1; ++q) DIMS[(k - 1) * Q1 + q] = cdim[q];
        for (int i = 0; i < Q1 * p; ++i) BOFF[(k - 1) * Q1 * p + i] = BOFFT[i];
        for (int q = 0; q < Q1; ++q) {
          cold[q] = d(k, q);
          cdim[q] = KEPT[q];
          coff[q] = YOFF[q];
        }
        coff[Q1] = YOFF[Q1];
      }
      sync();
    }
    if (truncate_sweep)
      for (int k = L; k > 1; --k) gauge_left(k, P.cutoff, P.maxm);
  }
};

}  // namespace ocg
