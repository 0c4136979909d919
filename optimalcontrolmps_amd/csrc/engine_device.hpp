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
//   data            (zc)    site k occupies [site_base[k], +site_cap[k]);
//                   inside it blocks (q, n) (rows dims[k-1][q], cols
//                   dims[k][q+n]) are packed row-major in (q, n) order, so
//                   the used part of a site is the prefix [0, used_k).
//
// Execution model: one chain = one workgroup of NT threads (NT a multiple of
// 64; the product build uses one wave64).  All bookkeeping is wave-parallel:
// per-sector tables are built by lane q with DPP prefix scans, per-(q, n)
// segment tables by chunked scans, and element -> block lookups use
// v_readlane over a register copy of the block prefix table (no serial
// thread-0 loops, no dependent LDS search chains).  Every wave primitive is
// reached by all lanes of its wave (uniform trip counts; per-element work is
// predicated inside).
#pragma once

#include <hip/hip_runtime.h>
#include <limits.h>

#include "engine.hpp"

#ifndef OCG_INLINE
#define OCG_INLINE __attribute__((always_inline))
#endif

// Jacobi rotation threshold |g_pq|^2 > OCG_JTOL2 |g_pp g_qq| (relative
// off-diagonal 1e-14 by default)
#ifndef OCG_JTOL2
#define OCG_JTOL2 1e-28
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

// LDS complex buffers: an address-space-3 double* with complex element access
// through a converting reference (clang does not let struct copy/assign
// operate through AS3 pointers).
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

// ---------------------------------------------------------------- wave64
__device__ __forceinline__ int rdlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ double rdlane(double v, int l) {
  long long b = __double_as_longlong(v);
  unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(unsigned long long)b, l);
  unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)((unsigned long long)b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// DPP row_shr:1,2,4,8 then row_bcast:15 / row_bcast:31 (CDNA wave64 scan idiom);
// lanes without a source read 0.
template <int CTRL, int RM>
__device__ __forceinline__ int dpp0(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, RM, 0xf, false); }
template <int CTRL, int RM>
__device__ __forceinline__ double dpp0(double v) {
  long long b = __double_as_longlong(v);
  int lo = dpp0<CTRL, RM>((int)(unsigned)(unsigned long long)b);
  int hi = dpp0<CTRL, RM>((int)(unsigned)((unsigned long long)b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// inclusive prefix sum over the 64 lanes of the wave
template <class T>
__device__ __forceinline__ T wscan(T v) {
  v += dpp0<0x111, 0xf>(v);
  v += dpp0<0x112, 0xf>(v);
  v += dpp0<0x114, 0xf>(v);
  v += dpp0<0x118, 0xf>(v);
  v += dpp0<0x142, 0xa>(v);
  v += dpp0<0x143, 0xc>(v);
  return v;
}
// inclusive prefix max (values >= 0)
__device__ __forceinline__ int wscan_max(int v) {
  v = max(v, dpp0<0x111, 0xf>(v));
  v = max(v, dpp0<0x112, 0xf>(v));
  v = max(v, dpp0<0x114, 0xf>(v));
  v = max(v, dpp0<0x118, 0xf>(v));
  v = max(v, dpp0<0x142, 0xa>(v));
  v = max(v, dpp0<0x143, 0xc>(v));
  return v;
}
__device__ __forceinline__ double wsum(double v) { return rdlane(wscan(v), 63); }
// exact a / b for 0 <= a < 2^22, b >= 1 (rcp estimate + one correction each way)
__device__ __forceinline__ int udiv(int a, int b, int& r) {
  int q = (int)((float)a * __builtin_amdgcn_rcpf((float)b));
  r = a - q * b;
  if (r < 0) { --q; r += b; }
  if (r >= b) { ++q; r -= b; }
  return q;
}

typedef int i4 __attribute__((vector_size(16)));

// Circle-method pairing table for even block orders m <= kPairMaxM:
// entry [pt_base(m) + r*m + x] = partner | (pair << 8) of index x in round
// r < kPairMaxM - 1; rounds r >= m - 1 hold idle entries (x | 0xFF << 8).
constexpr int kPairMaxM = 16;
constexpr int kPairRounds = kPairMaxM - 1;
constexpr int kPairTable = kPairRounds * 72;  // 15 * sum_{m = 2, 4, ..., 16} m
__host__ __device__ constexpr int pt_base(int m) { return kPairRounds * (m - 2) * m / 4; }

// ---------------------------------------------------------------- LDS map
struct LdsLayout {
  // complex buffers (offsets in zc units)
  int A, TH, G, G2, W, W2, X, Y, CR, S, GT, PH, ROT;
  int ncplx;
  // double buffers (offsets in doubles, after the complex region)
  int LAM, PP, SH, RED, SCAL, PROF;
  int ndbl;
  // int buffers (offsets in ints, after the double region)
  int DIMS, DIMX, MD, BOFF, BOFFT, TRO, TCO, THR, THC, THO, NQ, SIDE, GOFF, EOFF, MQ, POFF, KEPT, XOFF, YOFF, QST,
      CDIM, COLD, COFF, EQ, RANK, JB, KIDX, PT, ISCAL;
  int PLAN;  // P.nplan plan slots of plan_layout(P).stride ints
  int nint;
  int bytes;
};

// ---------------------------------------------------------------- plans
// A step runs the same sequence of two-site decompositions every time, and
// the block structure each one sees (the bond dimensions of the MPS at that
// point) rarely changes from one step to the next.  A plan slot per gate
// caches that structure: the Θ tables and, per Θ element, the operand
// offsets of the A_{i1} A_{i2} contraction (BT) and of the gate application
// (GA).  A step whose dims match the slot's key reuses them instead of
// rebuilding the tables and searching them element by element (the results
// are bitwise the same: only index arithmetic is cached).
// The decomposition's Gram layout (NQ/SIDE/MQ/GOFF/EOFF/POFF) and per-Gram-
// element operand offsets (GD) follow from the same key.  A second key, the
// kept dimension per sector (KK), selects the factor layout: XOFF/YOFF, the
// new offset tables of sites ts, ts+1 (BO1/BO2) and per-factor-element
// operand / destination offsets (XD, YD).
// Slot (ints): [0] valid, [1] Θ elements, [2] Jacobi rounds, [3] factor plan
// valid, [KEY] dims key (nsq), Θ tables TRO/TCO (SEG1 each) and THR/THC/THO
// (Q1P each), BT (2 per element: x1 | x2 << 16, dm | drc << 16), GA (GAW per
// element: gate row | sz << 16 | lo << 20 | a1 << 24 | a2 << 28, then the sz
// TH offsets as 16-bit pairs), Gram tables, GD (2 per element: a | b << 16,
// stride | len << 12 | side << 24 | diag << 25), KK, XOFF, YOFF, BO1, BO2,
// XD / YD (4 per element: a | g << 16, dest | len << 16, eoff | j << 16,
// n | stride << 12 | exact << 31).  Gauge moves use BT[2e] for the source of
// each matricised element, BO1 / BO2 for the new offset tables of the
// neighbour / moved site and SD (4 per element of the neighbour product S:
// first operand, second operand, length, second stride).
struct PlanLayout {
  int KEY, TRO, TCO, THR, THC, THO, BT, GA, GAW, NQ, SIDE, MQ, GOFF, EOFF, POFF, GD, KK, XOFF, YOFF, BO1, BO2, XD, YD,
      SD, PDO, PD, stride;
};
__host__ __device__ inline PlanLayout plan_layout(const OcgParams& P) {
  PlanLayout l;
  const int SEG1 = P.Q1 * P.p + 1, Q1P = (P.Q1 + 1 + 7) & ~7;
  auto al = [](int x) { return (x + 3) & ~3; };
  int i = 4;
  l.KEY = i; i = al(i + P.nsq);
  l.TRO = i; i = al(i + SEG1);
  l.TCO = i; i = al(i + SEG1);
  l.THR = i; i += Q1P;
  l.THC = i; i += Q1P;
  l.THO = i; i += Q1P;
  l.BT = i; i = al(i + 2 * P.plan_pe);
  l.GAW = 1 + (P.p + 1) / 2;
  l.GA = i; i = al(i + l.GAW * P.plan_pe);
  l.NQ = i; i += Q1P;
  l.SIDE = i; i += Q1P;
  l.MQ = i; i += Q1P;
  l.GOFF = i; i += Q1P;
  l.EOFF = i; i += Q1P;
  l.POFF = i; i += Q1P;
  l.GD = i; i = al(i + 2 * P.plan_pe);
  l.KK = i; i += Q1P;
  l.XOFF = i; i += Q1P;
  l.YOFF = i; i += Q1P;
  l.BO1 = i; i = al(i + SEG1);
  l.BO2 = i; i = al(i + SEG1);
  l.XD = i; i = al(i + 4 * P.plan_pe);
  l.YD = i; i = al(i + 4 * P.plan_pe);
  l.SD = i; i = al(i + 4 * P.plan_pe);
  l.PDO = i; i += Q1P;
  l.PD = i; i = al(i + 4 * P.plan_pe);
  l.stride = i;
  return l;
}

// Overlap-only kernels (<x|y>, <x|dH|y>): the MPS, four environments, the
// two T products and the staged site; every other buffer aliases offset 0
// and is never touched.  Small enough for several workgroups per CU.
__host__ __device__ inline LdsLayout lds_layout_ovl(const OcgParams& P, int nt) {
  LdsLayout l{};
  const int Q1 = P.Q1, SEG1 = Q1 * P.p + 1;
  const int Q1P = (Q1 + 1 + 7) & ~7;
  auto al = [](int x) { return (x + 3) & ~3; };
  int c = 0;
  l.A = c; c += P.cap;
  l.G = c; c += P.ecap;
  l.G2 = c; c += P.ecap;
  l.W = c; c += P.ecap;
  l.W2 = c; c += P.ecap;
  l.X = c; c += P.max_site_cap;
  l.Y = c; c += P.max_site_cap;
  l.S = c; c += P.max_site_cap;
  l.ncplx = c;
  int d = 0;
  l.RED = d; d += nt / 64 + 1;
  l.SCAL = d; d += 16;
  l.PROF = d; d += 32;
  l.ndbl = (d + 1) & ~1;
  int i = 0;
  l.DIMS = i; i = al(i + P.nsq);
  l.DIMX = i; i = al(i + P.nsq);
  l.BOFF = i; i = al(i + P.L * SEG1);
  l.BOFFT = i; i = al(i + SEG1);
  l.TCO = i; i = al(i + SEG1);
  l.THC = i; i += Q1P;
  l.THO = i; i += Q1P;
  l.XOFF = i; i += Q1P;
  l.YOFF = i; i += Q1P;
  l.QST = i; i += Q1P;
  l.ISCAL = i; i += 16;
  l.nint = i;
  l.bytes = l.ncplx * 16 + l.ndbl * 8 + l.nint * 4;
  return l;
}

__host__ __device__ inline LdsLayout lds_layout(const OcgParams& P, int nt) {
  LdsLayout l;
  const int Q1 = P.Q1, SEG1 = Q1 * P.p + 1;
  // per-sector tables: Q1+1 entries padded to a multiple of 8 (b128 searches)
  const int Q1P = (Q1 + 1 + 7) & ~7;
  auto al = [](int x) { return (x + 3) & ~3; };  // 16-byte aligned int offsets
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
  l.SH = d; d += P.nrot + 1;
  l.RED = d; d += nt / 64 + 1;
  l.SCAL = d; d += 16;
  l.PROF = d; d += 32;
  l.ndbl = (d + 1) & ~1;
  int i = 0;
  l.DIMS = i; i = al(i + P.nsq);
  l.DIMX = i; i = al(i + P.nsq);
  l.MD = i; i = al(i + 2 * P.nsq);
  l.BOFF = i; i = al(i + P.L * SEG1);
  l.BOFFT = i; i = al(i + SEG1);
  l.TRO = i; i = al(i + SEG1);
  l.TCO = i; i = al(i + SEG1);
  l.THR = i; i += Q1P;
  l.THC = i; i += Q1P;
  l.THO = i; i += Q1P;
  l.NQ = i; i += Q1P;
  l.SIDE = i; i += Q1P;
  l.GOFF = i; i += Q1P;
  l.EOFF = i; i += Q1P;
  l.MQ = i; i += Q1P;
  l.POFF = i; i += Q1P;
  l.KEPT = i; i += Q1P;
  l.XOFF = i; i += Q1P;
  l.YOFF = i; i += Q1P;
  l.QST = i; i += Q1P;
  l.CDIM = i; i += Q1P;
  l.COLD = i; i += Q1P;
  l.COFF = i; i += Q1P;
  l.EQ = i; i = al(i + P.evcap);
  l.RANK = i; i = al(i + P.evcap);
  l.JB = i; i = al(i + P.evcap);
  l.KIDX = i; i = al(i + P.evcap);
  l.PT = i; i = al(i + kPairTable);
  l.ISCAL = i; i += 16;
  l.PLAN = i; i += P.nplan > 0 ? P.nplan * plan_layout(P).stride : 0;
  l.nint = i;
  l.bytes = l.ncplx * 16 + l.ndbl * 8 + l.nint * 4;
  return l;
}

enum { kFromleft = 0, kFromright = 1 };

// scalar slots
enum { S_TOTAL = 0, S_KEPTW = 1 };
enum { I_M = 0, I_MAXROUNDS = 1, I_FLAG = 2 /* ..4 */, I_THT = 8, I_P2 = 9 };

template <int NT, bool OVL = false>
struct Chain {
  static_assert(NT % 64 == 0 && NT <= 1024, "a chain is a whole number of wave64s");
  static constexpr int NW = NT / 64;
  const OcgParams& P;
  const int tid, lane, SEG;
  const bool w0;
  lzp A, TH, G, G2, W, W2, X, Y, CR, S, GT, PH, ROT;
  LDS double *LAM, *PP, *SH, *RED, *SCAL, *PROF;
  LDS int *DIMS, *DIMX, *MD, *BOFF, *BOFFT, *TRO, *TCO, *THR, *THC, *THO, *NQ, *SIDE, *GOFF, *EOFF, *MQ, *POFF, *KEPT,
      *XOFF, *YOFF, *QST, *CDIM, *COLD, *COFF, *EQ, *RANK, *JB, *KIDX, *PT, *ISCAL;
  LDS int *PLN, *ps = nullptr;  // plan slots; the current decomposition's slot
  LDS int *TRO0, *TCO0, *THR0, *THC0, *THO0;  // scratch tables (no plan)
  LDS int *NQ0, *SIDE0, *MQ0, *GOFF0, *EOFF0, *POFF0, *XOFF0, *YOFF0;
  PlanLayout pl;
  bool phit = false;  // the current slot's key matched (uniform)
  double ph_u = __builtin_nan("");  // control value of PH[p..2p) (NaN: none yet)
  int ph_dir = -1;
  unsigned long long pf_last = 0;
  int pf_cur = 0;
  int pf_gauge = 0;  // profile build: cycles inside gauge moves also go to PROF[31]
  // algorithmic-traffic model accumulators (per lane, summed at the end)
  double m_bytes = 0, m_flops = 0;

  __device__ Chain(const OcgParams& P_, char* smem)
      : P(P_), tid(threadIdx.x), lane(threadIdx.x & 63), SEG(P_.Q1 * P_.p), w0(threadIdx.x < 64) {
    LdsLayout l = OVL ? lds_layout_ovl(P, NT) : lds_layout(P, NT);
    lzp cb{(LDS double*)smem};
    A = cb + l.A; TH = cb + l.TH; G = cb + l.G; G2 = cb + l.G2; W = cb + l.W; W2 = cb + l.W2; X = cb + l.X;
    Y = cb + l.Y; CR = cb + l.CR; S = cb + l.S; GT = cb + l.GT; PH = cb + l.PH; ROT = cb + l.ROT;
    LDS double* db = (cb + l.ncplx).p;
    LAM = db + l.LAM; PP = db + l.PP; SH = db + l.SH; RED = db + l.RED; SCAL = db + l.SCAL; PROF = db + l.PROF;
    LDS int* ib = (LDS int*)(db + l.ndbl);
    DIMS = ib + l.DIMS; DIMX = ib + l.DIMX; MD = ib + l.MD; BOFF = ib + l.BOFF; BOFFT = ib + l.BOFFT;
    TRO = ib + l.TRO; TCO = ib + l.TCO; THR = ib + l.THR; THC = ib + l.THC; THO = ib + l.THO; NQ = ib + l.NQ;
    SIDE = ib + l.SIDE; GOFF = ib + l.GOFF; EOFF = ib + l.EOFF; MQ = ib + l.MQ; POFF = ib + l.POFF;
    KEPT = ib + l.KEPT; XOFF = ib + l.XOFF; YOFF = ib + l.YOFF; QST = ib + l.QST; EQ = ib + l.EQ; RANK = ib + l.RANK;
    JB = ib + l.JB; KIDX = ib + l.KIDX; PT = ib + l.PT; CDIM = ib + l.CDIM; COLD = ib + l.COLD; COFF = ib + l.COFF;
    ISCAL = ib + l.ISCAL;
    PLN = ib + l.PLAN;
    pl = plan_layout(P);
    TRO0 = TRO; TCO0 = TCO; THR0 = THR; THC0 = THC; THO0 = THO;
    NQ0 = NQ; SIDE0 = SIDE; MQ0 = MQ; GOFF0 = GOFF; EOFF0 = EOFF; POFF0 = POFF; XOFF0 = XOFF; YOFF0 = YOFF;
  }

  // ------------------------------------------------------------- plans
  // Bind the Θ tables to plan slot s and test its key against the current
  // dims (each wave decides alone from LDS that is stable here, so no
  // barrier).  s < 0 or plans off: scratch tables, no plan.
  __device__ __forceinline__ void plan_begin(int s) {
    phit = false;
    if (s < 0 || s >= P.nplan) { plan_end(); return; }
    ps = PLN + s * pl.stride;
    TRO = ps + pl.TRO; TCO = ps + pl.TCO; THR = ps + pl.THR; THC = ps + pl.THC; THO = ps + pl.THO;
    NQ = ps + pl.NQ; SIDE = ps + pl.SIDE; MQ = ps + pl.MQ; GOFF = ps + pl.GOFF; EOFF = ps + pl.EOFF;
    POFF = ps + pl.POFF; XOFF = ps + pl.XOFF; YOFF = ps + pl.YOFF;
    bool diff = false;
    for (int i = lane; i < P.nsq; i += 64) diff |= DIMS[i] != ps[pl.KEY + i];
    phit = ps[0] != 0 && __ballot(diff) == 0;
  }
  __device__ __forceinline__ void plan_end() {
    ps = nullptr;
    phit = false;
    TRO = TRO0; TCO = TCO0; THR = THR0; THC = THC0; THO = THO0;
    NQ = NQ0; SIDE = SIDE0; MQ = MQ0; GOFF = GOFF0; EOFF = EOFF0; POFF = POFF0; XOFF = XOFF0; YOFF = YOFF0;
  }
  // after a miss: the slot now describes the current dims (called after the
  // phases that filled it, before the dims change; read again next step)
  __device__ __forceinline__ void plan_commit(int tot) {
    if (!ps || phit) return;
    for (int i = tid; i < P.nsq; i += NT) ps[pl.KEY + i] = DIMS[i];
    if (tid == 0) { ps[1] = tot; ps[0] = (tot <= P.plan_pe) ? 1 : 0; ps[3] = 0; }
  }

  __device__ __forceinline__ void sync() { __syncthreads(); }
  // LDS visibility among the lanes of one wave (no block barrier)
  __device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  // Diagnostic build only (-DOCG_PROFILE): thread 0 charges the shader-clock
  // cycles since the previous stamp to the category that was running.
  // Categories: 0 build_theta 1 apply_gate 2 gram 3 jacobi 4 rank/truncate
  // 5 factors X/Y (incl. the two-site write) 6 (unused) 7 gauge write-back 8 overlap 9 phases/norms
  // 10 load/store 11 apply_dH zip 12 other.
  __device__ __forceinline__ void pf(int cat) {
#ifdef OCG_PROFILE
    if (tid == 0) {
      unsigned long long t = __builtin_amdgcn_s_memtime();
      if (pf_last) {
        PROF[pf_cur] += double(t - pf_last);
        if (pf_gauge) PROF[31] += double(t - pf_last);
      }
      pf_last = t;
      pf_cur = cat;
    }
#else
    (void)cat;
#endif
  }
  __device__ __forceinline__ int d(int b, int q) const { return (q < 0 || q > P.Q) ? 0 : DIMS[b * P.Q1 + q]; }
  __device__ __forceinline__ int dx(int b, int q) const { return (q < 0 || q > P.Q) ? 0 : DIMX[b * P.Q1 + q]; }
  // per-site monotone block-offset table: [q*p + n] = start of block (q, n)
  // (empty blocks have zero length), [SEG] = used elements of the site
  __device__ __forceinline__ LDS int* boff(int k) const { return BOFF + (k - 1) * (SEG + 1); }
  __device__ __forceinline__ int bo(int k, int q, int n) const { return boff(k)[q * P.p + n]; }
  __device__ __forceinline__ int site_used(int k) const { return boff(k)[SEG]; }
  __device__ __forceinline__ lzp site(int k) { return A + P.site_base[k]; }

  // ------------------------------------------------------------- wave tables
  // block of element e in a per-sector prefix table T (Q1 starts, padded to a
  // multiple of 8, 16-byte aligned): last q with T[q] <= e.  Empty blocks
  // share the next block's start, so the last match is never empty.  Two
  // b128 broadcast loads per 8 sectors (one LDS round trip for Q1 <= 8).
  __device__ __forceinline__ int blk(const LDS int* T, int e) const {
    const int Q1 = P.Q1;
    int q = -1;
    for (int c = 0; c < Q1; c += 8) {
      const i4 a = *(const LDS i4*)(T + c);
      const i4 b = *(const LDS i4*)(T + c + 4);
      q += (a[0] <= e) + (c + 1 < Q1 && a[1] <= e) + (c + 2 < Q1 && a[2] <= e) + (c + 3 < Q1 && a[3] <= e) +
           (c + 4 < Q1 && b[0] <= e) + (c + 5 < Q1 && b[1] <= e) + (c + 6 < Q1 && b[2] <= e) +
           (c + 7 < Q1 && b[3] <= e);
    }
    return q;
  }
  // segment n of block q in a (q, n)-ordered prefix table TO containing
  // within-block offset x; o = offset of that segment relative to the block
  __device__ __forceinline__ int seg_in(const LDS int* TO, int q, int x, int& o) const {
    const int base = q * P.p, b0 = TO[base], lim = b0 + x;
    int n = 0, on = b0;
#pragma unroll
    for (int t = 1; t < OCG_MAXP; ++t)
      if (t < P.p) {
        int v = TO[base + t];
        if (v <= lim) { n = t; on = v; }
      }
    o = on - b0;
    return n;
  }
  // per-q starts of a (q, n) table into QST (one wave; caller syncs)
  __device__ __forceinline__ void qstarts(const LDS int* B) {
    if (lane < P.Q1) QST[lane] = B[lane * P.p];
  }
  // (q, n, start) of element e of a site laid out by the (q, n) table B
  // (QST must hold B's per-q starts)
  __device__ __forceinline__ void find_qn(const LDS int* B, int e, int& q, int& n, int& o) const {
    q = blk(QST, e);
    const int base = q * P.p;
    n = 0;
    o = B[base];
#pragma unroll
    for (int t = 1; t < OCG_MAXP; ++t)
      if (t < P.p) {
        int v = B[base + t];
        if (v <= e) { n = t; o = v; }
      }
  }
  // chunked exclusive scan over [0, n) by one wave: out[i] = sum_{j<i} len(j), out[n] = total
  // (if qs: qs[q] = out[q*p], the per-q starts of a (q, n) table)
  template <class F>
  __device__ OCG_INLINE int scan_excl(LDS int* out, int n, F len, LDS int* qs = nullptr) const {
    int carry = 0;
    for (int base = 0; base < n; base += 64) {
      const int i = base + lane;
      const int v = i < n ? len(i) : 0;
      const int inc = wscan(v);
      if (i < n) {
        out[i] = carry + inc - v;
        if (qs) {
          int q, nn;
          q = udiv(i, P.p, nn);
          if (nn == 0) qs[q] = carry + inc - v;
        }
      }
      carry += rdlane(inc, 63);
    }
    if (lane == 0) out[n] = carry;
    return carry;
  }
  // (q, n) of a flat segment index s = q*p + n
  __device__ __forceinline__ void qn_of(int s, int& q, int& n) const { q = udiv(s, P.p, n); }
  // block offsets of site k from the current dims (one wave)
  __device__ OCG_INLINE void site_offsets(int k) {
    scan_excl(boff(k), SEG, [&](int s) {
      int q, n;
      qn_of(s, q, n);
      return d(k - 1, q) * d(k, q + n);
    });
  }
  __device__ OCG_INLINE double block_sum(double v) {
    double w = wsum(v);
    if (NW == 1) return w;
    if (lane == 0) RED[tid >> 6] = w;
    sync();
    double s = 0;
    for (int i = 0; i < NW; ++i) s += RED[i];
    sync();
    return s;
  }
  // per-sector Θ tables from row-segment and column-segment lengths:
  // TRO/TCO (q, n) prefix tables, THR/THC block shapes (0 if empty), THO
  // block starts; returns the element count.  Uniform.
  template <class FR, class FC>
  __device__ OCG_INLINE int theta_tables(FR rowlen, FC collen) {
    if (w0) {
      scan_excl(TRO, SEG, [&](int s) { int q, n; qn_of(s, q, n); return rowlen(q, n); });
      scan_excl(TCO, SEG, [&](int s) { int q, n; qn_of(s, q, n); return collen(q, n); });
    }
    sync();
    if (w0) {
      const int q = lane;
      int R = 0, C = 0;
      if (q < P.Q1) { R = TRO[(q + 1) * P.p] - TRO[q * P.p]; C = TCO[(q + 1) * P.p] - TCO[q * P.p]; }
      if (R == 0 || C == 0) { R = 0; C = 0; }
      const int inc = wscan(R * C);
      if (q < P.Q1) { THR[q] = R; THC[q] = C; THO[q] = inc - R * C; }
      if (lane == 63) { THO[P.Q1] = inc; ISCAL[I_THT] = inc; }  // lane 63 holds the total
    }
    sync();
    return ISCAL[I_THT];
  }

  // ------------------------------------------------------------- I/O
  __device__ OCG_INLINE void load(const int* gdims, const zc* gdata) {
    pf(10);
    for (int i = tid; i < P.nsq; i += NT) DIMS[i] = gdims[i];
    sync();
    for (int k = 1 + (tid >> 6); k <= P.L; k += NW) site_offsets(k);
    sync();
    for (int k = 1; k <= P.L; ++k) {
      const int n = site_used(k), b = P.site_base[k];
      int i = tid;
      for (; i + 3 * NT < n; i += 4 * NT) {
        zc v0 = gdata[b + i], v1 = gdata[b + i + NT], v2 = gdata[b + i + 2 * NT], v3 = gdata[b + i + 3 * NT];
        A[b + i] = v0; A[b + i + NT] = v1; A[b + i + 2 * NT] = v2; A[b + i + 3 * NT] = v3;
      }
      for (; i < n; i += NT) A[b + i] = gdata[b + i];
    }
    sync();
  }
  __device__ OCG_INLINE void store(int* gdims, zc* gdata) {
    pf(10);
    for (int i = tid; i < P.nsq; i += NT) gdims[i] = DIMS[i];
    for (int k = 1; k <= P.L; ++k) {
      const int n = site_used(k), b = P.site_base[k];
      for (int i = tid; i < n; i += NT) gdata[b + i] = A[b + i];
    }
    sync();
  }
  // gate tables and the per-sector rank bound md[b][q] (Hilbert-space
  // Schmidt-rank bound; Maxm is applied by decompose) used to clamp numerically-zero
  // directions out of every decomposition (guards the LDS capacities).
  __device__ OCG_INLINE void load_tables(const zc* gf, const zc* gb, const int* md) {
    for (int i = tid; i < 32; i += NT) PROF[i] = 0.0;
    for (int s = tid; s < P.nplan; s += NT) PLN[s * pl.stride] = 0;  // no plan is valid yet
    if (OVL) return;  // overlaps need no gates, pair table or rank bounds
    // circle-method pairing table (see jpair)
    for (int e = tid; e < kPairTable; e += NT) {
      int m = 2;
      while (m < kPairMaxM && pt_base(m + 2) <= e) m += 2;
      int x;
      const int r = udiv(e - pt_base(m), m, x);
      int px = x;
      const int k = jpair(x, r, m, m, px);
      PT[e] = k < 0 ? (x | (0xFF << 8)) : (px | (k << 8));
    }
    for (int i = tid; i < P.gtotal; i += NT) { GT[i] = gf[i]; GT[P.gtotal + i] = gb[i]; }
    for (int i = tid; i < 2 * P.nsq; i += NT) MD[i] = md[i];
  }
  // traffic-model totals (valid in thread 0; uniform call)
  __device__ OCG_INLINE void model_totals(double& b, double& f) const {
    b = wsum(m_bytes);
    f = wsum(m_flops);
  }
  // complex elements of the current MPS (uniform)
  __device__ OCG_INLINE double mps_used() const {
    double v = (lane >= 1 && lane <= P.L) ? double(site_used(lane)) : 0.0;
    return wsum(v);
  }

  // ------------------------------------------------------------- norms
  __device__ OCG_INLINE double site_norm2(int k) {
    pf(9);
    const int n = site_used(k);
    double acc = 0;
    for (int i = tid; i < n; i += NT) acc += cabs2(site(k)[i]);
    return block_sum(acc);
  }
  __device__ OCG_INLINE void site_scale(int k, double f) {
    const int n = site_used(k);
    for (int i = tid; i < n; i += NT) site(k)[i] = cscale(site(k)[i], f);
    sync();
  }
  // multiply site k by a per-physical-index phase table ph[n]
  __device__ OCG_INLINE void site_phase(int k, lzp ph) {
    pf(9);
    const LDS int* B = boff(k);
    if (w0) qstarts(B);
    sync();
    const int tot = B[SEG];
    for (int e = tid; e < tot; e += NT) {
      int q, n, o;
      find_qn(B, e, q, n, o);
      site(k)[e] = cmul(site(k)[e], ph[n]);
    }
    sync();
  }

  // ------------------------------------------------------------- Θ
  // Two-site tensor for bond (i1, i1+1), blocks by middle QN q:
  //   rows (n1, a in bond i1-1 sector q-n1), cols (n2, c in bond i1+1 sector q+n2)
  __device__ OCG_INLINE void build_theta(int i1, int slot = -1) {
    pf(0);
    const int l = i1 - 1, mid = i1, r = i1 + 1;
    plan_begin(slot);
    int tot;
    if (phit) {
      tot = ps[1];
      if (tid == 0) ISCAL[I_THT] = tot;
    } else {
      pf(15);
      tot = theta_tables([&](int q, int n) { return d(l, q - n); }, [&](int q, int n) { return d(r, q + n); });
    }
    pf(0);
        // traffic model of this two-site update
    if (w0) {
      if (lane < P.Q1) {
        const double R = THR[lane], C = THC[lane], m = d(mid, lane), n = R < C ? R : C;
        m_flops += 8.0 * (R * C * m + R * C * P.p + n * n * (R > C ? R : C) + 2.0 * R * C * m);
      }
      if (lane == 0) m_bytes += 16.0 * (2.0 * (site_used(i1) + site_used(r)) + P.gtotal);
    }
    if (phit) {
      const LDS int* bt = ps + pl.BT;
      for (int e = tid; e < tot; e += NT) {
        const int w0_ = bt[2 * e], w1_ = bt[2 * e + 1];
        const int dm = w1_ & 0xffff, drc = (unsigned)w1_ >> 16;
        lzp X1 = A + (w0_ & 0xffff);
        lzp X2 = A + ((unsigned)w0_ >> 16);
        zc acc = c2(0, 0);
        for (int b = 0; b < dm; ++b) cacc(acc, X1[b], X2[b * drc]);
        TH[e] = acc;
      }
      sync();
      return;
    }
    const bool rec = ps != nullptr;
    for (int base = 0; base < tot; base += NT) {
      const int e = base + tid;
      const int q = blk(THO, e);
      if (e < tot) {
        const int C = THC[q];
        int col;
        const int row = udiv(e - THO[q], C, col);
        int o1, o2;
        const int n1 = seg_in(TRO, q, row, o1), n2 = seg_in(TCO, q, col, o2);
        const int ia = row - o1, ic = col - o2;
        const int dm = d(mid, q);
        zc acc = c2(0, 0);
        int x1 = 0, x2 = 0, drc = 0;
        if (dm > 0) {
          x1 = P.site_base[i1] + bo(i1, q - n1, n1) + ia * dm;
          drc = d(r, q + n2);
          x2 = P.site_base[r] + bo(r, q, n2) + ic;
          lzp X1 = A + x1;
          lzp X2 = A + x2;
          for (int b = 0; b < dm; ++b) cacc(acc, X1[b], X2[b * drc]);
        }
        TH[e] = acc;
        if (rec && e < P.plan_pe) {
          ps[pl.BT + 2 * e] = x1 | (x2 << 16);
          ps[pl.BT + 2 * e + 1] = dm | (drc << 16);
        }
      }
    }
    sync();
  }

  // pre-phase -> hopping gate (per Δ = n1+n2 block) -> post-phase, on every
  // (a, c) vector of Θ.  mode 0: left-moving (UF both, lonely & 1: the lonely
  // UT on n2 of an even chain); mode 1: right-moving (UT both after the gate;
  // lonely & 2: the lonely U_from of site L of an odd chain, doStep
  // src/BH_tDMRG.cpp:133-136, applied to the gate's input instead of the site,
  // since site L is untouched until this gate).  One thread per output
  // element; the result goes to X and the TH/X buffers are swapped.
  __device__ OCG_INLINE void apply_gate(int i1, int forward, int mode, int lonely) {
    pf(1);
    const int p = P.p;
    lzp gt = GT + (forward ? 0 : P.gtotal);
    lzp UF = PH;
    lzp UT = PH + p;
    const int tot = ISCAL[I_THT];
    if (phit) {
      const LDS int* ga = ps + pl.GA;
      for (int e = tid; e < tot; e += NT) {
        const LDS int* gd = ga + e * pl.GAW;
        const unsigned h = gd[0];
        const int sz = (h >> 16) & 15, lo = (h >> 20) & 15, a1 = (h >> 24) & 15, a2 = h >> 28, D = a1 + a2;
        lzp g = gt + int(h & 0xffff);
        zc acc = c2(0, 0);
        for (int x = 0; x < sz; ++x) {
          const int n1 = lo + x, n2 = D - n1;
          zc z = TH[(unsigned(gd[1 + (x >> 1)]) >> (16 * (x & 1))) & 0xffff];
          if (mode == 0) z = cmul(z, cmul(UF[n1], UF[n2]));
          else if (lonely & 2) z = cmul(z, UF[n2]);
          cacc(acc, g[x], z);
        }
        if (mode == 1) acc = cmul(acc, cmul(UT[a1], UT[a2]));
        else if (lonely & 1) acc = cmul(acc, UT[a2]);
        X[e] = acc;
      }
      sync();
      lzp t = TH; TH = X; X = t;
      return;
    }
    const bool rec = ps != nullptr;
    for (int base = 0; base < tot; base += NT) {
      const int e = base + tid;
      const int q = blk(THO, e);
      if (e < tot) {
        const int C = THC[q];
        int col;
        const int row = udiv(e - THO[q], C, col);
        int o1, o2;
        const int a1 = seg_in(TRO, q, row, o1), a2 = seg_in(TCO, q, col, o2);
        const int ia = row - o1, ic = col - o2;
        const int D = a1 + a2, ql = q - a1;
        const int lo = P.glo[D], sz = P.gsz[D], y = a1 - lo;
        lzp g = gt + P.goff[D] + y * sz;
        const bool rr = rec && e < P.plan_pe;
        LDS int* gd = rr ? ps + pl.GA + e * pl.GAW : nullptr;
        if (rr) gd[0] = (P.goff[D] + y * sz) | (sz << 16) | (lo << 20) | (a1 << 24) | (a2 << 28);
        zc acc = c2(0, 0);
        int pk = 0;
        for (int x = 0; x < sz; ++x) {
          const int n1 = lo + x, n2 = D - n1, qs = ql + n1;
          const int ro = TRO[qs * p + n1] - TRO[qs * p], co = TCO[qs * p + n2] - TCO[qs * p];
          const int ad = THO[qs] + (ro + ia) * THC[qs] + co + ic;
          zc z = TH[ad];
          if (mode == 0) z = cmul(z, cmul(UF[n1], UF[n2]));
          else if (lonely & 2) z = cmul(z, UF[n2]);
          cacc(acc, g[x], z);
          if (rr) {
            pk |= ad << (16 * (x & 1));
            if ((x & 1) || x + 1 == sz) { gd[1 + (x >> 1)] = pk; pk = 0; }
          }
        }
        if (mode == 1) acc = cmul(acc, cmul(UT[a1], UT[a2]));
        else if (lonely & 1) acc = cmul(acc, UT[a2]);
        X[e] = acc;
      }
    }
    sync();
    lzp t = TH; TH = X; X = t;
    plan_commit(tot);
  }

  // ------------------------------------------------------------- Jacobi
  // Pairing of index x of a block (m even, M = m-1 rounds) in round r of the
  // circle method: pair 0 = {r, M}; pair k = {(r+k) mod M, (r-k) mod M}.
  // Returns the pair id (-1 if x is idle this round) and its partner.
  __device__ __forceinline__ int jpair(int x, int r, int m, int n, int& px) const {
    const int M = m - 1;
    if (r >= M) return -1;
    int k;
    if (x == M) { px = r; k = 0; }
    else if (x == r) { px = M; k = 0; }
    else {
      int dd = x - r;
      if (dd < 0) dd += M;
      k = (2 * dd <= M) ? dd : M - dd;
      px = 2 * r - x;
      if (px < 0) px += M;
      if (px >= M) px -= M;
    }
    return (px < n) ? k : -1;
  }
  // coefficients of column x of J for pair (cs = (c, s), e):
  //   x = p: J[p][p] = c,     J[q][p] = -s e*
  //   x = q: J[q][q] = c e*,  J[p][q] = s
  __device__ __forceinline__ void jcol(int x, int px, zc cs, zc e, zc& jd, zc& jo) const {
    if (x < px) { jd = c2(cs.x, 0); jo = cscale(cconj(e), -cs.y); }
    else { jd = cscale(cconj(e), cs.x); jo = c2(cs.y, 0); }
  }
  // Gram element (i, j) of block q, with what phase B needs in every round
  struct JD {
    int i, j, n, m, go, po, pti, ptj;  // n == 0: no element; pt*: pair-table row bases (-1: m > kPairMaxM)
  };
  __device__ __forceinline__ JD jd_of(int e, int nel) const {
    JD r{0, 0, 0, 0, 0, 0, 0, 0};
    if (e < nel) {
      const int q = blk(GOFF, e);
      r.n = NQ[q]; r.m = MQ[q]; r.go = GOFF[q]; r.po = POFF[q];
      r.i = udiv(e - r.go, r.n, r.j);
      if (r.m <= kPairMaxM) { r.pti = pt_base(r.m) + r.i; r.ptj = pt_base(r.m) + r.j; }
      else { r.pti = -1; r.ptj = -1; }
    }
    return r;
  }
  // partner / pair of index x (table row base ptx) in round rnd; -1 if idle
  __device__ __forceinline__ int jlook(int x, int ptx, int rnd, int m, int n, int& px) const {
    if (rnd >= m - 1) { px = x; return -1; }
    int k;
    if (ptx >= 0) {
      const int v = PT[ptx + rnd * m];
      px = v & 255;
      k = v >> 8;
    } else {
      k = jpair(x, rnd, m, n, px);
    }
    return (px < n) ? k : -1;
  }
  // rotation pair t = (block q, pair k)
  struct JP {
    int k, n, m, go;  // n == 0: no pair
  };
  __device__ __forceinline__ JP jp_of(int t, int npair) const {
    JP r{0, 0, 0, 0};
    if (t < npair) {
      const int q = blk(POFF, t);
      r.k = t - POFF[q]; r.n = NQ[q]; r.m = MQ[q]; r.go = GOFF[q];
    }
    return r;
  }
  // rotate (p, q) iff |g_pq|^2 > tol^2 |g_pp g_qq| + (1e-18 (|g_pp| + |g_qq|))^2 (tol = 1e-14):
  // the Demmel-Veselic test bounds the orthonormality defect of the derived
  // factor, g_pq / (sigma_p sigma_q), by tol; the second term stops rotations
  // that are below working precision of the diagonal.  The same predicate is
  // the convergence test, so a converged sweep performs no rotation.
  __device__ __forceinline__ static bool jneed(double b2, double app, double aqq) {
    const double s = fabs(app) + fabs(aqq);
    return b2 > OCG_JTOL2 * fabs(app * aqq) + 1e-36 * s * s && b2 > 0.0;
  }
  // Phase A: complex Jacobi rotation zeroing g[p][q] of pair t in round rnd.
  // With D = aqq - app, b = g[p][q], r = |b| (the classical tan formula
  // t = sgn(D) / (|tau| + sqrt(1 + tau^2)), tau = D / (2 r), cleared of divisions):
  //   R = sqrt(D^2 + 4 r^2), E = |D| + R, c = E / sqrt(E^2 + 4 r^2),
  //   s = sgn(D) 2 r / sqrt(E^2 + 4 r^2), shift = sgn(D) 2 r^2 / E, e = b / r.
  __device__ __forceinline__ static void jrot_val(zc bv, double app, double aqq, zc& cs, zc& e, double& shift) {
    cs = c2(1.0, 0.0);
    e = c2(1.0, 0.0);
    shift = 0.0;
    double r2 = bv.x * bv.x + bv.y * bv.y;
    if (jneed(r2, app, aqq)) {
      // power-of-two rescale keeps r^2 and D^2 in range (exact, rare)
      double sc = 1.0;
      const double mb = fmax(fabs(bv.x), fabs(bv.y)), sz = fabs(app) + fabs(aqq);
      if (mb < 1e-120 || mb > 1e120 || sz > 1e120) {
        sc = ldexp(1.0, -ilogb(fmax(mb, sz)));
        bv = cscale(bv, sc); app *= sc; aqq *= sc;
        r2 = bv.x * bv.x + bv.y * bv.y;
      }
      const double rinv = rsqrt(r2), r = r2 * rinv;
      const double D = aqq - app, sg = D >= 0 ? 1.0 : -1.0;
      const double E = fabs(D) + sqrt(fma(D, D, 4.0 * r2));
      const double h = rsqrt(fma(E, E, 4.0 * r2));
      cs = c2(E * h, sg * 2.0 * r * h);
      e = c2(bv.x * rinv, bv.y * rinv);
      shift = sg * 2.0 * r2 / (E * sc);
    }
  }
  // The same rotation with the hardware reciprocal square root / reciprocal
  // plus one Newton-type refinement each (inputs kept in the normal range by
  // the rescale), branch-free apart from the rare rescale: ~40 instructions
  // instead of ~90 for the IEEE sqrt / division expansions.
  __device__ __forceinline__ static double rsq_ref(double x) {  // x > 0 normal
    const double y = __builtin_amdgcn_rsq(x);
    const double d = fma(-x * y, y, 1.0);  // 1 - x y^2
    return fma(y * d, fma(d, 0.375, 0.5), y);
  }
  __device__ __forceinline__ static double rcp_ref(double x) {
    double y = __builtin_amdgcn_rcp(x);
    y = fma(y, fma(-x, y, 1.0), y);
    return fma(y, fma(-x, y, 1.0), y);
  }
  // need = jneed(|bv|^2, app, aqq), evaluated by the caller.  Branch-free:
  // the power-of-two rescale factor is 1 (exact) unless a rescale is needed.
  __device__ __forceinline__ static void jrot_fast(zc bv, double app, double aqq, bool need, zc& cs, zc& e,
                                                   double& shift) {
    const double mb = fmax(fabs(bv.x), fabs(bv.y)), sz = fabs(app) + fabs(aqq);
    const bool resc = need && (mb < 1e-120 || mb > 1e120 || sz > 1e120);
    const double sc = resc ? ldexp(1.0, -ilogb(fmax(mb, sz))) : 1.0;
    bv = cscale(bv, sc);
    app *= sc;
    aqq *= sc;
    const double r2 = need ? bv.x * bv.x + bv.y * bv.y : 1.0;
    const double rinv = rsq_ref(r2), r = r2 * rinv;
    const double D = aqq - app, sg = D >= 0 ? 1.0 : -1.0;
    const double x = fma(D, D, 4.0 * r2);
    const double E = fabs(D) + x * rsq_ref(x);
    const double h = rsq_ref(fma(E, E, 4.0 * r2));
    cs = need ? c2(E * h, sg * 2.0 * r * h) : c2(1.0, 0.0);
    e = need ? c2(bv.x * rinv, bv.y * rinv) : c2(1.0, 0.0);
    shift = need ? sg * 2.0 * r2 * rcp_ref(E * sc) : 0.0;
  }
  __device__ __forceinline__ void jrot(const JP& d, int t, int rnd, lzp Gc) {
    if (d.n == 0) return;
    const int M = d.m - 1, n = d.n;
    zc cs = c2(1.0, 0.0), e = c2(1.0, 0.0);
    double shift = 0.0;
    if (rnd < M) {
      int a = rnd + d.k, b = rnd - d.k;
      if (d.k == 0) b = M;
      if (a >= M) a -= M;
      if (b < 0) b += M;
      const int pp_ = a < b ? a : b, qq_ = a < b ? b : a;
      if (qq_ < n) {
        lzp g = Gc + d.go;
        jrot_val(g[pp_ * n + qq_], zc(g[pp_ * n + pp_]).x, zc(g[qq_ * n + qq_]).x, cs, e, shift);
      }
    }
    ROT[2 * t] = cs;
    ROT[2 * t + 1] = e;
    SH[t] = shift;
  }
  // coefficients of column x of J for pair (cs = (c, s), e), branch-free:
  //   x = p (x < partner): J[p][p] = c,     J[q][p] = -s e*
  //   x = q:               J[q][q] = c e*,  J[p][q] = s
  __device__ __forceinline__ static void jcol(bool isp, zc cs, zc e, zc& jd, zc& jo) {
    const zc ce = cscale(cconj(e), cs.x), se = cscale(cconj(e), -cs.y);
    jd = isp ? c2(cs.x, 0.0) : ce;
    jo = isp ? se : c2(cs.y, 0.0);
  }
  // Phase B: G'[i][j] = (J^H G J)[i][j] and W'[i][j] = (W J)[i][j]
  __device__ __forceinline__ void jupd(const JD& d, int rnd, lzp Gc, lzp Wc, lzp Gn, lzp Wn, bool lastr, int fl) {
    if (d.n == 0) return;
    const int i = d.i, j = d.j, n = d.n, m = d.m, loc = i * n + j;
    lzp gs = Gc + d.go, ws = Wc + d.go;
    int pj, pi;
    const int kj = jlook(j, d.ptj, rnd, m, n, pj);
    const int ki = jlook(i, d.pti, rnd, m, n, pi);
    zc jjj = c2(1, 0), jpj = c2(0, 0), jii = c2(1, 0), jpi = c2(0, 0);
    bool rotj = false, roti = false;
    if (kj >= 0) {
      const zc cs = ROT[2 * (d.po + kj)], ee = ROT[2 * (d.po + kj) + 1];
      rotj = cs.y != 0.0;
      jcol(j < pj, cs, ee, jjj, jpj);
    }
    if (ki >= 0) {
      const zc cs = ROT[2 * (d.po + ki)], ee = ROT[2 * (d.po + ki) + 1];
      roti = cs.y != 0.0;
      jcol(i < pi, cs, ee, jii, jpi);
    }
    // W'[i][j] = W[i][j] J[j][j] + W[i][j'] J[j'][j]
    zc w = cmul(ws[loc], jjj);
    if (rotj) cacc(w, ws[i * n + pj], jpj);
    Wn[d.go + loc] = w;
    zc out;
    if (rotj && pi == j && ki >= 0) {
      out = c2(0, 0);  // the rotated 2x2 block: exact zero off-diagonal
    } else if (rotj && i == j) {
      const double sh = SH[d.po + kj];
      out = c2(zc(gs[loc]).x + (j < pj ? -sh : sh), 0);
    } else {
      // sum_{k in {i,i'}} sum_{l in {j,j'}} conj(J[k][i]) G[k][l] J[l][j]
      zc r0 = cmul(gs[loc], jjj);
      if (rotj) cacc(r0, gs[i * n + pj], jpj);
      out = cjmul(jii, r0);
      if (roti) {
        zc r1 = cmul(gs[pi * n + j], jjj);
        if (rotj) cacc(r1, gs[pi * n + pj], jpj);
        cjacc(out, jpi, r1);
      }
    }
    // convergence: the rotation predicate on the output of the sweep's last round
    if (lastr && i < j && jneed(cabs2(out), zc(gs[i * n + i]).x, zc(gs[j * n + j]).x))
      ISCAL[fl] = 1;  // benign race: every writer stores 1
    Gn[d.go + loc] = out;
  }
  // Branch-free phase B for blocks of order m <= kPairMaxM (all blocks of the
  // decomposition): the pairing comes from the table, idle / padded /
  // unrotated indices get identity coefficients by selects, and every element
  // computes both its G' and W' entries.
  __device__ __forceinline__ void jupd_fast(const JD& d, bool valid, int rnd, lzp Gc, lzp Wc, lzp Gn, lzp Wn,
                                            bool lastr, int fl) {
    const int i = d.i, j = d.j, n = d.n > 0 ? d.n : 1, loc = i * n + j;
    lzp gs = Gc + d.go, ws = Wc + d.go;
    const int vj = PT[d.ptj + rnd * d.m], vi = PT[d.pti + rnd * d.m];
    int pj = vj & 255, kj = vj >> 8, pi = vi & 255, ki = vi >> 8;
    const bool aj = kj != 0xFF && pj < n, ai = ki != 0xFF && pi < n;
    pj = aj ? pj : j;
    pi = ai ? pi : i;
    kj = aj ? kj : 0;
    ki = ai ? ki : 0;
    const zc csj = ROT[2 * (d.po + kj)], ej = ROT[2 * (d.po + kj) + 1];
    const zc csi = ROT[2 * (d.po + ki)], ei = ROT[2 * (d.po + ki) + 1];
    const double sh = SH[d.po + kj];
    const zc g00 = gs[loc], g01 = gs[i * n + pj], g10 = gs[pi * n + j], g11 = gs[pi * n + pj];
    const zc w0 = ws[loc], w1 = ws[i * n + pj];
    const bool rotj = aj && csj.y != 0.0, roti = ai && csi.y != 0.0;
    zc jjj, jpj, jii, jpi;
    jcol(j < pj, csj, ej, jjj, jpj);
    jcol(i < pi, csi, ei, jii, jpi);
    jjj = rotj ? jjj : c2(1, 0);
    jpj = rotj ? jpj : c2(0, 0);
    jii = roti ? jii : c2(1, 0);
    jpi = roti ? jpi : c2(0, 0);
    // W'[i][j] = W[i][j] J[j][j] + W[i][j'] J[j'][j]
    zc w = cmul(w0, jjj);
    cacc(w, w1, jpj);
    // G'[i][j] = sum_{k in {i,i'}} sum_{l in {j,j'}} conj(J[k][i]) G[k][l] J[l][j]
    zc r0 = cmul(g00, jjj);
    cacc(r0, g01, jpj);
    zc r1 = cmul(g10, jjj);
    cacc(r1, g11, jpj);
    zc out = cjmul(jii, r0);
    cjacc(out, jpi, r1);
    // the rotated 2x2 block: exact zero off-diagonal, shifted diagonal
    const bool zero = rotj && roti && pi == j;
    const bool diag = rotj && i == j;
    out = zero ? c2(0, 0) : out;
    out = diag ? c2(g00.x + (j < pj ? -sh : sh), 0) : out;
    if (valid) {
      Wn[d.go + loc] = w;
      Gn[d.go + loc] = out;
      if (lastr && i < j && jneed(cabs2(out), zc(gs[i * n + i]).x, zc(gs[j * n + j]).x))
        ISCAL[fl] = 1;  // benign race: every writer stores 1
    }
  }
  // Parallel (round-robin) complex Jacobi on all Gram blocks at once.
  // Block q: n = NQ[q] at G + GOFF[q]; eigenvectors accumulated in W.
  // Element/pair descriptors are computed once and kept in registers for
  // all rounds (JB_IT x NT elements, JA_IT x NT pairs; larger problems fall
  // back to per-round lookups).  Convergence is tested on the output of each
  // sweep's last round.  On exit Gc/Wc point at the converged buffers.
  // Register-resident Jacobi for decompositions whose blocks all have order
  // m <= S (S = 4 or 8): block b lives in one S*S-lane group of a wave (lane
  // S*i + j holds G[i][j] and W[i][j]; padding lanes hold zeros).  Per round
  // the lane holding the pivot g[p][q] (p < q paired this round) evaluates
  // the rotation (jrot_val, the phase-A formula); every lane then gathers the
  // rotations of its column pair and row pair and the three partner elements
  // of its 2x2 super-block with ds_bpermute and applies the phase-B update
  // (jupd_fast).  Same pairing, formulas and sweep structure as the LDS path,
  // but no block barrier: a wave sweeps its own blocks until its convergence
  // ballot is empty (sweeps over converged blocks are exact no-ops, so
  // per-wave termination changes nothing).  Writes G and W back in place;
  // the caller syncs.
  __device__ __forceinline__ static double bperm(double v, int addr) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_bpermute(addr, int(b)), hi = __builtin_amdgcn_ds_bpermute(addr, int(b >> 32));
    return __longlong_as_double((long long)(unsigned)lo | ((long long)hi << 32));
  }
  __device__ __forceinline__ static zc bpermz(zc v, int addr) { return c2(bperm(v.x, addr), bperm(v.y, addr)); }
  // DPP lane swaps inside a 16-lane row (one 4x4 block, lane 4 i + j):
  // xcol = lane ^ k (quad_perm), xrow = lane ^ 4k (row/half mirrors
  // composed with a quad swap), k = rnd + 1; rnd is a constant after unrolling
  template <int CTRL>
  __device__ __forceinline__ static double dppd(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, int(b), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, int(b >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double((long long)(unsigned)lo | ((long long)hi << 32));
  }
  template <int CTRL>
  __device__ __forceinline__ static zc dppz(zc v) { return c2(dppd<CTRL>(v.x), dppd<CTRL>(v.y)); }
  static constexpr int kQx1 = 0xB1, kQx2 = 0x4E, kQx3 = 0x1B, kRowMirror = 0x140, kHalfMirror = 0x141;
  __device__ __forceinline__ static zc xcol(zc v, int rnd) {
    return rnd == 0 ? dppz<kQx1>(v) : rnd == 1 ? dppz<kQx2>(v) : dppz<kQx3>(v);
  }
  __device__ __forceinline__ static zc xrow(zc v, int rnd) {
    if (rnd == 0) return dppz<kQx3>(dppz<kHalfMirror>(v));        // ^7 ^3 = ^4
    if (rnd == 1) return dppz<kHalfMirror>(dppz<kRowMirror>(v));  // ^15 ^7 = ^8
    return dppz<kQx3>(dppz<kRowMirror>(v));                       // ^15 ^3 = ^12
  }
  template <int S>
  __device__ OCG_INLINE void jacobi_reg(lzp Gc, lzp Wc, int maxr, const LDS int* gd) {
    constexpr int GS = S * S;     // lanes per block
    constexpr int BPW = 64 / GS;  // blocks per wave
    constexpr int MR = S - 1;     // rounds per sweep, at most
    const int Q1 = P.Q1;
    const int i = (lane / S) % S, j = lane % S, rb = lane & ~(GS - 1);
    const int wave = tid >> 6;
    auto at = [&](int r, int c) { return (rb + r * S + c) << 2; };  // bpermute byte address of (r, c)
    const int aii = at(i, i), ajj = at(j, j);
    for (int b0 = wave * BPW; b0 < Q1; b0 += BPW * NW) {
      const int q = b0 + lane / GS;
      const bool blk_ok = q < Q1;
      const int n = blk_ok ? NQ[q] : 0, m = blk_ok ? MQ[q] : 0, go = blk_ok ? GOFF[q] : 0;
      const int eo = blk_ok ? EOFF[q] : 0;
      const bool valid = i < n && j < n;
      const int loc = go + i * n + j;
      zc g = c2(0.0, 0.0), w;
      if (gd) {
        // Gram element straight from the plan's descriptor (no Gram phase):
        // the same sums, in the same order, as the Gram phase computes
        w = c2(i == j ? 1.0 : 0.0, 0.0);
        if (valid) {
          const unsigned a0 = gd[2 * loc], a1 = gd[2 * loc + 1];
          const int st = a1 & 0xfff, len = (a1 >> 12) & 0xfff;
          lzp Ta = TH + int(a0 & 0xffff), Tb = TH + int(a0 >> 16);
          if (((a1 >> 24) & 1) == 0) {
            for (int c = 0; c < len; ++c) cacc(g, Ta[c * st], cconj(Tb[c * st]));
          } else {
            for (int r = 0; r < len; ++r) cjacc(g, Ta[r * st], Tb[r * st]);
          }
        }
      } else {
        g = valid ? zc(Gc[loc]) : c2(0.0, 0.0);
        w = valid ? zc(Wc[loc]) : c2(i == j ? 1.0 : 0.0, 0.0);
      }
      pf(14);  // profile: Gram formation above (jacobi A), rounds below (jacobi B)
      // per-round roles: partners of i and j (idle / padded: self), the
      // bpermute addresses of the two rotations and three partner elements
      int arow[MR], acol[MR], aipj[MR], apij[MR], apipj[MR], fl[MR];
#pragma unroll
      for (int rnd = 0; rnd < MR; ++rnd) {
        int pi = i, pj = j, t;
        if constexpr (S == 4) {
          // order <= 4: round r pairs x with x ^ (r + 1) (a complete
          // round-robin of 4), so every partner element is a DPP lane swap
          const int k = rnd + 1;
          if (rnd < maxr && i < n && j < n) {  // pad lanes keep self
            if ((i ^ k) < n) pi = i ^ k;
            if ((j ^ k) < n) pj = j ^ k;
          }
          (void)t;
        } else if (rnd < maxr) {
          if (i < n && jpair(i, rnd, m, n, t) >= 0) pi = t;
          if (j < n && jpair(j, rnd, m, n, t) >= 0) pj = t;
        }
        arow[rnd] = at(i < pi ? i : pi, i < pi ? pi : i);
        acol[rnd] = at(j < pj ? j : pj, j < pj ? pj : j);
        aipj[rnd] = at(i, pj);
        apij[rnd] = at(pi, j);
        apipj[rnd] = at(pi, pj);
        // bit 0 pivot (i < j paired), 1 j < pj, 2 i < pi, 3 j moves, 4 i moves, 5 pi == j
        fl[rnd] = (i < j && pi == j ? 1 : 0) | (j < pj ? 2 : 0) | (i < pi ? 4 : 0) | (pj != j ? 8 : 0) |
                  (pi != i ? 16 : 0) | (pi == j ? 32 : 0);
      }
      int sweep = 0;
      bool done = false;
      for (; sweep < 40; ++sweep) {
        bool flag = false;
#pragma unroll
        for (int rnd = 0; rnd < MR; ++rnd) {
          if (rnd >= maxr) break;
          const int f = fl[rnd];
          // pivot lanes: rotation of pair (i, j)
          const double dpp = bperm(g.x, aii), dqq = bperm(g.x, ajj);
          // early exit: no pair of the wave's blocks passes the rotation
          // predicate, so the rest of this sweep is a chain of exact no-ops
          // and the end-of-sweep test would stop after it (same result)
          const bool need = jneed(cabs2(g), dpp, dqq);
          if (__ballot(valid && i < j && need) == 0) {
            done = true;
            break;
          }
          zc cs, e;
          double sh;
          jrot_fast(g, dpp, dqq, need, cs, e, sh);
          const bool piv = f & 1;
          cs = piv ? cs : c2(1.0, 0.0);
          sh = piv ? sh : 0.0;
          // rotations of the column pair (j, pj) and the row pair (i, pi)
          const zc csj = bpermz(cs, acol[rnd]), ej = bpermz(e, acol[rnd]);
          const zc csi = bpermz(cs, arow[rnd]), ei = bpermz(e, arow[rnd]);
          const double shj = bperm(sh, acol[rnd]);
          zc g01, g10, g11, w1;
          if constexpr (S == 4) {
            g01 = xcol(g, rnd);  // G[i][j ^ k]
            g10 = xrow(g, rnd);  // G[i ^ k][j]
            g11 = xrow(g01, rnd);
            w1 = xcol(w, rnd);
          } else {
            g01 = bpermz(g, aipj[rnd]); g10 = bpermz(g, apij[rnd]); g11 = bpermz(g, apipj[rnd]);
            w1 = bpermz(w, aipj[rnd]);
          }
          const bool rotj = (f & 8) && csj.y != 0.0, roti = (f & 16) && csi.y != 0.0;
          zc jjj, jpj, jii, jpi;
          jcol(f & 2, csj, ej, jjj, jpj);
          jcol(f & 4, csi, ei, jii, jpi);
          jjj = rotj ? jjj : c2(1, 0);
          jpj = rotj ? jpj : c2(0, 0);
          jii = roti ? jii : c2(1, 0);
          jpi = roti ? jpi : c2(0, 0);
          zc wn = cmul(w, jjj);
          cacc(wn, w1, jpj);
          zc r0 = cmul(g, jjj);
          cacc(r0, g01, jpj);
          zc r1 = cmul(g10, jjj);
          cacc(r1, g11, jpj);
          zc out = cjmul(jii, r0);
          cjacc(out, jpi, r1);
          const bool zero = rotj && roti && (f & 32);
          const bool diag = rotj && i == j;
          out = zero ? c2(0, 0) : out;
          out = diag ? c2(g.x + ((f & 2) ? -shj : shj), 0) : out;
#ifdef OCG_PROFILE
          if (tid == 0) PROF[30] += 1.0;  // rounds executed
#endif
          if (rnd == maxr - 1)  // convergence: the rotation predicate on the sweep's output
            flag = valid && i < j && jneed(cabs2(out), dpp, dqq);
          g = out;
          w = wn;
        }
        if (done || __ballot(flag) == 0) break;
      }
      if (sweep == 40 && lane == 0 && P.err) atomicOr(P.err, OCG_ERR_JACOBI);  // not converged: surfaced as OCG_ENUM
#ifdef OCG_PROFILE
      if (tid == 0) { PROF[20] += sweep + 1; PROF[21] += 1.0; PROF[22] += maxr; }  // sweeps, calls, rounds/sweep
#endif
      if (valid) {
        Gc[loc] = g;
        Wc[loc] = w;
      }
      // for the truncation: eigenvalue (clamped at 0), its rank inside the
      // block (descending, ties by index) and its sector, from the diagonal
      // lanes of the block (both waves, no LDS round trip)
      const double lam = g.x > 0 ? g.x : 0.0;
      int jb = 0;
#pragma unroll
      for (int t = 0; t < S; ++t) {
        const double lt = bperm(lam, at(t, t));
        jb += (t < n && t != i && (lt > lam || (lt == lam && t < i))) ? 1 : 0;
      }
      if (valid && i == j) {
        LAM[eo + i] = lam;
        JB[eo + i] = jb;
        EQ[eo + i] = q;
      }
    }
  }

  // gd: Gram descriptors of a plan hit (the register path forms the Gram
  // elements itself; only for 1 <= maxr <= 7)
  __device__ OCG_INLINE void jacobi(lzp& Gc, lzp& Wc, const LDS int* gd = nullptr) {
    constexpr int JB_IT = 4, JA_IT = 2;
    lzp Gn = (Gc == G) ? G2 : G;
    lzp Wn = (Wc == W) ? W2 : W;
    const int maxr = ISCAL[I_MAXROUNDS];
    if (maxr <= 0) return;
    if (maxr <= 3) {  // every block of order <= 4
      pf(13);
      jacobi_reg<4>(Gc, Wc, maxr, gd);
      sync();
      return;
    }
    if (maxr <= 7) {  // every block of order <= 8
      pf(13);
      jacobi_reg<8>(Gc, Wc, maxr, gd);
      sync();
      return;
    }
    const int npair = POFF[P.Q1];
    const int nel = GOFF[P.Q1];
    JD dB[JB_IT];
    JP dA[JA_IT];
    // every block small enough for the pairing table and all elements cached
    const bool fast = maxr <= kPairRounds && nel <= JB_IT * NT;
#pragma unroll
    for (int it = 0; it < JB_IT; ++it) dB[it] = jd_of(it * NT + tid, nel);
#pragma unroll
    for (int it = 0; it < JA_IT; ++it) dA[it] = jp_of(it * NT + tid, npair);
    int sweep = 0;
    for (; sweep < 40; ++sweep) {
      const int fl = I_FLAG + sweep % 3;
      for (int rnd = 0; rnd < maxr; ++rnd) {
        if (rnd == 0 && tid == 0) ISCAL[I_FLAG + (sweep + 1) % 3] = 0;
        pf(13);
#pragma unroll
        for (int it = 0; it < JA_IT; ++it)
          if (it * NT < npair) jrot(dA[it], it * NT + tid, rnd, Gc);
        for (int t = JA_IT * NT + tid; t < npair; t += NT) jrot(jp_of(t, npair), t, rnd, Gc);
        sync();
        pf(14);
        const bool lastr = rnd == maxr - 1;
        if (fast) {
#pragma unroll
          for (int it = 0; it < JB_IT; ++it)
            if (it * NT < nel) jupd_fast(dB[it], it * NT + tid < nel, rnd, Gc, Wc, Gn, Wn, lastr, fl);
        } else {
#pragma unroll
          for (int it = 0; it < JB_IT; ++it) jupd(dB[it], rnd, Gc, Wc, Gn, Wn, lastr, fl);
        }
        for (int e = JB_IT * NT + tid; e < nel; e += NT) jupd(jd_of(e, nel), rnd, Gc, Wc, Gn, Wn, lastr, fl);
        sync();
        pf(3);
        lzp tg = Gc; Gc = Gn; Gn = tg;
        lzp tw = Wc; Wc = Wn; Wn = tw;
      }
      const int more = ISCAL[fl];
      if (!more) break;
    }
    if (sweep == 40 && tid == 0 && P.err) atomicOr(P.err, OCG_ERR_JACOBI);  // not converged: surfaced as OCG_ENUM
#ifdef OCG_PROFILE
    if (tid == 0) { PROF[20] += sweep + 1; PROF[21] += 1.0; PROF[22] += maxr; }  // sweeps, calls, rounds/sweep
#endif
  }

  // ------------------------------------------------------------- decomposition
  // Block decomposition of TH (blocks THR x THC at THO) with truncation:
  //   Fromleft : TH = X Y, X orthonormal columns (left factor), Y carries norm
  //   Fromright: TH = X Y, Y orthonormal rows, X carries norm
  // The Gram matrix is formed on the smaller side of each block; the factor
  // on the other side is derived from TH.
  // If `normalize`, the norm-carrying factor is divided by sqrt(kept weight).
  // ts > 0: two-site update of sites (ts, ts+1): the new bond ts is written
  // to DIMS and X / Y go straight into the site tensors (rows (n1, a) of
  // site ts, cols (n2, c) of site ts+1) instead of the X / Y scratch.
  // `bound` = per-sector rank bound of the new bond (MD row, or MDZ row in
  // the dH zip-up); vectors beyond it are numerically zero and dropped.
  __device__ OCG_INLINE void decompose(int dir, double cutoff, int maxm, bool normalize, const LDS int* bound,
                                       int ts = 0) {
    pf(16);
    const int Q1 = P.Q1;
    if (phit) {  // Gram layout from the plan
      if (w0) {
        if (lane < Q1) KEPT[lane] = 0;
        if (lane == 0) {
          ISCAL[I_MAXROUNDS] = ps[2];
          ISCAL[I_FLAG] = 0; ISCAL[I_FLAG + 1] = 0; ISCAL[I_FLAG + 2] = 0;
        }
      }
    } else if (w0) {
      const int q = lane;
      const int R = q < Q1 ? THR[q] : 0, C = q < Q1 ? THC[q] : 0;
      const int n = (R == 0 || C == 0) ? 0 : (R <= C ? R : C);
      const int m = (n >= 2) ? (n + (n & 1)) : 0;
      const int ig = wscan(n * n), ie = wscan(n), ip = wscan(m / 2), mr = wscan_max(m > 0 ? m - 1 : 0);
      if (q < Q1) {
        NQ[q] = n; SIDE[q] = (R <= C) ? 0 : 1;  // 0: rows side (TH TH^H), 1: cols side (TH^H TH)
        MQ[q] = m; GOFF[q] = ig - n * n; EOFF[q] = ie - n; POFF[q] = ip - m / 2;
        KEPT[q] = 0;
      }
      if (lane == 63) {  // inclusive scans: lane 63 holds the totals
        GOFF[Q1] = ig; EOFF[Q1] = ie; POFF[Q1] = ip;
        ISCAL[I_MAXROUNDS] = mr;
        if (ps) ps[2] = mr;
        ISCAL[I_FLAG] = 0; ISCAL[I_FLAG + 1] = 0; ISCAL[I_FLAG + 2] = 0;
      }
    }
    sync();
#ifdef OCG_FAST_TRACE  // CPU emulation diagnostics: block orders of decompositions beyond the register Jacobi
    if (tid == 0 && ISCAL[I_MAXROUNDS] > 7) {
      printf("[lds-jacobi] orders");
      for (int q = 0; q < Q1; ++q) printf(" %d", NQ[q]);
      printf("\n");
    }
#endif
    pf(2);
    // Gram matrices and identity eigenvectors (on a plan hit with blocks of
    // order 2..8 the register Jacobi forms them itself)
    const bool fuse = phit && ps[2] >= 1 && ps[2] <= 7;
    if (fuse) {
    } else if (phit) {
      const int nel = GOFF[Q1];
      const LDS int* gdp = ps + pl.GD;
      for (int e = tid; e < nel; e += NT) {
        const unsigned a0 = gdp[2 * e], a1 = gdp[2 * e + 1];
        const int st = a1 & 0xfff, len = (a1 >> 12) & 0xfff;
        lzp Ta = TH + int(a0 & 0xffff), Tb = TH + int(a0 >> 16);
        zc acc = c2(0, 0);
        if (((a1 >> 24) & 1) == 0) {
          for (int c = 0; c < len; ++c) cacc(acc, Ta[c * st], cconj(Tb[c * st]));
        } else {
          for (int r = 0; r < len; ++r) cjacc(acc, Ta[r * st], Tb[r * st]);
        }
        G[e] = acc;
        W[e] = ((a1 >> 25) & 1) ? c2(1, 0) : c2(0, 0);
      }
    } else {
      const int nel = GOFF[Q1];
      for (int base = 0; base < nel; base += NT) {
        const int e = base + tid;
        const int q = blk(GOFF, e);
        if (e < nel) {
          const int n = NQ[q];
          int j;
          const int i = udiv(e - GOFF[q], n, j);
          lzp T = TH + THO[q];
          const int R = THR[q], C = THC[q];
          zc acc = c2(0, 0);
          if (SIDE[q] == 0) {
            for (int c = 0; c < C; ++c) cacc(acc, T[i * C + c], cconj(T[j * C + c]));
          } else {
            for (int r = 0; r < R; ++r) cjacc(acc, T[r * C + i], T[r * C + j]);
          }
          G[e] = acc;
          W[e] = (i == j) ? c2(1, 0) : c2(0, 0);
          if (ps && e < P.plan_pe) {
            const int o = THO[q], s0 = SIDE[q] == 0;
            ps[pl.GD + 2 * e] = (s0 ? o + i * C : o + i) | ((s0 ? o + j * C : o + j) << 16);
            ps[pl.GD + 2 * e + 1] = (s0 ? 1 : C) | ((s0 ? C : R) << 12) | ((s0 ? 0 : 1) << 24) | ((i == j) << 25);
          }
        }
      }
      // derived-factor products Θ w (cols-side blocks) / w^H Θ (rows-side
      // blocks) for every eigenvector: offsets PDO and descriptors PD
      // (Θ base, W base, length | side << 16, Θ stride | W stride << 16)
      if (NW >= 2 && ps && w0) {
        const int q = lane;
        int sz = 0;
        if (q < Q1 && NQ[q] > 0) sz = SIDE[q] ? THR[q] * NQ[q] : NQ[q] * THC[q];
        const int inc = wscan(sz);
        if (q < Q1) ps[pl.PDO + q] = inc - sz;
        if (lane == 63) ps[pl.PDO + Q1] = inc;
        wsync();
        const int tot = ps[pl.PDO + Q1];
        for (int e = lane; e < tot && e < P.plan_pe; e += 64) {
          const int qq = blk(ps + pl.PDO, e);
          const int n = NQ[qq], R = THR[qq], C = THC[qq], o = THO[qq], g = GOFF[qq], x = e - ps[pl.PDO + qq];
          LDS int* dd = ps + pl.PD + 4 * e;
          if (SIDE[qq]) {  // X[row][w] = sum_c Θ[row][c] W[c][w]
            int w;
            const int row = udiv(x, n, w);
            dd[0] = o + row * C; dd[1] = g + w; dd[2] = C | (1 << 16); dd[3] = 1 | (n << 16);
          } else {  // Y[w][col] = sum_r conj(W[r][w]) Θ[r][col]
            int col;
            const int w = udiv(x, C, col);
            dd[0] = o + col; dd[1] = g + w; dd[2] = R; dd[3] = C | (n << 16);
          }
        }
      }
    }
    if (!fuse) sync();
    lzp Gc = G;
    lzp Wc = W;
    pf(3);
    jacobi(Gc, Wc, fuse ? ps + pl.GD : nullptr);
    pf(4);
    // eigenvalues (clamped at 0) and their blocks
    const int T = EOFF[Q1];
    if (T <= 64) {
      // one wave: ranking, truncation and the kept set in registers, ballot
      // counts per sector, wave-level fences instead of block barriers
      // the register Jacobi (1 <= maxr <= 7) left LAM / JB / EQ behind
      const int mr_ = ISCAL[I_MAXROUNDS];
      const bool regj = mr_ >= 1 && mr_ <= 7;
      if (NW >= 2 && phit && tid >= 64 && tid < 128) {
        // wave 1, meanwhile: the derived-factor products for every eigenvector
        // into CR (the factor phase then only selects and scales them); same
        // sums in the same order as the factor phase's own loops
        const int tot = ps[pl.PDO + Q1];
        if (tot <= P.plan_pe)
          for (int e = lane; e < tot; e += 64) {
            const i4 dd = *(const LDS i4*)(ps + pl.PD + 4 * e);
            const int len = dd[2] & 0xffff, ts_ = dd[3] & 0xffff, ws = unsigned(dd[3]) >> 16;
            lzp Ta = TH + dd[0], Wg = Wc + dd[1];
            zc acc = c2(0, 0);
            if (dd[2] >> 16) {
              for (int c = 0; c < len; ++c) cacc(acc, Ta[c * ts_], Wg[c * ws]);
            } else {
              for (int r = 0; r < len; ++r) cjacc(acc, Wg[r * ws], Ta[r * ts_]);
            }
            CR[e] = acc;
          }
      }
      if (w0) {
        const int e = lane;
        const bool act = e < T;
        int q = 0;
        double lam = 0.0;
        if (regj) {
          if (act) { q = EQ[e]; lam = LAM[e]; }
        } else {
          q = blk(EOFF, e);
          if (act) {
            const int i = e - EOFF[q], n = NQ[q];
            const double g = zc(Gc[GOFF[q] + i * n + i]).x;
            lam = g > 0 ? g : 0.0;
            LAM[e] = lam;
          }
        }
        // Truncation (ITensor truncate; relative cutoff; floor 1e-30): in the
        // spectrum sorted descending (ties by flat index), position j >= 1 is
        // discarded iff j >= maxm, or the weight from j to the end is below
        // cutoff * total, or PP[j] <= 1e-30 total; the discarded set is a
        // suffix.  kept: not discarded and within the sector's rank bound,
        // ordered inside its block by descending weight (rank jb).
        bool kept = false;
        int m;
        double total;
        if (T <= maxm) {
          // maxm cannot bind: only eigenvalues below max(cut, floor) can be
          // discarded, and every other one ranks ahead of them, so the
          // suffix weights and ranks need the small ones alone (usually none)
          total = wsum(lam);
          const double cut = cutoff * total, floor_ = 1e-30 * total, thr = fmax(cut, floor_);
          int jb = 0;
          if (regj) {
            if (act) jb = JB[e];
          } else {
            const int eo = act ? EOFF[q] : 0, nq = act ? NQ[q] : 0;
            const int maxn = mr_ + 2;  // >= every block order
            for (int t = 0; t < maxn; ++t) {
              const int f = eo + t;
              const double lf = bperm(lam, (f & 63) << 2);
              jb += (t < nq && f != e && (lf > lam || (lf == lam && f < e))) ? 1 : 0;
            }
          }
          const bool small = act && (lam < thr || lam <= floor_);
          unsigned long long M = __ballot(small);
          bool disc = false;
          if (M) {
            const int nbig = T - __popcll(M);
            double S = lam;
            int rs = 0;
            while (M) {
              const int f = __ffsll((long long)M) - 1;
              M &= M - 1;
              const double lf = rdlane(lam, f);
              rs += (lf > lam || (lf == lam && f < e)) ? 1 : 0;
              if (f != e && (lf < lam || (lf == lam && f > e))) S += lf;
            }
            disc = small && nbig + rs >= 1 && (S < cut || lam <= floor_);
          }
          m = T - __popcll(__ballot(disc));
          kept = act && !disc && jb < bound[q];
          if (kept) KIDX[EOFF[q] + jb] = e - EOFF[q];
        } else {
          if (act) EQ[e] = q;
          wsync();
          // global rank (descending; ties by flat index) and rank within the block
          int rk = 0, jb = 0;
          if (act) {
            int f = 0;
            for (; f + 3 < T; f += 4) {
              const double l0 = LAM[f], l1 = LAM[f + 1], l2 = LAM[f + 2], l3 = LAM[f + 3];
              const int b0 = EQ[f], b1 = EQ[f + 1], b2 = EQ[f + 2], b3 = EQ[f + 3];
              const int c0 = (l0 > lam) || (l0 == lam && f < e), c1 = (l1 > lam) || (l1 == lam && f + 1 < e);
              const int c2_ = (l2 > lam) || (l2 == lam && f + 2 < e), c3 = (l3 > lam) || (l3 == lam && f + 3 < e);
              rk += c0 + c1 + c2_ + c3;
              jb += (c0 & (b0 == q)) + (c1 & (b1 == q)) + (c2_ & (b2 == q)) + (c3 & (b3 == q));
            }
            for (; f < T; ++f) {
              const double lf = LAM[f];
              const int c = (lf > lam) || (lf == lam && f < e);
              rk += c;
              jb += c & (EQ[f] == q);
            }
            PP[rk] = lam;
          }
          wsync();
          total = wsum(act ? PP[lane] : 0.0);
          const double cut = cutoff * total, floor_ = 1e-30 * total;
          const int j = T - 1 - lane;  // lane 0 = smallest
          const double v = j >= 0 ? PP[j] : 0.0;
          const double suf = wscan(v);
          const bool disc = j >= 1 && (j >= maxm || suf < cut || v <= floor_);
          m = T - __popcll(__ballot(disc));
          kept = act && rk < m && jb < bound[q];
          if (kept) KIDX[EOFF[q] + jb] = e - EOFF[q];
        }
        pf(18);
        const double kw = wsum(kept ? lam : 0.0);
        int kq = 0;
        for (int s = 0; s < Q1; ++s) {
          const int c = __popcll(__ballot(kept && q == s));
          kq = (lane == s) ? c : kq;
        }
        // factor plan: 1 = the slot's factor layout matches kq, 2 = record it
        int p2 = 0;
        if (ps) {
          const bool same = phit && ps[3] != 0 && __ballot(lane < Q1 && ps[pl.KK + lane] != kq) == 0;
          p2 = same ? 1 : 2;
        }
        if (lane < Q1) KEPT[lane] = kq;
        if (p2 == 2 && lane < Q1) ps[pl.KK + lane] = kq;
        if (lane == 0) { ISCAL[I_M] = m; SCAL[S_TOTAL] = total; SCAL[S_KEPTW] = kw; ISCAL[I_P2] = p2; }
        if (p2 != 1) {
          const int R = lane < Q1 ? THR[lane] : 0, C = lane < Q1 ? THC[lane] : 0;
          const int ix = wscan(R * kq), iy = wscan(kq * C);
          if (lane < Q1) { XOFF[lane] = ix - R * kq; YOFF[lane] = iy - kq * C; }
          if (lane == 63) { XOFF[Q1] = ix; YOFF[Q1] = iy; }
        }
        pf(19);
        if (ts) {  // two-site update: new bond ts and the layouts of sites ts, ts+1
          if (lane < Q1) DIMS[ts * Q1 + lane] = kq;
          if (p2 == 1) {
            for (int i = lane; i <= SEG; i += 64) {
              boff(ts)[i] = ps[pl.BO1 + i];
              boff(ts + 1)[i] = ps[pl.BO2 + i];
            }
          } else {
            wsync();
            site_offsets(ts);
            site_offsets(ts + 1);
            if (p2 == 2) {
              wsync();
              for (int i = lane; i <= SEG; i += 64) {
                ps[pl.BO1 + i] = boff(ts)[i];
                ps[pl.BO2 + i] = boff(ts + 1)[i];
              }
            }
          }
        }
      }
      sync();
    } else {
      {
        for (int base = 0; base < T; base += NT) {
          const int e = base + tid;
          const int q = blk(EOFF, e);
          if (e < T) {
            const int i = e - EOFF[q], n = NQ[q];
            const double lam = zc(Gc[GOFF[q] + i * n + i]).x;
            LAM[e] = lam > 0 ? lam : 0.0;
            EQ[e] = q;
          }
        }
      }
      sync();
      // global rank (descending; ties by flat index) and rank within the block
      // (the competitors are read as LDS broadcasts, four in flight)
      for (int e = tid; e < T; e += NT) {
        const double le = LAM[e];
        const int be = EQ[e];
        int rk = 0, jb = 0;
        int f = 0;
        for (; f + 3 < T; f += 4) {
          const double l0 = LAM[f], l1 = LAM[f + 1], l2 = LAM[f + 2], l3 = LAM[f + 3];
          const int b0 = EQ[f], b1 = EQ[f + 1], b2 = EQ[f + 2], b3 = EQ[f + 3];
          const int c0 = (l0 > le) || (l0 == le && f < e), c1 = (l1 > le) || (l1 == le && f + 1 < e);
          const int c2_ = (l2 > le) || (l2 == le && f + 2 < e), c3 = (l3 > le) || (l3 == le && f + 3 < e);
          rk += c0 + c1 + c2_ + c3;
          jb += (c0 & (b0 == be)) + (c1 & (b1 == be)) + (c2_ & (b2 == be)) + (c3 & (b3 == be));
        }
        for (; f < T; ++f) {
          const double lf = LAM[f];
          const int c = (lf > le) || (lf == le && f < e);
          rk += c;
          jb += c & (EQ[f] == be);
        }
        RANK[e] = rk;
        JB[e] = jb;
        PP[rk] = le;
      }
      sync();
      // truncation (ITensor truncate; relative cutoff; floor 1e-30): the
      // discarded set {j >= 1 : j >= maxm or sum_{i>=j} PP[i] < cutoff*total or
      // PP[j] <= 1e-30 total} is a suffix of the sorted spectrum
      if (w0) {
        double total = 0;
        for (int b = 0; b < T; b += 64) total += wsum((b + lane < T) ? PP[b + lane] : 0.0);
        const double cut = cutoff * total, floor_ = 1e-30 * total;
        double carry = 0;
        int nd = 0;
        for (int cb = 0; cb < T; cb += 64) {
          const int j = T - 1 - cb - lane;  // lane 0 = smallest
          const double v = j >= 0 ? PP[j] : 0.0;
          const double inc = wscan(v);
          const double suf = carry + inc;
          const bool disc = j >= 1 && (j >= maxm || suf < cut || v <= floor_);
          nd += __popcll(__ballot(disc));
          carry += rdlane(inc, 63);
        }
        if (lane == 0) { ISCAL[I_M] = T - nd; SCAL[S_TOTAL] = total; ISCAL[I_P2] = 0; }
      }
      sync();
      // kept vectors: global rank < m and within the sector's rank bound
      {
        const int m = ISCAL[I_M];
        double kw = 0;
        for (int e = tid; e < T; e += NT) {
          const int q = EQ[e], jb = JB[e];
          if (RANK[e] < m && jb < bound[q]) {
            __hip_atomic_fetch_add(&KEPT[q], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // ds_add_u32
            KIDX[EOFF[q] + jb] = e - EOFF[q];
            kw += LAM[e];
          }
        }
        kw = block_sum(kw);
        if (tid == 0) SCAL[S_KEPTW] = kw;
      }
      sync();
      if (w0) {
        const int q = lane;
        const int k = q < Q1 ? KEPT[q] : 0, R = q < Q1 ? THR[q] : 0, C = q < Q1 ? THC[q] : 0;
        const int ix = wscan(R * k), iy = wscan(k * C);
        if (q < Q1) { XOFF[q] = ix - R * k; YOFF[q] = iy - k * C; }
        if (lane == 63) { XOFF[Q1] = ix; YOFF[Q1] = iy; }
      }
      sync();
      if (ts) {
        if (w0 && lane < Q1) DIMS[ts * Q1 + lane] = KEPT[lane];
        sync();
        if (NW == 1) {
          site_offsets(ts);
          site_offsets(ts + 1);
        } else if (tid < 64) site_offsets(ts);
        else if (tid < 128) site_offsets(ts + 1);
        sync();
      }
    }
    pf(5);
    // materialise X (R x k) and Y (k x C) per block
    const double kwv = SCAL[S_KEPTW];
    const double inv = (normalize && kwv > 1e-32) ? 1.0 / sqrt(kwv) : 1.0;
    const int xt = XOFF[Q1], yt = YOFF[Q1];
    const int pm = ISCAL[I_P2];  // 1: factor plan, 2: record it
    if (pm == 1) {
      // X: exact side u = W[a + w], else Θ w (len terms, Θ stride st, W stride n).
      // With two or more waves, X goes to wave 0 and Y to wave 1 (the two
      // factors are independent), else one after the other.
      const int wv = tid >> 6;
      const int xs = NW >= 2 ? (wv == 0 ? lane : xt) : tid, xstep = NW >= 2 ? 64 : NT;
      const int ys = NW >= 2 ? (wv == 1 ? lane : yt) : tid, ystep = NW >= 2 ? 64 : NT;
      for (int e = xs; e < xt; e += xstep) {
        const i4 dd = *(const LDS i4*)(ps + pl.XD + 4 * e);
        const int a = dd[0] & 0xffff, g = unsigned(dd[0]) >> 16, dest = dd[1] & 0xffff, len = unsigned(dd[1]) >> 16;
        const int eb = dd[2] & 0xffff, j = unsigned(dd[2]) >> 16, n = dd[3] & 0xfff, st = (dd[3] >> 12) & 0x7ffff;
        const int w = KIDX[eb + j];
        const double sig = sqrt(LAM[eb + w]);
        zc out;
        if (dd[3] < 0) {
          out = Wc[a + w];
          if (dir == kFromright) out = cscale(out, sig * inv);
        } else {
          zc acc;
          if (NW >= 2) {
            acc = CR[a + w * g];  // precomputed Θ w (a: row base, g: w multiplier)
          } else {
            acc = c2(0, 0);
            lzp Ta = TH + a, Wg = Wc + g + w;
            for (int c = 0; c < len; ++c) cacc(acc, Ta[c * st], Wg[c * n]);
          }
          if (dir == kFromleft) out = (sig > 0) ? cscale(acc, 1.0 / sig) : c2(0, 0);
          else out = cscale(acc, inv);
        }
        // gauge move (ts = 0): the orthonormal factor goes to its site, the other to scratch
        if (ts || dir == kFromleft) A[dest] = out;
        else X[e] = out;
      }
      pf(23);
      // Y: exact side v^H = conj(W[a + w]), else w^H Θ
      for (int e = ys; e < yt; e += ystep) {
        const i4 dd = *(const LDS i4*)(ps + pl.YD + 4 * e);
        const int a = dd[0] & 0xffff, g = unsigned(dd[0]) >> 16, dest = dd[1] & 0xffff, len = unsigned(dd[1]) >> 16;
        const int eb = dd[2] & 0xffff, j = unsigned(dd[2]) >> 16, n = dd[3] & 0xfff, st = (dd[3] >> 12) & 0x7ffff;
        const int w = KIDX[eb + j];
        const double sig = sqrt(LAM[eb + w]);
        zc out;
        if (dd[3] < 0) {
          out = cconj(Wc[a + w]);
          if (dir == kFromleft) out = cscale(out, sig * inv);
        } else {
          zc acc;
          if (NW >= 2) {
            acc = CR[a + w * g];  // precomputed w^H Θ (a: column base, g: w multiplier)
          } else {
            acc = c2(0, 0);
            lzp Ta = TH + a, Wg = Wc + g + w;
            for (int r = 0; r < len; ++r) cjacc(acc, Wg[r * n], Ta[r * st]);
          }
          if (dir == kFromright) out = (sig > 0) ? cscale(acc, 1.0 / sig) : c2(0, 0);
          else out = cscale(acc, inv);
        }
        if (ts || dir == kFromright) A[dest] = out;
        else Y[e] = out;
      }
      sync();
      return;
    }
    for (int base = 0; base < xt; base += NT) {
      const int e = base + tid;
      const int q = blk(XOFF, e);
      if (e < xt) {
        const int k = KEPT[q], C = THC[q], n = NQ[q];
        int j;
        const int row = udiv(e - XOFF[q], k, j);
        const int w = KIDX[EOFF[q] + j];
        const double sig = sqrt(LAM[EOFF[q] + w]);
        lzp Tq = TH + THO[q];
        lzp Wq = Wc + GOFF[q];
        zc out;
        if (SIDE[q] == 0) {
          out = Wq[row * n + w];  // u exact
          if (dir == kFromright) out = cscale(out, sig * inv);
        } else {
          zc acc = c2(0, 0);  // Θ w
          for (int c = 0; c < C; ++c) cacc(acc, Tq[row * C + c], Wq[c * n + w]);
          if (dir == kFromleft) out = (sig > 0) ? cscale(acc, 1.0 / sig) : c2(0, 0);
          else out = cscale(acc, inv);
        }
        int dest = 0;
        if (ts) {  // rows (n1, a) of site ts
          int o;
          const int n1 = seg_in(TRO, q, row, o);
          dest = P.site_base[ts] + bo(ts, q - n1, n1) + (row - o) * k + j;
          A[dest] = out;
        } else X[e] = out;
        if (pm == 2 && e < P.plan_pe) {
          const bool ex = SIDE[q] == 0;
          LDS int* dd = ps + pl.XD + 4 * e;
          dd[0] = ex ? (GOFF[q] + row * n) | (GOFF[q] << 16)
                     : (NW >= 2 ? (ps[pl.PDO + q] + row * n) | (1 << 16) : (THO[q] + row * C) | (GOFF[q] << 16));
          dd[1] = dest | (C << 16);
          dd[2] = EOFF[q] | (j << 16);
          dd[3] = n | (1 << 12) | (ex ? int(0x80000000u) : 0);
        }
      }
    }
    pf(23);
    for (int base = 0; base < yt; base += NT) {
      const int e = base + tid;
      const int q = blk(YOFF, e);
      if (e < yt) {
        const int R = THR[q], C = THC[q], n = NQ[q];
        int col;
        const int j = udiv(e - YOFF[q], C, col);
        const int w = KIDX[EOFF[q] + j];
        const double sig = sqrt(LAM[EOFF[q] + w]);
        lzp Tq = TH + THO[q];
        lzp Wq = Wc + GOFF[q];
        zc out;
        if (SIDE[q] == 1) {
          out = cconj(Wq[col * n + w]);  // v^H exact
          if (dir == kFromleft) out = cscale(out, sig * inv);
        } else {
          zc acc = c2(0, 0);  // w^H Θ
          for (int r = 0; r < R; ++r) cjacc(acc, Wq[r * n + w], Tq[r * C + col]);
          if (dir == kFromright) out = (sig > 0) ? cscale(acc, 1.0 / sig) : c2(0, 0);
          else out = cscale(acc, inv);
        }
        int dest = 0;
        if (ts) {  // cols (n2, c) of site ts+1
          int o;
          const int n2 = seg_in(TCO, q, col, o);
          dest = P.site_base[ts + 1] + bo(ts + 1, q, n2) + j * d(ts + 1, q + n2) + (col - o);
          A[dest] = out;
        } else Y[e] = out;
        if (pm == 2 && e < P.plan_pe) {
          const bool ex = SIDE[q] == 1;
          LDS int* dd = ps + pl.YD + 4 * e;
          dd[0] = ex ? (GOFF[q] + col * n) | (GOFF[q] << 16)
                     : (NW >= 2 ? (ps[pl.PDO + q] + col) | (C << 16) : (THO[q] + col) | (GOFF[q] << 16));
          dd[1] = dest | (R << 16);
          dd[2] = EOFF[q] | (j << 16);
          dd[3] = n | (C << 12) | (ex ? int(0x80000000u) : 0);
        }
      }
    }
    sync();
    if (pm == 2 && tid == 0)
      ps[3] = (xt <= P.plan_pe && yt <= P.plan_pe && (NW < 2 || ps[pl.PDO + Q1] <= P.plan_pe)) ? 1 : 0;
  }

  // single-site matricisation of site k into TH
  //   left (Fromleft grouping): rows (n, a in bond k-1 sector q-n), cols c in bond k sector q
  //   right (Fromright grouping): rows a in bond k-1 sector q, cols (n, c in bond k sector q+n)
  __device__ OCG_INLINE void site_to_theta(int k, bool left) {
    pf(7);
    if (phit) {  // plan: source offset of every matricised element
      pf(28);
      const int tot = ps[1];
      const LDS int* bt = ps + pl.BT;
      for (int e = tid; e < tot; e += NT) TH[e] = A[bt[2 * e]];
      sync();
      return;
    }
    int tot;
    if (left)
      tot = theta_tables([&](int q, int n) { return d(k - 1, q - n); },
                         [&](int q, int n) { return n == 0 ? d(k, q) : 0; });
    else
      tot = theta_tables([&](int q, int n) { return n == 0 ? d(k - 1, q) : 0; },
                         [&](int q, int n) { return d(k, q + n); });
    pf(28);
    for (int base = 0; base < tot; base += NT) {
      const int e = base + tid;
      const int q = blk(THO, e);
      if (e < tot) {
        const int C = THC[q];
        int col, o;
        const int row = udiv(e - THO[q], C, col);
        int src;
        if (left) {
          const int n = seg_in(TRO, q, row, o);
          src = bo(k, q - n, n) + (row - o) * C + col;
        } else {
          const int n = seg_in(TCO, q, col, o);
          src = bo(k, q, n) + row * d(k, q + n) + (col - o);
        }
        src += P.site_base[k];
        TH[e] = A[src];
        if (ps && e < P.plan_pe) ps[pl.BT + 2 * e] = src;
      }
    }
    sync();
    plan_commit(tot);
  }

  // move the orthogonality centre k -> k+1 (ITensor position, one bond).
  // slot >= 0: plan slot of this gauge move (see plans); on a plan hit the
  // decomposition writes X straight into site k and the neighbour product
  // and the new offset tables come from the slot.
  __device__ OCG_INLINE void gauge_right(int k, double cutoff, int maxm, int slot = -1) {
    plan_begin(slot);
    site_to_theta(k, true);
    decompose(kFromleft, cutoff, maxm, false, MD + k * P.Q1);
    pf(24);
    const int pm = ps ? ISCAL[I_P2] : 0;  // 1: plan hit, 2: record
    if (pm == 1) {
      pf(25);
      const int ns = ps[pl.BO1 + SEG];
      const LDS int* sd = ps + pl.SD;
      for (int e = tid; e < ns; e += NT) {  // S = Y * A_{k+1}
        const i4 dd = *(const LDS i4*)(sd + 4 * e);
        lzp Yq = Y + dd[0];
        lzp Ab = A + dd[1];
        zc acc = c2(0, 0);
        for (int b = 0; b < dd[2]; ++b) cacc(acc, Yq[b], Ab[b * dd[3]]);
        S[e] = acc;
      }
      sync();
      pf(26);
      if (w0 && lane < P.Q1) DIMS[k * P.Q1 + lane] = KEPT[lane];
      for (int i = tid; i <= SEG; i += NT) {
        boff(k)[i] = ps[pl.BO2 + i];
        boff(k + 1)[i] = ps[pl.BO1 + i];
      }
      for (int e = tid; e < ns; e += NT) site(k + 1)[e] = S[e];
      sync();
      plan_end();
      return;
    }
    // new layout of site k+1 (rows = new bond k) into BOFFT
    if (w0) {
      scan_excl(BOFFT, SEG, [&](int s) {
        int q, n;
        qn_of(s, q, n);
        return KEPT[q] * d(k + 1, q + n);
      }, QST);
      if (pm == 2) {
        wsync();
        for (int i = lane; i <= SEG; i += 64) ps[pl.BO1 + i] = BOFFT[i];
      }
    }
    sync();
    pf(25);
    // S = Y * A_{k+1}   (per (q, n): k_q x d(k+1, q+n))
    const int ns = BOFFT[SEG];
    {
      for (int base = 0; base < ns; base += NT) {
        const int e = base + tid;
        int q, n, o;
        find_qn(BOFFT, e, q, n, o);
        if (e < ns) {
          const int cc = d(k + 1, q + n), dold = d(k, q);
          int c;
          const int i = udiv(e - o, cc, c);
          const int yo = YOFF[q] + i * dold, ao = P.site_base[k + 1] + bo(k + 1, q, n) + c;
          lzp Yq = Y + yo;
          lzp Ab = A + ao;
          zc acc = c2(0, 0);
          for (int b = 0; b < dold; ++b) cacc(acc, Yq[b], Ab[b * cc]);
          S[e] = acc;
          if (pm == 2 && e < P.plan_pe) {
            LDS int* dd = ps + pl.SD + 4 * e;
            dd[0] = yo; dd[1] = ao; dd[2] = dold; dd[3] = cc;
          }
        }
      }
    }
    sync();
    pf(26);
    if (w0 && lane < P.Q1) DIMS[k * P.Q1 + lane] = KEPT[lane];
    sync();
    if (w0) {
      site_offsets(k);
      if (pm == 2) {
        wsync();
        for (int i = lane; i <= SEG; i += 64) ps[pl.BO2 + i] = boff(k)[i];
      }
    }
    for (int i = tid; i <= SEG; i += NT) boff(k + 1)[i] = BOFFT[i];
    sync();
    pf(27);
    // A_k <- X ; A_{k+1} <- S
    const int xt = XOFF[P.Q1];
    for (int base = 0; base < xt; base += NT) {
      const int e = base + tid;
      const int q = blk(XOFF, e);
      if (e < xt) {
        const int kq = KEPT[q];
        int j, o;
        const int row = udiv(e - XOFF[q], kq, j);
        const int n = seg_in(TRO, q, row, o);
        const int dest = P.site_base[k] + bo(k, q - n, n) + (row - o) * kq + j;
        A[dest] = X[e];
        if (pm == 2 && e < P.plan_pe) {
          LDS int* dd = ps + pl.XD + 4 * e;
          dd[1] = (dd[1] & int(0xffff0000u)) | dest;
        }
      }
    }
    for (int e = tid; e < ns; e += NT) site(k + 1)[e] = S[e];
    sync();
    if (pm == 2 && tid == 0) ps[3] = (ps[3] != 0 && ns <= P.plan_pe) ? 1 : 0;
    plan_end();
  }

  // move the orthogonality centre k -> k-1 (on a plan hit Y goes straight
  // into site k)
  __device__ OCG_INLINE void gauge_left(int k, double cutoff, int maxm, int slot = -1) {
    plan_begin(slot);
    site_to_theta(k, false);
    decompose(kFromright, cutoff, maxm, false, MD + (k - 1) * P.Q1);
    pf(24);
    const int pm = ps ? ISCAL[I_P2] : 0;
    if (pm == 1) {
      pf(25);
      const int ns = ps[pl.BO1 + SEG];
      const LDS int* sd = ps + pl.SD;
      for (int e = tid; e < ns; e += NT) {  // S = A_{k-1} * X
        const i4 dd = *(const LDS i4*)(sd + 4 * e);
        lzp Ab = A + dd[0];
        lzp Xq = X + dd[1];
        zc acc = c2(0, 0);
        for (int b = 0; b < dd[2]; ++b) cacc(acc, Ab[b], Xq[b * dd[3]]);
        S[e] = acc;
      }
      sync();
      pf(26);
      if (w0 && lane < P.Q1) DIMS[(k - 1) * P.Q1 + lane] = KEPT[lane];
      for (int i = tid; i <= SEG; i += NT) {
        boff(k)[i] = ps[pl.BO2 + i];
        boff(k - 1)[i] = ps[pl.BO1 + i];
      }
      for (int e = tid; e < ns; e += NT) site(k - 1)[e] = S[e];
      sync();
      plan_end();
      return;
    }
    // new layout of site k-1 (cols = new bond k-1) into BOFFT
    if (w0) {
      scan_excl(BOFFT, SEG, [&](int s) {
        int ql, n;
        qn_of(s, ql, n);
        return (ql + n <= P.Q) ? d(k - 2, ql) * KEPT[ql + n] : 0;
      }, QST);
      if (pm == 2) {
        wsync();
        for (int i = lane; i <= SEG; i += 64) ps[pl.BO1 + i] = BOFFT[i];
      }
    }
    sync();
    pf(25);
    // S = A_{k-1} * X   (per (ql, n): d(k-2, ql) x k_{ql+n})
    const int ns = BOFFT[SEG];
    {
      for (int base = 0; base < ns; base += NT) {
        const int e = base + tid;
        int ql, n, o;
        find_qn(BOFFT, e, ql, n, o);
        if (e < ns) {
          const int q = ql + n, kq = KEPT[q], dold = d(k - 1, q);
          int j;
          const int i = udiv(e - o, kq, j);
          const int ao = P.site_base[k - 1] + bo(k - 1, ql, n) + i * dold, xo = XOFF[q] + j;
          lzp Ab = A + ao;
          lzp Xq = X + xo;
          zc acc = c2(0, 0);
          for (int b = 0; b < dold; ++b) cacc(acc, Ab[b], Xq[b * kq]);
          S[e] = acc;
          if (pm == 2 && e < P.plan_pe) {
            LDS int* dd = ps + pl.SD + 4 * e;
            dd[0] = ao; dd[1] = xo; dd[2] = dold; dd[3] = kq;
          }
        }
      }
    }
    sync();
    pf(26);
    if (w0 && lane < P.Q1) DIMS[(k - 1) * P.Q1 + lane] = KEPT[lane];
    sync();
    if (w0) {
      site_offsets(k);
      if (pm == 2) {
        wsync();
        for (int i = lane; i <= SEG; i += 64) ps[pl.BO2 + i] = boff(k)[i];
      }
    }
    for (int i = tid; i <= SEG; i += NT) boff(k - 1)[i] = BOFFT[i];
    sync();
    pf(27);
    const int yt = YOFF[P.Q1];
    for (int base = 0; base < yt; base += NT) {
      const int e = base + tid;
      const int q = blk(YOFF, e);
      if (e < yt) {
        const int C = THC[q];
        int col, o;
        const int j = udiv(e - YOFF[q], C, col);
        const int n = seg_in(TCO, q, col, o);
        const int dest = P.site_base[k] + bo(k, q, n) + j * d(k, q + n) + (col - o);
        A[dest] = Y[e];
        if (pm == 2 && e < P.plan_pe) {
          LDS int* dd = ps + pl.YD + 4 * e;
          dd[1] = (dd[1] & int(0xffff0000u)) | dest;
        }
      }
    }
    for (int e = tid; e < ns; e += NT) site(k - 1)[e] = S[e];
    sync();
    if (pm == 2 && tid == 0) ps[3] = (ps[3] != 0 && ns <= P.plan_pe) ? 1 : 0;
    plan_end();
  }

  // gslot: running index of the step's gauge moves (plan slots follow the
  // gate slots); null for callers outside a step (no plans)
  __device__ OCG_INLINE void position(int& centre, int target, int* gslot = nullptr) {
    while (centre != target) {
      const int slot = gslot ? P.ngates + (*gslot)++ : -1;
      pf(pf_cur);
      pf_gauge = 1;
      if (centre < target) { gauge_right(centre, OCG_GAUGE_CUTOFF, 1 << 30, slot); ++centre; }
      else { gauge_left(centre, OCG_GAUGE_CUTOFF, 1 << 30, slot); --centre; }
      pf(pf_cur);
      pf_gauge = 0;
    }
  }

  // ------------------------------------------------------------- step
  // BH_tDMRG::step (src/BH_tDMRG.cpp:111-125) + doStep (:127-230).
  // The gate loop is written with one decompose call site and one gauge-move
  // call site so the (large) decomposition is inlined only twice.
  // final_gauge = false (trajectory chains except their last step, Hessian
  // rows): the closing position(1) (:206-218) is left out and the
  // orthogonality centre stays on the last gate's left site, which is
  // normalised instead of site 1.  The state is the same (the move only
  // regauges sites 1-2 and drops directions below the 1e-14 gauge cutoff),
  // and everything that follows — the next step's first gate contracts sites
  // 1 and 2 into one Θ; overlaps, norms; exactApplyMPO, whose zip-up sees an
  // isometry at site 1 — is gauge invariant, so a chain saves one of its six
  // decompositions per step.  ocg_steps keeps the closing move.
  __device__ OCG_INLINE void step(double ufrom, double uto, int forward, bool final_gauge = true) {
    const int L = P.L, p = P.p;
    const double tau = forward ? P.dt : -P.dt;
    pf(29);
    // U phases exp(-i u tau n(n-1) / 4) (initUGates, :74-108).  Consecutive
    // steps of a chain share a control value (this step's u_from is the last
    // step's u_to, same direction), so only the new set is evaluated.  The
    // first reader is apply_gate, behind build_theta's barrier.
    if (tid < p) {
      const double nn = double(tid) * double(tid - 1);
      double s, c;
      zc f;
      if (ufrom == ph_u && forward == ph_dir) {
        f = PH[p + tid];
      } else if (P.imag) {
        f = c2(exp(-0.25 * ufrom * tau * nn), 0.0);  // exp(-tau U/4 n(n-1)): imaginary time
      } else {
        sincos(-0.25 * ufrom * tau * nn, &s, &c);
        f = c2(c, s);
      }
      PH[tid] = f;
      if (P.imag) {
        PH[p + tid] = c2(exp(-0.25 * uto * tau * nn), 0.0);
      } else {
        sincos(-0.25 * uto * tau * nn, &s, &c);
        PH[p + tid] = c2(c, s);
      }
    }
    ph_u = uto;
    ph_dir = forward;
    // the lonely U_from on site L of an odd chain (:133-136) is applied by the
    // gate (L-1, L) (apply_gate lonely & 2)
    int centre = 1, gslot = 0;
    bool movingFromLeft = true;
    for (int g = 0; g < P.ngates; ++g) {
      const int i1 = P.gate_i1[g], i2 = i1 + 1;
      build_theta(i1, g);
      if (movingFromLeft) apply_gate(i1, forward, 0, (i2 == L && L % 2 == 0) ? 1 : 0);
      else apply_gate(i1, forward, 1, (L % 2 != 0 && i2 == L) ? 2 : 0);
      // next gate: right of this one -> Fromleft, centre i2, move to ni1;
      //            left of it / last -> Fromright, centre i1, move to ni2 / 1
      const bool more = g + 1 < P.ngates;
      const int ni1 = more ? P.gate_i1[g + 1] : 0, ni2 = ni1 + 1;
      const int dir = (more && ni1 >= i2) ? kFromleft : kFromright;
      decompose(dir, P.cutoff, P.maxm, true, MD + i1 * P.Q1, i1);  // writes sites i1, i2
      plan_end();
      centre = (dir == kFromleft) ? i2 : i1;
      const int target = !more ? (final_gauge ? 1 : centre) : (dir == kFromleft ? ni1 : ni2);
      position(centre, target, &gslot);
      if (more && (i2 == ni1 || i1 == ni2)) movingFromLeft = false;
    }
    // lonely U_to on site 1 (:222-223), then psi.normalize() (:228)
    if (centre != 1) {
      // the phase is diagonal in site 1's physical index (commutes with the
      // gauge); the norm of the MPS is the norm of the centre site
      site_phase(1, PH + p);
      const double n2 = site_norm2(centre);
      if (n2 > 0) site_scale(centre, 1.0 / sqrt(n2));
    } else if (site_used(1) <= NT) {
      // one pass: the phased element stays in a register for the scaling
      // (same products, same per-thread sums as the three-pass form below)
      pf(9);
      const LDS int* B = boff(1);
      const int tot = B[SEG];
      zc z = c2(0.0, 0.0);
      double acc = 0.0;
      if (tid < tot) {
        int n = 0;  // site 1: blocks (q = 0, n) in n order
#pragma unroll
        for (int t = 1; t < OCG_MAXP; ++t)
          if (t < p && B[t] <= tid) n = t;
        z = cmul(site(1)[tid], PH[p + n]);
        acc = cabs2(z);
      }
      const double n2 = block_sum(acc);
      if (tid < tot) site(1)[tid] = n2 > 0 ? cscale(z, 1.0 / sqrt(n2)) : z;
      sync();
    } else {
      site_phase(1, PH + p);
      double n2 = site_norm2(1);
      if (n2 > 0) site_scale(1, 1.0 / sqrt(n2));
    }
  }

  // ------------------------------------------------------------- overlaps
  // <X|Y> (with_dH = 0) or <X| sum_k 0.5 n_k(n_k-1) |Y> (with_dH = 1);
  // X: an MPS in global memory (slot dims gd, data gx); Y: this chain's MPS.
  // Environments are block-diagonal in q: E_q is dX[b][q] x dY[b][q].
  // E0 carries the identity string, E1 the strings with dH already applied
  // (the bond-dimension-2 MPO of propagatorDeriv, src/BH_tDMRG.cpp:10-14).
  // Per site: T_q = E_q Y_q (Y_q = right-grouped site block, cols (n, c)),
  // then En_{q'} = sum_n X_(q'-n,n)^H T_(q'-n)[:, (n, .)].
  // Scratch: G/G2/W/W2 (environments), X/Y (T0/T1), S (staged X site),
  // XOFF/YOFF (env offsets), BOFFT (X site offsets), TCO/THC/THO (T tables).
  __device__ OCG_INLINE zc overlap(const int* gd, const zc* gx, int with_dH) {
    pf(8);
    const int p = P.p, Q1 = P.Q1;
    lzp E0 = G;  lzp E1 = G2;
    lzp N0 = W;  lzp N1 = W2;
    for (int i = tid; i < P.nsq; i += NT) DIMX[i] = gd[i];
    sync();
    if (w0) {
      const int q = lane;
      const int sz = q < Q1 ? dx(0, q) * d(0, q) : 0;
      const int inc = wscan(sz);
      if (q < Q1) XOFF[q] = inc - sz;
      if (lane == 63) { XOFF[Q1] = inc; E0[0] = c2(1, 0); E1[0] = c2(0, 0); }
    }
    sync();
    for (int k = 1; k <= P.L; ++k) {
      if (w0) {
        scan_excl(BOFFT, SEG, [&](int s) {  // X site k block offsets
          int q, n;
          qn_of(s, q, n);
          return dx(k - 1, q) * dx(k, q + n);
        });
        scan_excl(TCO, SEG, [&](int s) {  // T column segments (n, c in bond k sector q+n)
          int q, n;
          qn_of(s, q, n);
          return d(k, q + n);
        });
      }
      sync();
      if (w0) {
        const int q = lane;
        int sz = 0, C = 0, nsz = 0;
        if (q < Q1) {
          C = TCO[(q + 1) * p] - TCO[q * p];
          const int rx = dx(k - 1, q), ry = d(k - 1, q);
          sz = (rx > 0 && ry > 0) ? rx * C : 0;
          nsz = dx(k, q) * d(k, q);
        }
        const int it = wscan(sz), in = wscan(nsz);
        if (q < Q1) { THC[q] = C; THO[q] = it - sz; YOFF[q] = in - nsz; }
        if (lane == 63) { THO[Q1] = it; YOFF[Q1] = in; }
      }
      // stage X site k in LDS: issue the loads before the T contraction, land them after
      const int nx = BOFFT[SEG];
      const zc* sx = gx + P.site_base[k];
      zc pre[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (tid + u * NT < nx) pre[u] = sx[tid + u * NT];
      sync();
      // T0 = E0_q Y_q -> X buffer, T1 = E1_q Y_q -> Y buffer
      const int tT = THO[Q1];
      {
                for (int base = 0; base < tT; base += NT) {
          const int e = base + tid;
          const int q = blk(THO, e);
          if (e < tT) {
            const int C = THC[q], ry = d(k - 1, q);
            int col, o;
            const int i = udiv(e - THO[q], C, col);
            const int n = seg_in(TCO, q, col, o);
            const int cy = d(k, q + n);
            lzp yb = site(k) + bo(k, q, n) + (col - o);
            lzp e0 = E0 + XOFF[q] + i * ry;
            lzp e1 = E1 + XOFF[q] + i * ry;
            zc t0 = c2(0, 0), t1 = c2(0, 0);
            for (int b = 0; b < ry; ++b) {
              const zc yv = yb[b * cy];
              cacc(t0, e0[b], yv);
              if (with_dH) cacc(t1, e1[b], yv);
            }
            X[e] = t0;
            if (with_dH) Y[e] = t1;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (tid + u * NT < nx) S[tid + u * NT] = pre[u];
      for (int i = tid + 4 * NT; i < nx; i += NT) S[i] = sx[i];
      sync();
      // En_q' = sum_n X_(q'-n, n)^H T_(q'-n)[:, (n, .)]   (E1 also gets f(n) X^H T0)
      const int ne = YOFF[Q1];
      {
        for (int base = 0; base < ne; base += NT) {
          const int e = base + tid;
          const int qq = blk(YOFF, e);
          if (e < ne) {
            const int cy = d(k, qq), cx = dx(k, qq);
            int j;
            const int a = udiv(e - YOFF[qq], cy, j);
            zc acc0 = c2(0, 0), acc1 = c2(0, 0);
            for (int n = 0; n < p && n <= qq; ++n) {
              const int q = qq - n;
              const int rx = dx(k - 1, q);
              if (rx == 0 || d(k - 1, q) == 0) continue;
              const int C = THC[q];
              lzp xb = S + BOFFT[q * p + n] + a;
              const int tc = THO[q] + TCO[q * p + n] - TCO[q * p] + j;
              zc s0 = c2(0, 0), s1 = c2(0, 0);
              for (int i = 0; i < rx; ++i) {
                const zc xv = xb[i * cx];
                cjacc(s0, xv, X[tc + i * C]);
                if (with_dH) cjacc(s1, xv, Y[tc + i * C]);
              }
              acc0 = cadd(acc0, s0);
              if (with_dH) acc1 = cadd(acc1, cadd(s1, cscale(s0, P.dH[n])));
            }
            N0[e] = acc0;
            if (with_dH) N1[e] = acc1;
          }
        }
      }
      sync();
      lzp t0 = E0; E0 = N0; N0 = t0;
      lzp t1 = E1; E1 = N1; N1 = t1;
      for (int i = tid; i <= Q1; i += NT) XOFF[i] = YOFF[i];
      sync();
    }
    zc res = c2(0, 0);
    const int oq = XOFF[P.Q];
    if (XOFF[Q1] > oq) res = with_dH ? zc(E1[oq]) : zc(E0[oq]);
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
    if (w0) {
      const int q = lane;
      const int dq = q < Q1 ? d(0, q) : 0, sz = 2 * dq * dq;
      const int inc = wscan(sz);
      if (q < Q1) { CDIM[q] = dq; COLD[q] = dq; COFF[q] = inc - sz; }
      if (lane == 63) { COFF[Q1] = inc; CR[0] = c2(1, 0); CR[1] = c2(0, 0); }  // MPO left boundary s = 0
    }
    sync();
    for (int k = 1; k <= L; ++k) {
      const bool last = (k == L);
      // M_k: rows (n, a' in new bond k-1, sector q-n), cols (t, c in old bond k, sector q)
      const int tot = theta_tables([&](int q, int n) { return (q - n >= 0) ? CDIM[q - n] : 0; },
                                   [&](int q, int n) { return n == 0 ? (last ? d(k, q) : 2 * d(k, q)) : 0; });
      {
                for (int base = 0; base < tot; base += NT) {
          const int e = base + tid;
          const int q = blk(THO, e);
          if (e < tot) {
            const int C = THC[q];
            int col, o;
            const int row = udiv(e - THO[q], C, col);
            const int n = seg_in(TRO, q, row, o);
            const int ap = row - o, ql = q - n;
            const int dc = d(k, q);
            const int t = last ? 1 : (col >= dc ? 1 : 0);
            const int c = last ? col : col - t * dc;
            const int dl = COLD[ql];                          // old rows of A_k blocks
            lzp Ab = site(k) + bo(k, ql, n) + c;              // dl x dc (old layout)
            lzp Cq = CR + COFF[ql] + ap * 2 * dl;
            zc v0 = c2(0, 0), v1 = c2(0, 0);
            for (int a = 0; a < dl; ++a) {
              const zc av = Ab[a * dc];
              cacc(v0, Cq[a], av);
              cacc(v1, Cq[dl + a], av);
            }
            TH[e] = (t == 0) ? v0 : c2(P.dH[n] * v0.x + v1.x, P.dH[n] * v0.y + v1.y);
          }
        }
      }
      sync();
      if (last) {
        if (w0 && lane < Q1) DIMS[(L - 1) * Q1 + lane] = CDIM[lane];
        sync();
        if (w0) site_offsets(L);
        sync();
                for (int base = 0; base < tot; base += NT) {
          const int e = base + tid;
          const int q = blk(THO, e);
          if (e < tot) {
            const int C = THC[q];
            int col, o;
            const int row = udiv(e - THO[q], C, col);
            const int n = seg_in(TRO, q, row, o);
            site(L)[bo(L, q - n, n) + (row - o) * C + col] = TH[e];
          }
        }
        sync();
        break;
      }
      decompose(kFromleft, OCG_GAUGE_CUTOFF, 1 << 30, false, MD + P.nsq + k * Q1);
      pf(11);
      // new layout of site k: rows = new bond k-1 (CDIM), cols = KEPT
      if (w0)
        scan_excl(BOFFT, SEG, [&](int s) {
          int q, n;
          qn_of(s, q, n);
          return (q + n <= P.Q) ? CDIM[q] * KEPT[q + n] : 0;
        });
      sync();
      // S <- X in the new layout of site k; CR <- Y (next carry)
      const int xt = XOFF[Q1], yt = YOFF[Q1];
      {
        for (int base = 0; base < xt; base += NT) {
          const int e = base + tid;
          const int q = blk(XOFF, e);
          if (e < xt) {
            const int kq = KEPT[q];
            int j, o;
            const int row = udiv(e - XOFF[q], kq, j);
            const int n = seg_in(TRO, q, row, o);
            S[BOFFT[(q - n) * p + n] + (row - o) * kq + j] = X[e];
          }
        }
      }
      for (int e = tid; e < yt; e += NT) CR[e] = Y[e];
      sync();
      const int ns = BOFFT[SEG];
      for (int e = tid; e < ns; e += NT) site(k)[e] = S[e];
      // commit: bond k-1 gets its new dims; bond k keeps the OLD dims
      // (A_{k+1} is still laid out with them) until site k+1 is rebuilt.
      for (int i = tid; i <= SEG; i += NT) boff(k)[i] = BOFFT[i];
      if (w0) {
        if (lane < Q1) {
          if (k > 1) DIMS[(k - 1) * Q1 + lane] = CDIM[lane];
          COLD[lane] = d(k, lane);
          CDIM[lane] = KEPT[lane];
          COFF[lane] = YOFF[lane];
        }
        if (lane == 0) COFF[Q1] = YOFF[Q1];
      }
      sync();
    }
    if (truncate_sweep)
      for (int k = L; k > 1; --k) gauge_left(k, P.cutoff, P.maxm);
  }
};

}  // namespace ocg
