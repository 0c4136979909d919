// Device side of the HBM-resident tDMRG engine (large bond dimensions).
//
// The LDS chain engine (engine_device.hpp) keeps a whole MPS inside one
// workgroup; that stops at about L=8, chi=80.  This engine keeps every MPS,
// two-site tensor, Gram matrix and eigenvector block in HBM and runs each
// phase of a decomposition as one batched launch over all (chain, U(1)
// sector) problems of a batch of chains (psi, xi, Hessian rows ...):
//
//   k_gemm        batched, segmented complex GEMM on v_mfma_f64_16x16x4f64
//                 (Θ = A_i1 A_i2, Gram ΘΘ^H / Θ^HΘ, factors U^HΘ / ΘW, gauge
//                 products, overlap transfer matrices)
//   k_gate        pre-phase -> hopping gate (per Δ = n1+n2 block) -> post-phase
//                 on every (a, c) vector of Θ (src/BH_tDMRG.cpp:150-159)
//   k_heev_vals   Householder tridiagonalisation of each Hermitian Gram block
//                 + Sturm bisection of every eigenvalue (descending)
//   k_truncate    per chain: global ranking over sectors, ITensor cutoff/Maxm
//                 rule, kept dimension per sector (denmatDecomp's truncate)
//   k_heev_vecs   inverse iteration for the kept eigenvalues, classical
//                 Gram-Schmidt (twice), back-transformation to the Gram basis
//   k_copy        scaled / conjugate-transposed block copies, phases, norms
//
// Shapes are known to the host (it reads back the kept dimensions after each
// truncation), which builds the per-launch task lists; kernels only walk them.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef HBM_INLINE
#define HBM_INLINE __attribute__((always_inline))
#endif

namespace hbm {

struct __attribute__((aligned(16))) z {
  double x, y;
};
__host__ __device__ __forceinline__ z mk(double x, double y) { z r; r.x = x; r.y = y; return r; }
__device__ __forceinline__ z zadd(z a, z b) { return mk(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ z zsub(z a, z b) { return mk(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ z zmul(z a, z b) { return mk(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
__device__ __forceinline__ z zcj(z a) { return mk(a.x, -a.y); }
__device__ __forceinline__ z zsc(z a, double s) { return mk(a.x * s, a.y * s); }
// conj(a) * b
__device__ __forceinline__ z zcjmul(z a, z b) { return mk(a.x * b.x + a.y * b.y, a.x * b.y - a.y * b.x); }

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int NT = 256;  // threads per workgroup of every kernel here (4 wave64s)

// ------------------------------------------------------------------ tasks
// GEMM segment: alpha * op(A)[m x k] * op(B)[k x n]; op 0 = N, 1 = C (conj^T)
struct GSeg {
  const z* A;
  const z* B;
  int lda, ldb, k, ops;  // ops: bit 0 opA, bit 1 opB
  double alpha;
};
// C[m x n] (ld ldc) = rs[i] * cs[j] * sc * sum over segments; no segment: C = 0.
// Scale pointers are optional; smode bits select sqrt/inverse forms of the
// eigenvalue-derived scales (see scale_of).
struct GTask {
  z* C;
  int ldc, m, n;
  int seg0, nseg;
  const double* rs;
  const double* cs;
  const double* sc;
  int smode;  // bits 0-1 rs mode, 2-3 cs mode, 4-5 sc mode: 0 plain, 1 sqrt(max(x,0)), 2 1/sqrt (0 if x <= 0)
  int tile0;  // prefix of 32x32 tiles over tasks
};
// element copies: dst[i][j] = f * rs[i] * cs[j] * sc * (conj^T? conj(src[j][i]) : src[i][j])
// mode bit 0: conj-transpose, bit 1: zero fill (src unused), bit 2: sum of
// squares (k_sumsq's task lists only), bit 3: fill with f.
struct CTask {
  const z* src;
  z* dst;
  int rows, cols, lds, ldd;
  int mode, smode;
  z f;
  const double* rs;
  const double* cs;
  const double* sc;
  long long e0;  // prefix of elements over tasks
};

__device__ __forceinline__ double scale_of(const double* p, int i, int mode) {
  if (!p) return 1.0;
  const double x = p[i];
  if (mode == 1) return x > 0 ? sqrt(x) : 0.0;
  if (mode == 2) return x > 0 ? 1.0 / sqrt(x) : 0.0;
  return x;
}

// last task t with prefix[t] <= e (prefix strictly increasing over non-empty tasks)
template <class T, class F>
__device__ __forceinline__ int find_task(const T* tasks, int ntask, long long e, F prefix) {
  int lo = 0, hi = ntask - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (prefix(tasks[mid]) <= e) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// ------------------------------------------------------------------ GEMM
// One workgroup = one 32x32 tile of one task; wave w owns the 16x16 sub-tile
// (w >> 1, w & 1).  K is staged through LDS in chunks of 16 (re and im planes
// separately, padded; the next chunk's global loads are in flight while the
// current one feeds the MFMAs), each chunk feeds up to 4 k-steps of 4 complex
// MFMA groups (k-steps past the segment's k are skipped):
//   re += a.re b.re - a.im b.im,  im += a.re b.im + a.im b.re
// (v_mfma_f64_16x16x4f64 operands: lane l holds A[l & 15][k = l >> 4] and
// B[k = l >> 4][l & 15]; results col = l & 15, row = (l >> 4) + 4 r).
// (GK 32 and 64 measured slower on the config-4 mix: fewer workgroups per CU.)
constexpr int GT = 32, GK = 16;
// xcd != 0: workgroups b and b + 8 (which the dispatcher places on one XCD,
// MI355X_MICROARCH.md §Workgroup dispatch) take consecutive tiles, so a task's
// tiles share that XCD's L2 for their common operand rows / columns (speed
// only: any bijection of workgroups onto tiles computes the same result)
__global__ __launch_bounds__(NT) void k_gemm(const GTask* __restrict__ tasks, const int2* __restrict__ tile_task,
                                             const GSeg* __restrict__ segs, int xcd) {
  constexpr int EA = GT * GK / NT;  // staged elements per thread and operand
  __shared__ double Ar[GT][GK + 1], Ai[GT][GK + 1], Br[GK][GT + 1], Bi[GK][GT + 1];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int tile = blockIdx.x;
  if (xcd) {
    const int nb = gridDim.x, base = nb >> 3, rem = nb & 7, x = blockIdx.x & 7;
    tile = x * base + (x < rem ? x : rem) + (blockIdx.x >> 3);
  }
  // tile -> (task, its first segment) from the host's table: one dependent load
  // instead of a binary search over freshly uploaded task records, then the
  // task and first-segment records in parallel (the small launches' latency)
  const int2 tt = tile_task[tile];
  const GTask T = tasks[tt.x];
  GSeg S0{};
  if (tt.y >= 0) S0 = segs[tt.y];
  const int tl = tile - T.tile0;
  const int ntn = (T.n + GT - 1) / GT;
  const int m0 = (tl / ntn) * GT, n0 = (tl % ntn) * GT;
  const int wm = (wv >> 1) * 16, wn = (wv & 1) * 16;
  // a wave whose 16x16 sub-tile lies wholly outside the task (m or n not a
  // multiple of 32: 25 % of the config-4 MFMA work) still stages operands but
  // issues no MFMA; its outputs are never stored, so nothing else changes
  const bool live = m0 + wm < T.m && n0 + wn < T.n;
  d4 cr = {0, 0, 0, 0}, ci = {0, 0, 0, 0};
  for (int s = 0; s < T.nseg; ++s) {
    const GSeg S = s == 0 ? S0 : segs[T.seg0 + s];
    const bool ca = S.ops & 1, cb = (S.ops >> 1) & 1;
    // global -> registers for the chunk at k0 (issued one chunk ahead of its MFMAs)
    z va[EA], vb[EA];
    auto gload = [&](int k0) {
#pragma unroll
      for (int t = 0; t < EA; ++t) {
        const int e = tid + NT * t;
        int r, kk;
        if (!ca) { r = e / GK; kk = e % GK; }
        else { kk = e / GT; r = e % GT; }
        z v = mk(0, 0);
        const int gr = m0 + r, gk = k0 + kk;
        if (gr < T.m && gk < S.k) {
          v = ca ? S.A[(size_t)gk * S.lda + gr] : S.A[(size_t)gr * S.lda + gk];
          if (ca) v.y = -v.y;
          v = zsc(v, S.alpha);
        }
        va[t] = v;
      }
#pragma unroll
      for (int t = 0; t < EA; ++t) {
        const int e = tid + NT * t;
        int kk, c;
        if (!cb) { kk = e / GT; c = e % GT; }
        else { c = e / GK; kk = e % GK; }
        z v = mk(0, 0);
        const int gc = n0 + c, gk = k0 + kk;
        if (gc < T.n && gk < S.k) {
          v = cb ? S.B[(size_t)gc * S.ldb + gk] : S.B[(size_t)gk * S.ldb + gc];
          if (cb) v.y = -v.y;
        }
        vb[t] = v;
      }
    };
    if (S.k > 0) gload(0);
    for (int k0 = 0; k0 < S.k; k0 += GK) {
      // stage op(A)[m0.., k0..] (32 x GK) and op(B)[k0.., n0..] (GK x 32)
#pragma unroll
      for (int t = 0; t < EA; ++t) {
        const int e = tid + NT * t;
        const int r = !ca ? e / GK : e % GT, kk = !ca ? e % GK : e / GT;
        Ar[r][kk] = va[t].x;
        Ai[r][kk] = va[t].y;
        const int kb = !cb ? e / GT : e % GK, c = !cb ? e % GT : e / GK;
        Br[kb][c] = vb[t].x;
        Bi[kb][c] = vb[t].y;
      }
      __syncthreads();
      if (k0 + GK < S.k) gload(k0 + GK);
#pragma unroll
      for (int ks = 0; ks < GK; ks += 4) {
        if (live && k0 + ks < S.k) {  // k-steps past the end would only add zeros
          const int ar = wm + (lane & 15), kk = ks + (lane >> 4), bc = wn + (lane & 15);
          const double are = Ar[ar][kk], aim = Ai[ar][kk];
          const double bre = Br[kk][bc], bim = Bi[kk][bc];
          cr = __builtin_amdgcn_mfma_f64_16x16x4f64(are, bre, cr, 0, 0, 0);
          cr = __builtin_amdgcn_mfma_f64_16x16x4f64(-aim, bim, cr, 0, 0, 0);
          ci = __builtin_amdgcn_mfma_f64_16x16x4f64(are, bim, ci, 0, 0, 0);
          ci = __builtin_amdgcn_mfma_f64_16x16x4f64(aim, bre, ci, 0, 0, 0);
        }
      }
      __syncthreads();
    }
  }
  const double sc = scale_of(T.sc, 0, (T.smode >> 4) & 3);
  const int col = n0 + wn + (lane & 15);
  if (col >= T.n) return;
  const double csv = scale_of(T.cs, col, (T.smode >> 2) & 3) * sc;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = m0 + wm + (lane >> 4) + 4 * r;
    if (row < T.m) {
      const double f = scale_of(T.rs, row, T.smode & 3) * csv;
      T.C[(size_t)row * T.ldc + col] = mk(cr[r] * f, ci[r] * f);
    }
  }
}

// ------------------------------------------------------------------ copies
__global__ __launch_bounds__(NT) void k_copy(const CTask* __restrict__ tasks, int ntask, long long total) {
  for (long long e = (long long)blockIdx.x * NT + threadIdx.x; e < total; e += (long long)gridDim.x * NT) {
    const int ti = find_task(tasks, ntask, e, [](const CTask& t) { return t.e0; });
    const CTask& T = tasks[ti];
    const long long x = e - T.e0;
    const int i = int(x / T.cols), j = int(x - (long long)i * T.cols);
    z v = (T.mode & 8) ? T.f : mk(0, 0);
    if (!(T.mode & 10)) {
      v = (T.mode & 1) ? zcj(T.src[(size_t)j * T.lds + i]) : T.src[(size_t)i * T.lds + j];
      const double s = scale_of(T.rs, i, T.smode & 3) * scale_of(T.cs, j, (T.smode >> 2) & 3) *
                       scale_of(T.sc, 0, (T.smode >> 4) & 3);
      v = zsc(zmul(v, T.f), s);
    }
    T.dst[(size_t)i * T.ldd + j] = v;
  }
}

// ------------------------------------------------------------------ gate
// Per chain: Θ base, its sector tables (thoff, C, ro[q*p+n], co[q*p+n]; -1 =
// absent) and the step parameters.
struct GateChain {
  z* th;
  const int* tab;  // [0, Q1) thoff, [Q1, 2Q1) C, [2Q1, 2Q1 + Q1 p) ro, then co
  double uf, ut, tau;
  int fwd, mode, lonely;
};
struct GateTask {
  int chain, ql, qr, nl, nr;
  long long e0;
};
struct GateConst {
  int p, Q1, glo[24], gsz[24], goff[24];
  int imag;  // imaginary-time steps (ground-state preparation)
};
// exp(-i 0.25 u tau n (n-1)) (BH_tDMRG::initUGates, src/BH_tDMRG.cpp:83-87);
// imaginary time: exp(-0.25 u tau n (n-1))
__device__ __forceinline__ z uphase(double u, double tau, int n, int imag) {
  if (imag) return mk(exp(-0.25 * u * tau * double(n * (n - 1))), 0.0);
  double s, c;
  sincos(-0.25 * u * tau * double(n * (n - 1)), &s, &c);
  return mk(c, s);
}
__global__ __launch_bounds__(NT) void k_gate(const GateTask* __restrict__ tasks, int ntask, long long total,
                                             const GateChain* __restrict__ chains, GateConst gc, const z* gf,
                                             const z* gb) {
  for (long long e = (long long)blockIdx.x * NT + threadIdx.x; e < total; e += (long long)gridDim.x * NT) {
    const int ti = find_task(tasks, ntask, e, [](const GateTask& t) { return t.e0; });
    const GateTask T = tasks[ti];
    const GateChain C = chains[T.chain];
    const long long x = e - T.e0;
    const int a = int(x / T.nr), c = int(x - (long long)a * T.nr);
    const int p = gc.p, Q1 = gc.Q1;
    const int D = T.qr - T.ql;
    const int lo = gc.glo[D], sz = gc.gsz[D];
    const int* thoff = C.tab;
    const int* tC = C.tab + Q1;
    const int* ro = C.tab + 2 * Q1;
    const int* co = C.tab + 2 * Q1 + Q1 * p;
    z v[12], w[12];
    size_t addr[12];
    for (int y = 0; y < sz; ++y) {
      const int n1 = lo + y, n2 = D - n1, q = T.ql + n1;
      const int r0 = (q < Q1) ? ro[q * p + n1] : -1, c0 = (q < Q1) ? co[q * p + n2] : -1;
      if (r0 < 0 || c0 < 0) { addr[y] = ~size_t(0); v[y] = mk(0, 0); continue; }
      addr[y] = (size_t)thoff[q] + (size_t)(r0 + a) * tC[q] + c0 + c;
      z t = C.th[addr[y]];
      if (C.mode == 0) t = zmul(t, zmul(uphase(C.uf, C.tau, n1, gc.imag), uphase(C.uf, C.tau, n2, gc.imag)));
      v[y] = t;
    }
    const z* G = (C.fwd ? gf : gb) + gc.goff[D];
    for (int y = 0; y < sz; ++y) {
      z s = mk(0, 0);
      for (int xx = 0; xx < sz; ++xx) s = zadd(s, zmul(G[y * sz + xx], v[xx]));
      const int n1 = lo + y, n2 = D - n1;
      if (C.mode == 1) s = zmul(s, zmul(uphase(C.ut, C.tau, n1, gc.imag), uphase(C.ut, C.tau, n2, gc.imag)));
      else if (C.lonely) s = zmul(s, uphase(C.ut, C.tau, n2, gc.imag));
      w[y] = s;
    }
    for (int y = 0; y < sz; ++y)
      if (addr[y] != ~size_t(0)) C.th[addr[y]] = w[y];
  }
}

// ------------------------------------------------------------------ eigen
// One Hermitian Gram block per problem.  A (n x n, ld n) is overwritten by
// the Householder vectors (column j, rows j+1..n-1).  Work arrays: d (n),
// e (n), tau (n), ph (n complex: the phases delta that make the tridiagonal
// real), w (n eigenvalues, descending), Z / Dv (n x n doubles each, inverse
// iteration), U (n x k complex, ld k: the kept eigenvectors, descending).
struct EProb {
  z* A;
  double *d, *e, *tau, *w, *Z, *Dv;
  z* ph;
  z* U;
  int n, q;
  const int* kept;  // kept count of this sector (written by k_truncate)
  // eigenvalues below thr_rel * trace may be left unresolved (k_heev_vals_reg):
  // they are provably inside the discarded tail of the truncation (hbm_eig.hpp)
  double thr_rel;
  // 1: the register kernel leaves the eigenvalues to k_heev_bisect, after
  // k_heev_thresh has raised thr_rel to the decomposition's Maxm boundary
  int defer;
  // shifts per thread and multisection round (bisect_all / multisect): 1 (plain
  // bisection, the default) or 4 (OCG_HBM_BISECT_KS=4)
  int ks;
};

template <class T>
__device__ __forceinline__ T block_sum(T v, T* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int tid = threadIdx.x;
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  T s = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += red[i];
  return s;
}

// sum |x|^2 over the tasks [t0[b], t0[b+1]) of view b, one workgroup per view:
// every thread sums a fixed set of elements, then a fixed-order tree, so the
// result does not depend on scheduling or on the other views of the launch
// (an atomicAdd per element made the norms, and with them every normalised
// state, vary in the last bits from run to run)
__global__ __launch_bounds__(NT) void k_sumsq(const CTask* __restrict__ tasks, const int* __restrict__ t0,
                                              double* __restrict__ out) {
  __shared__ double red[NT / 64];
  const int b = blockIdx.x;
  double s = 0;
  for (int t = t0[b]; t < t0[b + 1]; ++t) {
    const CTask& T = tasks[t];
    const long long n = (long long)T.rows * T.cols;
    for (long long x = threadIdx.x; x < n; x += NT) {
      const int i = int(x / T.cols), j = int(x - (long long)i * T.cols);
      const z v = T.src[(size_t)i * T.lds + j];
      s += v.x * v.x + v.y * v.y;
    }
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[b] = s;
}

constexpr int kLdsOrder = 88;  // Gram blocks up to this order are reduced inside LDS

// Householder reduction (Hermitian reflectors H = I - tau u u^H, tau real):
// Q^H A Q = T_c with subdiagonal beta_j, Q = H_0 ... H_{n-2}.
__device__ HBM_INLINE void tridiag(z* A, int n, double* tau, z* beta, z* LU, z* LP, double* red, double* scal) {
  const int tid = threadIdx.x;
  for (int j = 0; j + 1 < n; ++j) {
    const int m = n - j - 1;
    z* x = A + (size_t)(j + 1) * n + j;
    double s = 0;
    for (int i = 1 + tid; i < m; i += NT) {
      const z v = x[(size_t)i * n];
      s += v.x * v.x + v.y * v.y;
    }
    s = block_sum(s, red);
    if (tid == 0) {
      const z a = x[0];
      const double aa = sqrt(a.x * a.x + a.y * a.y), xn = sqrt(aa * aa + s);
      double t = 0;
      z b = mk(0, 0), u0 = a;
      if (xn > 0) {
        const z ph = aa > 0 ? mk(a.x / aa, a.y / aa) : mk(1, 0);
        b = mk(-ph.x * xn, -ph.y * xn);
        u0 = mk(a.x + ph.x * xn, a.y + ph.y * xn);
        const double ua = aa + xn;
        t = 2.0 / (ua * ua + s);
      }
      tau[j] = t;
      beta[j] = b;
      scal[0] = t;
      scal[1] = u0.x;
      scal[2] = u0.y;
    }
    __syncthreads();
    const double t = scal[0];
    if (t == 0.0) continue;  // column already reduced: H = I
    const z u0 = mk(scal[1], scal[2]);
    for (int i = tid; i < m; i += NT) LU[i] = (i == 0) ? u0 : x[(size_t)i * n];
    __syncthreads();
    if (tid == 0) x[0] = u0;  // Householder vector lives in column j
    // p = t A_t u with A_t = A[j+1.., j+1..] Hermitian: p_i = sum_k conj(A_t[k][i]) u_k
    const z* At = A + (size_t)(j + 1) * n + (j + 1);
    for (int i = tid; i < m; i += NT) {
      z acc = mk(0, 0);
      const z* col = At + i;
      for (int k = 0; k < m; ++k) {
        const z av = col[(size_t)k * n], uk = LU[k];
        acc.x += av.x * uk.x + av.y * uk.y;
        acc.y += av.x * uk.y - av.y * uk.x;
      }
      LP[i] = zsc(acc, t);
    }
    __syncthreads();
    double kk = 0;
    for (int i = tid; i < m; i += NT) {
      const z ui = LU[i], pi = LP[i];
      kk += ui.x * pi.x + ui.y * pi.y;  // Re(conj(u_i) p_i)
    }
    kk = 0.5 * t * block_sum(kk, red);
    for (int i = tid; i < m; i += NT) LP[i] = zsub(LP[i], zsc(LU[i], kk));  // w = p - K u
    __syncthreads();
    z* Aw = A + (size_t)(j + 1) * n + (j + 1);
    for (int e = tid; e < m * m; e += NT) {
      const int i = e / m, k = e - i * m;
      const z ui = LU[i], wi = LP[i], uk = LU[k], wk = LP[k];
      z v = Aw[(size_t)i * n + k];
      // v -= u_i conj(w_k) + w_i conj(u_k)
      v.x -= ui.x * wk.x + ui.y * wk.y + wi.x * uk.x + wi.y * uk.y;
      v.y -= ui.y * wk.x - ui.x * wk.y + wi.y * uk.x - wi.x * uk.y;
      Aw[(size_t)i * n + k] = v;
    }
    __syncthreads();
  }
}

// # eigenvalues of the real symmetric tridiagonal (d, e2 = e^2) below s
__device__ __forceinline__ int sturm(const double* d, const double* e2, int n, double s, double pivmin) {
  double q = d[0] - s;
  if (fabs(q) < pivmin) q = -pivmin;
  int c = q < 0 ? 1 : 0;
  for (int i = 1; i < n; ++i) {
    q = d[i] - s - e2[i - 1] / q;
    if (fabs(q) < pivmin) q = -pivmin;
    c += q < 0 ? 1 : 0;
  }
  return c;
}

// From the reduced tridiagonal (diagonal in Ld, complex subdiagonal beta in LB):
// the phases making it real (P.ph), d / e (P.d, P.e), and every eigenvalue by
// bisection (thread t -> the t-th largest), for an NTH-thread workgroup.
template <int NTH>
__device__ __forceinline__ void vals_from_tridiag(const EProb& P, int n, double* Ld, double* Le2, const z* LB) {
  const int tid = threadIdx.x;
  __syncthreads();
  if (tid == 0) {
    z dl = mk(1, 0);
    P.ph[0] = dl;
    for (int j = 0; j + 1 < n; ++j) {
      const z b = LB[j];
      const double ab = sqrt(b.x * b.x + b.y * b.y);
      if (ab > 0) dl = zmul(dl, mk(b.x / ab, b.y / ab));
      P.ph[j + 1] = dl;
      P.e[j] = ab;
      Le2[j] = ab * ab;
    }
    P.e[n - 1] = 0;
    Le2[n - 1] = 0;
  }
  for (int j = tid; j < n; j += NTH) P.d[j] = Ld[j];
  __syncthreads();
  // Gershgorin bounds, pivmin (LAPACK dstebz conventions)
  double gl = 1e300, gu = -1e300, emax = 0;
  for (int i = tid; i < n; i += NTH) {
    const double el = i > 0 ? sqrt(Le2[i - 1]) : 0.0, er = i + 1 < n ? sqrt(Le2[i]) : 0.0;
    gl = fmin(gl, Ld[i] - el - er);
    gu = fmax(gu, Ld[i] + el + er);
    emax = fmax(emax, Le2[i]);
  }
  for (int o = 32; o > 0; o >>= 1) {
    gl = fmin(gl, __shfl_xor(gl, o, 64));
    gu = fmax(gu, __shfl_xor(gu, o, 64));
    emax = fmax(emax, __shfl_xor(emax, o, 64));
  }
  __shared__ double bb[3][NTH / 64];
  if ((tid & 63) == 0) { bb[0][tid >> 6] = gl; bb[1][tid >> 6] = gu; bb[2][tid >> 6] = emax; }
  __syncthreads();
  gl = bb[0][0]; gu = bb[1][0]; emax = bb[2][0];
  for (int i = 1; i < NTH / 64; ++i) { gl = fmin(gl, bb[0][i]); gu = fmax(gu, bb[1][i]); emax = fmax(emax, bb[2][i]); }
  const double eps = 2.220446049250313e-16, safmin = 2.2250738585072014e-308;
  const double tnorm = fmax(fabs(gl), fabs(gu));
  const double pivmin = safmin * fmax(1.0, emax);
  gl -= 2.0 * eps * tnorm * n + 2.0 * pivmin;
  gu += 2.0 * eps * tnorm * n + 2.0 * pivmin;
  const double atol = 4.0 * eps * tnorm;
  for (int t = tid; t < n; t += NTH) {
    const int idx = n - 1 - t;  // ascending index of the t-th largest
    double lo = gl, hi = gu;
    for (int it = 0; it < 128 && hi - lo > atol + 2.0 * eps * fmax(fabs(lo), fabs(hi)); ++it) {
      const double mid = 0.5 * (lo + hi);
      if (sturm(Ld, Le2, n, mid, pivmin) > idx) hi = mid;
      else lo = mid;
    }
    P.w[t] = 0.5 * (lo + hi);
  }
}

// eigenvalues: tridiagonalise (in LDS for small orders), make the tridiagonal
// real, bisect every eigenvalue (thread t -> the t-th largest)
__device__ __forceinline__ void heev_vals_lds_body(const EProb& P, char* smem) {
  const int n = P.n, tid = threadIdx.x;
  if (n <= 0) return;
  __shared__ double red[NT / 64], scal[4];
  if (n == 1) {
    if (tid == 0) {
      P.w[0] = P.A[0].x;
      P.ph[0] = mk(1, 0);
      P.d[0] = P.A[0].x;
      P.e[0] = 0;
      P.tau[0] = 0;
    }
    return;
  }
  // LDS: [u (n) | p/w (n) | beta (n) as z][d (n) | e2 (n) doubles][A copy (n^2 z) if small]
  z* LU = (z*)smem;
  z* LP = LU + n;
  z* LB = LP + n;
  double* Ld = (double*)(LB + n);
  double* Le2 = Ld + n;
  const bool inl = n <= kLdsOrder;
  z* A = inl ? (z*)(Le2 + n) : P.A;  // 64 n bytes in: 16-byte aligned
  if (inl) {
    for (int e = tid; e < n * n; e += NT) A[e] = P.A[e];
    __syncthreads();
  }
  tridiag(A, n, P.tau, LB, LU, LP, red, scal);
  for (int j = tid; j < n; j += NT) Ld[j] = A[(size_t)j * n + j].x;
  if (inl) {
    __syncthreads();
    for (int e = tid; e < n * n; e += NT) P.A[e] = A[e];
  }
  vals_from_tridiag<NT>(P, n, Ld, Le2, LB);
}

__device__ __forceinline__ double hrand(unsigned i, unsigned j) {
  unsigned h = i * 0x9E3779B1u ^ (j + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
  return (double(h) + 0.5) * (2.0 / 4294967296.0) - 1.0;
}

// kept eigenvectors: inverse iteration on the real tridiagonal (one thread
// per eigenvalue, LDL^T without pivoting, tiny pivots replaced), classical
// Gram-Schmidt twice in descending order, then U = Q D Z
__global__ __launch_bounds__(NT) void k_heev_vecs(const EProb* __restrict__ probs, int nprob) {
  extern __shared__ __align__(16) char smem[];
  const EProb P = probs[blockIdx.x];
  const int n = P.n, tid = threadIdx.x;
  if (n <= 0) return;
  const int k = *P.kept;
  if (k <= 0) return;
  if (n == 1) {
    if (tid == 0) P.U[0] = mk(1, 0);
    return;
  }
  double* Ld = (double*)smem;
  double* Le = Ld + n;
  double* Lc = Le + n;  // Gram-Schmidt coefficients
  __shared__ double red[NT / 64];
  for (int i = tid; i < n; i += NT) { Ld[i] = P.d[i]; Le[i] = P.e[i]; }
  __syncthreads();
  double tn = 0;
  for (int i = tid; i < n; i += NT) tn = fmax(tn, fabs(Ld[i]) + Le[i] + (i > 0 ? Le[i - 1] : 0.0));
  for (int o = 32; o > 0; o >>= 1) tn = fmax(tn, __shfl_xor(tn, o, 64));
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = tn;
  __syncthreads();
  tn = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  const double tiny = 2.220446049250313e-16 * fmax(tn, 1e-300);
  double* Z = P.Z;   // [i][j], ld n
  double* Dv = P.Dv;
  for (int j = tid; j < k; j += NT) {
    const double lam = P.w[j];
    // pivots of T - lam I = L D L^T
    double q = Ld[0] - lam;
    if (fabs(q) < tiny) q = q < 0 ? -tiny : tiny;
    Dv[j] = q;
    for (int i = 1; i < n; ++i) {
      q = Ld[i] - lam - Le[i - 1] * Le[i - 1] / q;
      if (fabs(q) < tiny) q = q < 0 ? -tiny : tiny;
      Dv[(size_t)i * n + j] = q;
    }
    for (int i = 0; i < n; ++i) Z[(size_t)i * n + j] = hrand(i, j);
    for (int it = 0; it < 3; ++it) {
      // forward: y_{i+1} = b_{i+1} - l_i y_i, l_i = e_i / q_i
      double y = Z[j], qp = Dv[j];
      for (int i = 1; i < n; ++i) {
        const size_t o = (size_t)i * n + j;
        y = Z[o] - Le[i - 1] / qp * y;
        Z[o] = y;
        qp = Dv[o];
      }
      // backward: x_i = (y_i - e_i x_{i+1}) / q_i
      double xn = Z[(size_t)(n - 1) * n + j] / Dv[(size_t)(n - 1) * n + j];
      Z[(size_t)(n - 1) * n + j] = xn;
      double ss = xn * xn;
      for (int i = n - 2; i >= 0; --i) {
        const size_t o = (size_t)i * n + j;
        xn = (Z[o] - Le[i] * xn) / Dv[o];
        Z[o] = xn;
        ss += xn * xn;
      }
      const double inv = ss > 0 ? 1.0 / sqrt(ss) : 0.0;
      for (int i = 0; i < n; ++i) Z[(size_t)i * n + j] *= inv;
    }
  }
  __syncthreads();
  // classical Gram-Schmidt, twice, in descending eigenvalue order
  for (int j = 1; j < k; ++j) {
    for (int pass = 0; pass < 2; ++pass) {
      for (int i = tid; i < j; i += NT) {
        double c = 0;
        for (int r = 0; r < n; ++r) c += Z[(size_t)r * n + i] * Z[(size_t)r * n + j];
        Lc[i] = c;
      }
      __syncthreads();
      for (int r = tid; r < n; r += NT) {
        double s = 0;
        const double* zr = Z + (size_t)r * n;
        for (int i = 0; i < j; ++i) s += Lc[i] * zr[i];
        Z[(size_t)r * n + j] -= s;
      }
      __syncthreads();
    }
    double ss = 0;
    for (int r = tid; r < n; r += NT) { const double v = Z[(size_t)r * n + j]; ss += v * v; }
    ss = block_sum(ss, red);
    const double inv = ss > 0 ? 1.0 / sqrt(ss) : 0.0;
    for (int r = tid; r < n; r += NT) Z[(size_t)r * n + j] *= inv;
    __syncthreads();
  }
  // U = Q D Z: rows scaled by delta_r, then reflectors j = n-2 .. 0
  z* U = P.U;
  for (int e = tid; e < n * k; e += NT) {
    const int r = e / k, c = e - r * k;
    U[e] = zsc(P.ph[r], Z[(size_t)r * n + c]);
  }
  __syncthreads();
  for (int j = n - 2; j >= 0; --j) {
    const double t = P.tau[j];
    if (t == 0.0) continue;
    const z* u = P.A + j;  // u[r] = A[r][j], r = j+1 .. n-1
    for (int c = tid; c < k; c += NT) {
      z s = mk(0, 0);
      for (int r = j + 1; r < n; ++r) s = zadd(s, zcjmul(u[(size_t)r * n], U[(size_t)r * k + c]));
      s = zsc(s, t);
      for (int r = j + 1; r < n; ++r) U[(size_t)r * k + c] = zsub(U[(size_t)r * k + c], zmul(u[(size_t)r * n], s));
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ truncation
// One item = one decomposition of one chain: its problems [p0, p0 + np) in
// sector order.  ITensor truncate as the LDS engine applies it (DESIGN.md
// §3): in the spectrum sorted descending (ties: sector, then index),
// position j >= 1 is discarded iff j >= maxm, the weight from j to the end
// is below cutoff * total, or PP[j] <= 1e-30 total; kept per sector is then
// capped by the sector's Schmidt-rank bound.  Outputs kept[q] (per problem:
// *EProb.kept), the kept weight and inv = 1/sqrt(kept weight) (1 when not
// normalising or the weight is below 1e-32).
struct TItem {
  int p0, np;
  double cutoff;
  int maxm, normalize;
  int* kept;        // per problem of the item (the EProb.kept targets)
  const int* bound; // per problem: Schmidt-rank bound of its sector
  double* keptw;    // [0] kept weight, [1] inv
};
constexpr int kMaxEig = 5120;  // eigenvalues of one decomposition (>= p chi for chi <= 512, p <= 9)
constexpr int TNT = 1024;      // threads of k_truncate: the O(T^2) ranking spread over 16 waves
template <class T>
__device__ __forceinline__ T block_sum_t(T v, T* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int tid = threadIdx.x;
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  T s = 0;
#pragma unroll
  for (int i = 0; i < TNT / 64; ++i) s += red[i];
  return s;
}
// Every step below is the round-5 kernel's arithmetic in the same order (so the
// kept counts and weights are bit-identical); what changed is where latency
// went: the problems' sizes and eigenvalue pointers are read by one thread per
// problem at once (not one problem after another), the eigenvalues are gathered
// by flat index, the global rank comes from binary searches in the other
// sectors' descending lists (not an all-pairs count), the suffix rule reads its
// sorted values eight at a time, and the kept counts stay in LDS.
constexpr int kTruncMaxNp = 128;  // problems per item on the fast path (more: the all-pairs rank)
__global__ __launch_bounds__(TNT) void k_truncate(const TItem* __restrict__ items, const EProb* __restrict__ probs) {
  extern __shared__ __align__(16) char smem[];
  const TItem I = items[blockIdx.x];
  const int tid = threadIdx.x;
  double* LAM = (double*)smem;       // flat eigenvalues (sector order, descending inside)
  double* PP = LAM + kMaxEig;        // sorted descending
  int* RK = (int*)(PP + kMaxEig);    // global rank of each flat eigenvalue
  int* PO = RK + kMaxEig;            // problem offsets (np + 1)
  __shared__ double red[TNT / 64];
  __shared__ int sm[2];
  __shared__ const double* WP[kTruncMaxNp];
  __shared__ int KQ[kTruncMaxNp];
  __shared__ int unsorted;
  const int np = I.np;
  const bool fastp = np <= kTruncMaxNp;
  if (fastp) {
    for (int i = tid; i < np; i += TNT) {
      const EProb& P = probs[I.p0 + i];
      PO[i] = P.n;
      WP[i] = P.w;
    }
    if (tid == 0) unsorted = 0;
    __syncthreads();
    if (tid == 0) {
      int o = 0;
      for (int i = 0; i < np; ++i) {
        const int n = PO[i];
        PO[i] = o;
        o += n;
      }
      PO[np] = o;
    }
  } else if (tid == 0) {
    int o = 0;
    for (int i = 0; i < np; ++i) { PO[i] = o; o += probs[I.p0 + i].n; }
    PO[np] = o;
  }
  __syncthreads();
  const int T = PO[np];
  // the problem of flat index e: the last i with PO[i] <= e
  auto prob_of = [&](int e) {
    int lo = 0, hi = np - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (PO[mid] <= e) lo = mid;
      else hi = mid - 1;
    }
    return lo;
  };
  if (fastp) {
    for (int e = tid; e < T; e += TNT) {
      const int i = prob_of(e);
      LAM[e] = fmax(WP[i][e - PO[i]], 0.0);
    }
  } else {
    for (int i = 0; i < np; ++i) {
      const EProb& P = probs[I.p0 + i];
      for (int j = tid; j < P.n; j += TNT) LAM[PO[i] + j] = fmax(P.w[j], 0.0);
    }
  }
  __syncthreads();
  // global rank: (lambda desc, flat index asc); problems are in sector order
  if (fastp) {
    // every sector's list descending? (the multisection's midpoints of a
    // degenerate cluster could come out a rounding step out of order)
    for (int e = tid; e + 1 < T; e += TNT)
      if (LAM[e] < LAM[e + 1] && prob_of(e) == prob_of(e + 1)) unsorted = 1;
    __syncthreads();
  }
  if (fastp && !unsorted) {
    // rank = the index inside its own (descending) sector + per other sector
    // the length of its prefix ahead of it: > l after it, >= l before it
    for (int e = tid; e < T; e += TNT) {
      const double l = LAM[e];
      const int i = prob_of(e);
      int rk = e - PO[i];
      for (int i2 = 0; i2 < np; ++i2) {
        if (i2 == i) continue;
        const int b = PO[i2];
        int lo = 0, hi = PO[i2 + 1] - b;
        const bool ge = i2 < i;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          const double v = LAM[b + mid];
          if (ge ? v >= l : v > l) lo = mid + 1;
          else hi = mid;
        }
        rk += lo;
      }
      RK[e] = rk;
      PP[rk] = l;
    }
  } else {
    for (int e = tid; e < T; e += TNT) {
      const double l = LAM[e];
      int rk = 0;
      for (int f = 0; f < T; ++f) {
        const double lf = LAM[f];
        rk += (lf > l || (lf == l && f < e)) ? 1 : 0;
      }
      RK[e] = rk;
      PP[rk] = l;
    }
  }
  double tot = 0;
  for (int e = tid; e < T; e += TNT) tot += LAM[e];
  tot = block_sum_t(tot, red);
  __syncthreads();
  if (tid == 0) {
    int m = T;
    if (tot > 0) {
      const double cut = I.cutoff * tot, flo = 1e-30 * tot;
      double S = 0;
      // smallest m >= 1 such that every position j >= m is discarded (the
      // discarded set is a suffix: both tests are monotone in j); the values
      // are read eight ahead, the sum keeps its order
      int j = T - 1;
      bool stop = false;
      while (j >= 1 && !stop) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = PP[j - u >= 1 ? j - u : 1];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (!stop && j >= 1) {
            const double sj = S + v[u];
            if (j >= I.maxm || sj < cut || v[u] <= flo) {
              S = sj;
              --j;
            } else {
              stop = true;
            }
          }
        }
      }
      m = j + 1;
    } else {
      m = T > 0 ? 1 : 0;
    }
    sm[0] = m;
  }
  __syncthreads();
  const int m = sm[0];
  // kept per sector: its eigenvalues of global rank < m (a prefix of its
  // descending list), capped by the sector's rank bound
  for (int i = tid; i < np; i += TNT) {
    int kq = 0;
    for (int e = PO[i]; e < PO[i + 1]; ++e) kq += RK[e] < m ? 1 : 0;
    const int kb = kq < I.bound[i] ? kq : I.bound[i];
    I.kept[i] = kb;
    if (fastp) KQ[i] = kb;
  }
  __syncthreads();
  double kw = 0;
  for (int i = 0; i < np; ++i) {
    const int ki = fastp ? KQ[i] : I.kept[i];
    for (int j = tid; j < ki; j += TNT) kw += LAM[PO[i] + j];
  }
  kw = block_sum_t(kw, red);
  if (tid == 0) {
    I.keptw[0] = kw;
    I.keptw[1] = (I.normalize && kw > 1e-32) ? 1.0 / sqrt(kw) : 1.0;
  }
}
// dynamic LDS of k_truncate for np problems
__host__ __device__ inline int truncate_lds(int np) { return kMaxEig * (8 + 8 + 4) + 4 * (np + 2); }

}  // namespace hbm

#include "hbm_eig.hpp"
