// Register-resident Hermitian eigensolver of the HBM engine (Gram blocks of
// order 64 < n <= 192: the sector blocks of chi = 256 chains).
//
// The reference's truncation (ITensor denmatDecomp, called at
// src/BH_tDMRG.cpp:178,191,209) diagonalises rho = Θ Θ^H per U(1) sector.
// k_heev_vals (hbm_device.hpp) streams the Gram block through L2 for every
// Householder column once it outgrows LDS (n > 88): 1.5 ms per n = 194
// block, bound by one CU's L2 bandwidth.  Here one 512-thread workgroup keeps
// the whole lower triangle of the block in VGPRs (42 complex per lane, 168
// VGPRs) for the n - 1 Householder steps, so the O(n^3) traffic never leaves
// the CU; only O(n) vectors go through LDS.
//
// Thread grid 16 x 32: lane l of wave w is thread-row r = 2w + (l >> 5) and
// thread-column c = l & 31; element (i, k), i >= k, lives in thread (i mod 16,
// k mod 32), slot (a = i / 16, b = k / 32).  Slots with a < 2b hold no lower
// element and are not stored.
//
// Same conventions as the L2 kernels, so either vecs kernel can follow either
// vals kernel: Householder vector j in column j of P.A (rows j+1..n-1,
// u[j+1] = u0), H_j = I - tau_j u u^H, subdiagonal beta_j made real by the
// phases P.ph, eigenvalues descending in P.w.
#pragma once

namespace hbm {

constexpr int RNT = 256;                 // threads of the register tridiagonalisation (1 wave per SIMD)
constexpr int VNT = 512;                 // threads of the eigenvector kernel
constexpr int RATMAX = 13;               // largest slot grid (k_heev_vals_reg<13>)
constexpr int RNMAX = 16 * RATMAX;       // 208
constexpr int kRegMin = 16;              // blocks of order >= kRegMin go to the register kernels (tiny ones: LDS kernel)
constexpr int kRegSplit = 192;           // n <= 192: 12 x 12 slots (no spills); up to 208: 13 x 13
// slot grid used for a block of order n (16 rows per slot)
__host__ __device__ constexpr int reg_grid(int n) {
  return n <= 32 ? 2 : n <= 64 ? 4 : n <= 128 ? 8 : n <= kRegSplit ? 12 : 13;
}

// Workgroup barrier that waits for LDS traffic only: __syncthreads() also
// drains the global stores of the Householder vectors (vmcnt(0)) at every
// barrier, which no other workgroup reads during this kernel.
#ifdef HBM_STAMP  // diagnostic builds (tools/eig_bench): per-phase shader cycles of wave 0
#define STAMP(slot)                                                                 \
  do {                                                                              \
    __builtin_amdgcn_sched_barrier(0);                                              \
    unsigned long long t_;                                                          \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");      \
    __builtin_amdgcn_sched_barrier(0);                                              \
    stamp_acc[slot] += t_ - stamp_last;                                             \
    stamp_last = t_;                                                                \
  } while (0)
#else
#define STAMP(slot) do {} while (0)
#endif
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// q <- (d - x) - e2 / q with a refined hardware reciprocal (v_rcp_f64 + one
// Newton step: relative error ~1e-18, far below the bisection tolerance)
__device__ __forceinline__ double sturm_next(double dmx, double e2, double q) {
  double r = __builtin_amdgcn_rcp(q);
  r = fma(r, fma(-q, r, 1.0), r);
  return fma(-e2, r, dmx);
}
// counts of eigenvalues of the real symmetric tridiagonal (d, e2) below four shifts
__device__ __forceinline__ void sturm_count4(const double* d, const double* e2, int n, const double* x,
                                             double pivmin, int* cnt) {
  double q[4];
  int c[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    q[t] = d[0] - x[t];
    if (fabs(q[t]) < pivmin) q[t] = -pivmin;
    c[t] = q[t] < 0 ? 1 : 0;
  }
  // four steps' LDS loads issued ahead of their dependent chains
  int i = 1;
  for (; i + 3 < n; i += 4) {
    double dv[4], ev[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { dv[u] = d[i + u]; ev[u] = e2[i + u - 1]; }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        q[t] = sturm_next(dv[u] - x[t], ev[u], q[t]);
        if (fabs(q[t]) < pivmin) q[t] = -pivmin;
        c[t] += q[t] < 0 ? 1 : 0;
      }
  }
  for (; i < n; ++i) {
    const double di = d[i], ei = e2[i - 1];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      q[t] = sturm_next(di - x[t], ei, q[t]);
      if (fabs(q[t]) < pivmin) q[t] = -pivmin;
      c[t] += q[t] < 0 ? 1 : 0;
    }
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) cnt[t] = c[t];
}

// counts below KS shifts (sturm_count4's recurrence and guard for any KS)
template <int KS>
__device__ __forceinline__ void sturm_countk(const double* d, const double* e2, int n, const double* x,
                                             double pivmin, int* cnt) {
  double q[KS];
  int c[KS];
#pragma unroll
  for (int t = 0; t < KS; ++t) {
    q[t] = d[0] - x[t];
    if (fabs(q[t]) < pivmin) q[t] = -pivmin;
    c[t] = q[t] < 0 ? 1 : 0;
  }
  int i = 1;
  for (; i + 3 < n; i += 4) {
    double dv[4], ev[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { dv[u] = d[i + u]; ev[u] = e2[i + u - 1]; }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int t = 0; t < KS; ++t) {
        q[t] = sturm_next(dv[u] - x[t], ev[u], q[t]);
        if (fabs(q[t]) < pivmin) q[t] = -pivmin;
        c[t] += q[t] < 0 ? 1 : 0;
      }
  }
  for (; i < n; ++i) {
    const double di = d[i], ei = e2[i - 1];
#pragma unroll
    for (int t = 0; t < KS; ++t) {
      q[t] = sturm_next(di - x[t], ei, q[t]);
      if (fabs(q[t]) < pivmin) q[t] = -pivmin;
      c[t] += q[t] < 0 ? 1 : 0;
    }
  }
#pragma unroll
  for (int t = 0; t < KS; ++t) cnt[t] = c[t];
}
// Multisection of the eigenvalues te = t0 .. t0 + ne - 1 (descending) of the
// resolved ones: g = NTH / ne threads per eigenvalue (NTH / SPE in the split
// kernel), KS shifts per thread, so KS g + 1 sub-intervals per round.  One
// thread per eigenvalue and one shift (KS = 1, plain bisection) does the least
// Sturm work per digit (rounds x shifts: 50 x 1 against 22 x 4), and at one
// wave per SIMD the sequences are issue-bound, so it is the fastest choice.
template <int KS, int NTH>
__device__ __forceinline__ void multisect(const double* Ld, const double* Le2, int n, double gl0, double gu,
                                          double atol, double pivmin, int t0, int ne, int g, double* w, double* lo,
                                          double* hi, int* cnt) {
  const int tid = threadIdx.x;
  const double eps = 2.220446049250313e-16;
  const int t = tid / g, s = tid - t * g, te = t0 + t;
  const int np = KS * g + 1;  // sub-intervals per round
  __syncthreads();
  for (int tt = tid; tt < ne; tt += NTH) { lo[tt] = gl0; hi[tt] = gu; }
  __syncthreads();
  for (int it = 0; it < 256; ++it) {
    bool active = false;
    if (t < ne) {
      const double l = lo[t], h = hi[t];
      active = h - l > atol + 2.0 * eps * fmax(fabs(l), fabs(h));
      if (active) {
        double x[KS];
#pragma unroll
        for (int q = 0; q < KS; ++q) x[q] = l + (h - l) * double(KS * s + q + 1) / np;
        sturm_countk<KS>(Ld, Le2, n, x, pivmin, cnt + KS * tid);
      }
    }
    if (!__syncthreads_or(active)) break;
    if (t < ne && s == 0 && active) {
      const int idx = n - 1 - te;  // ascending index of the te-th largest
      const double l = lo[t], h = hi[t];
      double nl = l, nh = h;
      for (int q = 1; q < np; ++q) {
        const double x = l + (h - l) * double(q) / np;
        if (cnt[KS * (t * g) + q - 1] > idx) { nh = x; break; }
        nl = x;
      }
      lo[t] = nl;
      hi[t] = nh;
    }
    __syncthreads();
  }
  for (int tt = tid; tt < ne; tt += NTH) w[t0 + tt] = 0.5 * (lo[tt] + hi[tt]);
}

// All eigenvalues (descending) of a real symmetric tridiagonal held in LDS
// (Ld, Le2 = e^2), by multisection: g = NTH / n threads per eigenvalue, each
// evaluating four Sturm counts per round (LAPACK dstebz bounds / tolerances).
// Work arrays in LDS: lo, hi (n), cnt (4 * NTH ints).
template <int NTH>
__device__ __forceinline__ void bisect_all(const double* Ld, const double* Le2, int n, double thr_rel, double* w,
                                           double* lo, double* hi, int* cnt, int ks = 4) {
  const int tid = threadIdx.x;
  __shared__ double bb[4][NTH / 64];
  __shared__ int sres;
  double gl = 1e300, gu = -1e300, emax = 0, tr = 0;
  for (int i = tid; i < n; i += NTH) {
    const double el = i > 0 ? sqrt(Le2[i - 1]) : 0.0, er = i + 1 < n ? sqrt(Le2[i]) : 0.0;
    gl = fmin(gl, Ld[i] - el - er);
    gu = fmax(gu, Ld[i] + el + er);
    emax = fmax(emax, Le2[i]);
    tr += Ld[i];
  }
  for (int o = 32; o > 0; o >>= 1) {
    gl = fmin(gl, __shfl_xor(gl, o, 64));
    gu = fmax(gu, __shfl_xor(gu, o, 64));
    emax = fmax(emax, __shfl_xor(emax, o, 64));
    tr += __shfl_xor(tr, o, 64);
  }
  if ((tid & 63) == 0) { bb[0][tid >> 6] = gl; bb[1][tid >> 6] = gu; bb[2][tid >> 6] = emax; bb[3][tid >> 6] = tr; }
  __syncthreads();
  gl = bb[0][0]; gu = bb[1][0]; emax = bb[2][0]; tr = bb[3][0];
  for (int i = 1; i < NTH / 64; ++i) {
    gl = fmin(gl, bb[0][i]); gu = fmax(gu, bb[1][i]); emax = fmax(emax, bb[2][i]); tr += bb[3][i];
  }
  const double eps = 2.220446049250313e-16, safmin = 2.2250738585072014e-308;
  const double tnorm = fmax(fabs(gl), fabs(gu));
  const double pivmin = safmin * fmax(1.0, emax);
  gl -= 2.0 * eps * tnorm * n + 2.0 * pivmin;
  gu += 2.0 * eps * tnorm * n + 2.0 * pivmin;
  const double atol = 4.0 * eps * tnorm;
  // eigenvalues below thr are not resolved: their number from one Sturm
  // count, each set to their mean (trace minus the resolved ones)
  const double thr = thr_rel * tr;
  if (tid == 0) {
    int below = 0;
    if (thr > 0) {
      double x[4] = {thr, thr, thr, thr};
      int c4[4];
      sturm_count4(Ld, Le2, n, x, pivmin, c4);
      below = c4[0];
    }
    sres = n - below;
  }
  __syncthreads();
  const int nres = sres;
  // resolved eigenvalues (the nres largest) in rounds of NTH
  if (ks == 1) {  // uniform (EProb::ks)
    for (int t0 = 0; t0 < nres; t0 += NTH) {
      const int ne = nres - t0 < NTH ? nres - t0 : NTH;
      multisect<1, NTH>(Ld, Le2, n, nres < n ? fmax(gl, thr) : gl, gu, atol, pivmin, t0, ne, NTH / ne, w, lo, hi, cnt);
    }
  } else
  for (int t0 = 0; t0 < nres; t0 += NTH) {
    const int ne = nres - t0 < NTH ? nres - t0 : NTH;
    const int g = NTH / ne;  // threads per eigenvalue
    const int t = tid / g, s = tid - t * g, te = t0 + t;
    const int np = 4 * g + 1;  // sub-intervals per round
    __syncthreads();
    for (int tt = tid; tt < ne; tt += NTH) { lo[tt] = nres < n ? fmax(gl, thr) : gl; hi[tt] = gu; }
    __syncthreads();
    for (int it = 0; it < 128; ++it) {
      bool active = false;
      if (t < ne) {
        const double l = lo[t], h = hi[t];
        active = h - l > atol + 2.0 * eps * fmax(fabs(l), fabs(h));
        if (active) {
          double x[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) x[q] = l + (h - l) * double(4 * s + q + 1) / np;
          sturm_count4(Ld, Le2, n, x, pivmin, cnt + 4 * tid);
        }
      }
      if (!__syncthreads_or(active)) break;
      if (t < ne && s == 0 && active) {
        const int idx = n - 1 - te;  // ascending index of the te-th largest
        const double l = lo[t], h = hi[t];
        double nl = l, nh = h;
        for (int q = 1; q < np; ++q) {
          const double x = l + (h - l) * double(q) / np;
          if (cnt[4 * (t * g) + q - 1] > idx) { nh = x; break; }
          nl = x;
        }
        lo[t] = nl;
        hi[t] = nh;
      }
      __syncthreads();
    }
    for (int tt = tid; tt < ne; tt += NTH) w[t0 + tt] = 0.5 * (lo[tt] + hi[tt]);
  }
  if (nres < n) {
    __syncthreads();
    double sr = 0;
    for (int t = tid; t < nres; t += NTH) sr += w[t];
    for (int o = 32; o > 0; o >>= 1) sr += __shfl_xor(sr, o, 64);
    if ((tid & 63) == 0) bb[0][tid >> 6] = sr;
    __syncthreads();
    sr = 0;
    for (int i = 0; i < NTH / 64; ++i) sr += bb[0][i];
    const double mean = fmin(fmax((tr - sr) / (n - nres), 0.0), thr);
    for (int t = nres + tid; t < n; t += NTH) w[t] = mean;
  }
}

// Householder tridiagonalisation with the block in registers + eigenvalues.
// idx: the problems of this launch (blockIdx.x -> probs[idx[blockIdx.x]]).
//
// Thread grid 16 x 16: lane l of wave w is thread-row r = 4w + (l >> 4) and
// thread-column c = l & 15; element (i, k), i >= k, lives in thread
// (i mod 16, k mod 16), slot (a = i / 16, b = k / 16), b <= a: 91 complex per
// lane (364 registers; the compiler keeps the overflow in AGPRs).
//
// Branch-free sweeps: the LDS vectors u, p are zero outside the trailing
// block [j+1, n), so dead rows and columns contribute nothing to the matvec
// and are left unchanged by the rank-2 update.  Only the diagonal slots
// (a = b) mix lower and upper elements; their lane masks (c <= r, c < r) are
// fixed per thread (upper elements accumulate garbage in the update and are
// masked out of the matvec).
__device__ __forceinline__ z zsel(bool p, z a, z b) {
  z r;
  r.x = p ? a.x : b.x;
  r.y = p ? a.y : b.y;
  return r;
}
// dynamic LDS of the register tridiagonalisation for slot grid RAT
__host__ __device__ constexpr int reg_lds_bytes(int RAT) {
  return 16 * (2 * RAT * 16 * 17 + 5 * 16 * RAT + 2) + 8 * (2 * 16 * RAT + 3 * (RNT / 64)) + 64;
}
template <int RAT>
__device__ __forceinline__ void heev_vals_reg_body(const EProb& P, char* smem) {
  constexpr int RNS = RAT * (RAT + 1) / 2;  // slot (a, b), b <= a, at a (a + 1) / 2 + b
  constexpr int NM = 16 * RAT;
  const int n = P.n;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int r = 4 * wv + (lane >> 4), c = lane & 15;
  // LDS (carved from the launch's dynamic buffer): row / column partials
  // (rows padded to 17 against bank conflicts), vectors
  typedef z Part[16][17];
  Part* rowbuf = (Part*)smem;
  Part* colbuf = rowbuf + RAT;
  z(*su)[NM] = (z(*)[NM])(colbuf + RAT);
  z* sp = (z*)(su + 2);
  z* sbeta = sp + NM;
  z* salpha = sbeta + NM;
  double* sd = (double*)(salpha + 2);
  double* se2 = sd + NM;
  double(*sred)[RNT / 64] = (double(*)[RNT / 64])(se2 + NM);
  double* skp = (double*)(sred + 2);

  for (int i = tid; i < NM; i += RNT) {
    su[0][i] = mk(0, 0);
    su[1][i] = mk(0, 0);
    sp[i] = mk(0, 0);
  }
  const bool dle = c <= r, dlt = c < r;  // diagonal-slot masks
  double Ar[RNS], Ai[RNS];
#pragma unroll
  for (int a = 0; a < RAT; ++a)
#pragma unroll
    for (int b = 0; b <= a; ++b) {
      const int s = a * (a + 1) / 2 + b;
      const int i = 16 * a + r, k = 16 * b + c;
      z v = mk(0, 0);
      if (i < n && k <= i) v = P.A[(size_t)i * n + k];
      Ar[s] = v.x;
      Ai[s] = v.y;
    }
  __syncthreads();
  // column j's owners (c = j mod 16): publish x = A[j+1.., j] (zeros at j-1,
  // j), the partial norm over rows >= j+2 (one per wave) and the final
  // diagonal A[j][j]
  auto colprep = [&](int j) {
    double sacc = 0;
    const int bj = j >> 4;  // uniform
    if (tid == 0 && j >= 1) su[j & 1][j - 1] = mk(0, 0);  // stale entry below the owners' rows
    if (c == (j & 15)) {
      z* u = su[j & 1];
#pragma unroll
      for (int b = 0; b < RAT; ++b) {
        if (b != bj) continue;  // uniform
#pragma unroll
        for (int a = b; a < RAT; ++a) {
          constexpr int dummy = 0;
          (void)dummy;
          const int s = a * (a + 1) / 2 + b;  // slot of (a, b)
          const int i = 16 * a + r;
          const bool live = i >= j + 1 && i < n;
          const double xr = live ? Ar[s] : 0.0, xi = live ? Ai[s] : 0.0;
          if (i < NM) u[i] = mk(xr, xi);
          if (i == j) sd[j] = Ar[s];
          if (i == j + 1) salpha[j & 1] = mk(xr, xi);
          sacc = fma(xr, xr, fma(xi, xi, sacc));
        }
      }
    }
    sacc += __shfl_xor(sacc, 16, 64);
    sacc += __shfl_xor(sacc, 32, 64);
    if (lane == (j & 15)) sred[j & 1][wv] = sacc;
  };
#ifdef HBM_STAMP
  unsigned long long stamp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, stamp_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(stamp_last)::"memory");
#endif
  colprep(0);
  for (int j = 0; j + 1 < n; ++j) {
    STAMP(0);
    lds_barrier();  // A: column j published
    STAMP(1);
    z* u = su[j & 1];
    double snorm = 0;
#pragma unroll
    for (int q = 0; q < RNT / 64; ++q) snorm += sred[j & 1][q];
    const z alpha = salpha[j & 1];
    // colprep summed |x|^2 over rows >= j+1 (alpha included): xn = ||x||,
    // tau = 2 / (|u0|^2 + |tail|^2) = 1 / (xn (xn + |alpha|)) without cancellation
    const double aa = sqrt(alpha.x * alpha.x + alpha.y * alpha.y), xn = sqrt(snorm);
    double tau = 0;
    z beta = mk(0, 0), u0 = alpha;
    if (xn > 0) {
      const double ia = aa > 0 ? 1.0 / aa : 0.0;
      const z ph = aa > 0 ? mk(alpha.x * ia, alpha.y * ia) : mk(1, 0);
      beta = mk(-ph.x * xn, -ph.y * xn);
      u0 = mk(alpha.x + ph.x * xn, alpha.y + ph.y * xn);
      tau = 1.0 / (xn * (xn + aa));
    }
    if (tid == 0) {
      P.tau[j] = tau;
      sbeta[j] = beta;
    }
    STAMP(2);
    // every thread computed the same u0: element j + 1 of the Householder vector
    // is taken from the register (the LDS copy still holds alpha until
    // colprep(j + 2) clears it), so no barrier publishes it
    const int j1 = j + 1;
    auto uat = [&](int i) { return i == j1 ? u0 : u[i]; };
    // Householder vector -> column j of P.A (rows j+1 ..)
    for (int i = j + 1 + tid; i < n; i += RNT) P.A[(size_t)i * n + j] = uat(i);
    const int a0 = (j + 1) >> 4;  // first live slot row / column (uniform)
    if (tau != 0.0) {  // uniform: every thread computed the same reflector
      // ---- p = tau A_t u (lower storage: row and column contributions)
      const int aend = (n + 15) >> 4;  // slot rows holding rows < n (uniform)
      z uk[RAT], cp[RAT];
#pragma unroll
      for (int b = 0; b < RAT; ++b) {
        uk[b] = (b >= a0 && b < aend) ? uat(16 * b + c) : mk(0, 0);
        cp[b] = mk(0, 0);
      }
#pragma unroll
      for (int a = 0; a < RAT; ++a) {
        if (a < a0 || a >= aend) continue;
        const z ui = uat(16 * a + r);
        z acc = mk(0, 0);
#pragma unroll
        for (int b = 0; b <= a; ++b) {
          if (b < a0) continue;
          const int s = a * (a + 1) / 2 + b;
          double ar = Ar[s], ai = Ai[s], cr = Ar[s], ci = Ai[s];
          if (b == a) {
            ar = dle ? ar : 0.0;
            ai = dlt ? ai : 0.0;  // the diagonal is real
            cr = dlt ? cr : 0.0;
            ci = dlt ? ci : 0.0;
          }
          acc.x = fma(ar, uk[b].x, fma(-ai, uk[b].y, acc.x));
          acc.y = fma(ar, uk[b].y, fma(ai, uk[b].x, acc.y));
          cp[b].x = fma(cr, ui.x, fma(ci, ui.y, cp[b].x));  // conj(A) ui
          cp[b].y = fma(cr, ui.y, fma(-ci, ui.x, cp[b].y));
        }
        rowbuf[a][r][c] = acc;
      }
#pragma unroll
      for (int b = 0; b < RAT; ++b)
        if (b >= a0 && b < aend) colbuf[b][r][c] = cp[b];
      STAMP(4);
      lds_barrier();  // B: partials in LDS
      STAMP(5);
      // ---- p_k for k in the trailing block, and Re(u^H p) partials
      double kp = 0;
      {
        const int k = j + 1 + tid;
        if (k < n) {
          const int a = k >> 4, cc = k & 15;
          z sacc = mk(0, 0);
#pragma unroll
          for (int q = 0; q < 16; ++q) sacc = zadd(sacc, zadd(rowbuf[a][cc][q], colbuf[a][q][cc]));
          const z pk = zsc(sacc, tau);
          sp[k] = pk;
          const z ukk = uat(k);
          kp = ukk.x * pk.x + ukk.y * pk.y;
        }
        if (tid == 0) sp[j] = mk(0, 0);  // leaves the trailing block
      }
      for (int o = 32; o > 0; o >>= 1) kp += __shfl_xor(kp, o, 64);
      if (lane == 0) skp[wv] = kp;
      STAMP(6);
      lds_barrier();  // C: p and the K partials in LDS
      STAMP(5);
      double K = 0;
#pragma unroll
      for (int q = 0; q < RNT / 64; ++q) K += skp[q];
      K *= 0.5 * tau;
      // ---- A_t -= u w^H + w u^H, w = p - K u (zero outside the trailing block)
#pragma unroll
      for (int b = 0; b < RAT; ++b) {
        const int k = 16 * b + c;
        cp[b] = (b >= a0 && b < aend) ? zsub(sp[k], zsc(uk[b], K)) : mk(0, 0);  // cp now holds w_k
      }
#pragma unroll
      for (int a = 0; a < RAT; ++a) {
        if (a < a0 || a >= aend) continue;
        const int i = 16 * a + r;
        const z ui = uat(i);
        const z wi = zsub(sp[i], zsc(ui, K));
#pragma unroll
        for (int b = 0; b <= a; ++b) {
          if (b < a0) continue;
          const int s = a * (a + 1) / 2 + b;
          // v -= u_i conj(w_k) + w_i conj(u_k)
          Ar[s] = fma(-ui.x, cp[b].x, fma(-ui.y, cp[b].y, fma(-wi.x, uk[b].x, fma(-wi.y, uk[b].y, Ar[s]))));
          Ai[s] = fma(-ui.y, cp[b].x, fma(ui.x, cp[b].y, fma(-wi.y, uk[b].x, fma(wi.x, uk[b].y, Ai[s]))));
        }
      }
    } else {
      lds_barrier();  // keep this column's reads of sred ahead of colprep(j + 1)
    }
    STAMP(7);
    colprep(j + 1);
  }
#ifdef HBM_STAMP
  STAMP(0);
  if (tid == 0)
    for (int q = 0; q < 8; ++q) P.Z[q] = double(stamp_acc[q]);
#endif
  __syncthreads();
  // ---- real tridiagonal: d (diagonal), |beta| (off-diagonal), phases
  if (tid == 0) {
    z dl = mk(1, 0);
    P.ph[0] = dl;
    for (int j = 0; j + 1 < n; ++j) {
      const z b = sbeta[j];
      const double ab = sqrt(b.x * b.x + b.y * b.y);
      if (ab > 0) dl = zmul(dl, mk(b.x / ab, b.y / ab));
      P.ph[j + 1] = dl;
      P.e[j] = ab;
      se2[j] = ab * ab;
    }
    P.e[n - 1] = 0;
    se2[n - 1] = 0;
  }
  for (int j = tid; j < n; j += RNT) P.d[j] = sd[j];
  __syncthreads();
  // ---- eigenvalues (work arrays reuse the partial buffers)
  double* lo = (double*)&rowbuf[0][0][0];
  double* hi = lo + NM;
  int* cnt = (int*)(hi + NM);
#ifndef HBM_NO_BISECT  // timing builds of tools/eig_bench only
  if (!P.defer) bisect_all<RNT>(sd, se2, n, P.thr_rel, P.w, lo, hi, cnt, P.ks);
#endif
}

// lane l's value of v (l uniform)
__device__ __forceinline__ double rdl(double v, int l) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(unsigned long long)b, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)((unsigned long long)b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// ------------------------------------------------- certified Cholesky (gauge moves)
// A gauge move (MPS::position: cutoff 1e-14, no Maxm) keeps every eigenvalue
// of its Gram blocks when the smallest exceeds 10 x cutoff x total (the
// eigen path would discard nothing), and then any factorisation with the
// moving side orthonormal gives the same state and bond dims.  The host
// (Engine::fast_certify / fast_factors) factors those moves by CholeskyQR2;
// this kernel gives one Gram block's Cholesky factor G = R^H R (R upper),
// R^-1 and the certificate inputs: trace(G) and ||R^-1||_F^2, whose inverse
// bounds lambda_min(G) from below (||R^-1||_2 <= ||R^-1||_F).
struct CholProb {
  const z* G;   // n x n Hermitian (ld n)
  z* R;         // out: upper factor, zero below (ld n)
  z* Ri;        // out: R^-1, upper (ld n)
  double* res;  // out: [0] trace(G), [1] ||R^-1||_F^2 or -1 (a pivot <= 0)
  int n;
};
constexpr int kCholMax = 64;  // orders held in LDS (G and R^-1: 2 x 64 x 65 complex)
// one workgroup per block, blocked by 16 rows of R: wave 0 factors the
// panel (rows b0..b0+15, lane = column b0 + lane) in registers, the pivots and
// the entries conj(R[i][a]) coming by readlane; a barrier; the trailing upper
// triangle takes the panel's rank-16 update (threads over elements); a
// barrier.  Then column j of R^-1 by thread j (back substitution).
__global__ __launch_bounds__(NT) void k_chol_cert(const CholProb* __restrict__ probs) {
  __shared__ z Gs[kCholMax][kCholMax + 1];
  __shared__ z Rs[kCholMax][kCholMax + 1];
  __shared__ double red[NT / 64];
  __shared__ int sbad;
  const CholProb P = probs[blockIdx.x];
  const int n = P.n, tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  for (int e = tid; e < n * n; e += NT) {
    const int i = e / n, j = e - i * n;
    Gs[i][j] = P.G[e];
  }
  __syncthreads();
  const double tr = block_sum(tid < n ? Gs[tid][tid].x : 0.0, red);
  bool ok = true;
  for (int b0 = 0; b0 < n; b0 += 16) {
    const int be = b0 + 16 < n ? b0 + 16 : n;
    if (wv == 0) {
      const int col = b0 + lane;  // n - b0 <= 64 columns from b0 on
      const bool lv = col < n;
      z pr[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const int row = b0 + c;
        pr[c] = (lv && row < be && col >= row) ? Gs[row][col] : mk(0, 0);
      }
      int pbad = 0;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const int i = b0 + c;
        if (i < be && !pbad) {  // uniform
          const double d = rdl(pr[c].x, c);  // lane c holds column i: its row-i entry
          if (!(d > 0)) {
            pbad = 1;
          } else {
            const double rii = sqrt(d), inv = 1.0 / rii;
            if (col > i) pr[c] = zsc(pr[c], inv);
            else if (col == i) pr[c] = mk(rii, 0);
#pragma unroll
            for (int c2 = c + 1; c2 < 16; ++c2) {
              const int a = b0 + c2;
              if (a < be) {  // G[a][b] -= conj(R[i][a]) R[i][b], b = col >= a
                const z ra = mk(rdl(pr[c].x, c2), -rdl(pr[c].y, c2));
                if (lv && col >= a) pr[c2] = zsub(pr[c2], zmul(ra, pr[c]));
              }
            }
          }
        }
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const int row = b0 + c;
        if (lv && row < be && col >= row) Gs[row][col] = pr[c];
      }
      if (lane == 0) sbad = pbad;
    }
    __syncthreads();
    if (sbad) { ok = false; break; }  // uniform
    const int m = n - be;
    for (int e = tid; e < m * m; e += NT) {
      const int aa = e / m, bb = e - aa * m;
      if (bb < aa) continue;
      const int a = be + aa, b = be + bb;
      z acc = Gs[a][b];
      for (int i = b0; i < be; ++i) acc = zsub(acc, zmul(zcj(Gs[i][a]), Gs[i][b]));
      Gs[a][b] = acc;
    }
    __syncthreads();
  }
  // column j of R^-1 by the four lanes 4j .. 4j+3 (one wave holds 16 columns):
  // each row's dot product split over the lanes, summed by two xor shuffles
  // inside the group (its lanes run the same trip count), the entry written by
  // the group's first lane and read back by all four (same wave: LDS in order)
  double inv2 = 0;
  {
    const int j = tid >> 2, s4 = tid & 3;
    if (ok && j < n) {
      const double djj = 1.0 / Gs[j][j].x;
      if (s4 == 0) {
        Rs[j][j] = mk(djj, 0);
        inv2 = djj * djj;
      }
      for (int i = j - 1; i >= 0; --i) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        z acc = mk(0, 0);
        for (int l = i + 1 + s4; l <= j; l += 4) acc = zadd(acc, zmul(Gs[i][l], Rs[l][j]));
        acc.x += __shfl_xor(acc.x, 1, 64);
        acc.y += __shfl_xor(acc.y, 1, 64);
        acc.x += __shfl_xor(acc.x, 2, 64);
        acc.y += __shfl_xor(acc.y, 2, 64);
        const z v = zsc(acc, -1.0 / Gs[i][i].x);
        if (s4 == 0) {
          Rs[i][j] = v;
          inv2 += v.x * v.x + v.y * v.y;
        }
      }
    }
  }
  inv2 = block_sum(inv2, red);  // uniform ok: every thread takes the same path
  if (!ok) {
    if (tid == 0) { P.res[0] = tr; P.res[1] = -1.0; }
    return;
  }
  for (int e = tid; e < n * n; e += NT) {
    const int i = e / n, j = e - i * n;
    P.R[e] = j >= i ? Gs[i][j] : mk(0, 0);
    P.Ri[e] = j >= i ? Rs[i][j] : mk(0, 0);
  }
  if (tid == 0) { P.res[0] = tr; P.res[1] = inv2; }
}

// ------------------------------------------------- Maxm boundary, then bisection
// When Maxm can bind (a decomposition with more than Maxm + 1 eigenvalues),
// the truncation keeps at most the Maxm largest of all its sectors' eigenvalues
// and needs the others only through their sum (trace - resolved: exact), so the
// sectors' eigenvalues below the (Maxm + 1)-th largest never have to be
// resolved.  k_heev_thresh brackets that eigenvalue for one decomposition by
// multisection over the union of its sectors' tridiagonals (Sturm counts
// summed over sectors), and raises each deferred sector's thr_rel to 0.999 x
// the bracket's lower end; k_heev_bisect then resolves only the eigenvalues
// above it (bisect_all: the others are set to their mean, below the
// threshold, so they rank behind every kept one and the suffix sums of the
// truncation rule stay exact).
constexpr int THN = 1024;          // threads of k_heev_thresh
constexpr int THC = 32;            // candidate shifts per multisection round
constexpr int kThrMaxT = 5120;     // eigenvalues of one decomposition (= kMaxEig)
__global__ __launch_bounds__(THN) void k_heev_thresh(const TItem* __restrict__ items, const int* __restrict__ which,
                                                    EProb* __restrict__ probs) {
  extern __shared__ __align__(16) char smem_th[];
  const TItem I = items[which[blockIdx.x]];
  const int tid = threadIdx.x, np = I.np;
  double* Ld = reinterpret_cast<double*>(smem_th);  // every sector's d, then e^2
  double* Le2 = Ld + kThrMaxT;
  __shared__ int off[65], cnt[THC];
  __shared__ double tr[64], piv[64], gub[64], sx[2];
  if (tid == 0) {
    int o = 0;
    for (int q = 0; q < np; ++q) { off[q] = o; o += probs[I.p0 + q].n; }
    off[np] = o;
  }
  __syncthreads();
  const int T = off[np];
  for (int q = 0; q < np; ++q) {
    const EProb& P = probs[I.p0 + q];
    for (int i = tid; i < P.n; i += THN) {
      Ld[off[q] + i] = P.d[i];
      Le2[off[q] + i] = P.e[i] * P.e[i];
    }
  }
  __syncthreads();
  // per sector: trace, Gershgorin upper bound, pivmin (one wave per sector)
  const int wv = tid >> 6, lane = tid & 63;
  for (int q = wv; q < np; q += THN / 64) {
    const int n = off[q + 1] - off[q];
    const double* d = Ld + off[q];
    const double* e2 = Le2 + off[q];
    double t = 0, g = -1e300, em = 0;
    for (int i = lane; i < n; i += 64) {
      const double el = i > 0 ? sqrt(e2[i - 1]) : 0.0, er = i + 1 < n ? sqrt(e2[i]) : 0.0;
      t += d[i];
      g = fmax(g, d[i] + el + er);
      em = fmax(em, e2[i]);
    }
    for (int o = 32; o > 0; o >>= 1) {
      t += __shfl_xor(t, o, 64);
      g = fmax(g, __shfl_xor(g, o, 64));
      em = fmax(em, __shfl_xor(em, o, 64));
    }
    if (lane == 0) { tr[q] = t; gub[q] = g; piv[q] = 2.2250738585072014e-308 * fmax(1.0, em); }
  }
  __syncthreads();
  if (tid == 0) {
    double g = 0;
    for (int q = 0; q < np; ++q) g = fmax(g, gub[q]);
    sx[0] = 0.0;              // lo: count(lambda > lo) >= target
    sx[1] = g * (1.0 + 1e-12) + 1e-300;  // hi: count(lambda > hi) < target
  }
  __syncthreads();
  const int target = I.maxm + 1;
  for (int round = 0; round < 12; ++round) {
    const double lo = sx[0], hi = sx[1];
    if (!(hi - lo > 1e-3 * hi)) break;  // uniform
    if (tid < THC) cnt[tid] = 0;
    __syncthreads();
    // (sector, candidate) pairs: count of eigenvalues above x_c = n - #below
    for (int pr = tid; pr < np * THC; pr += THN) {
      const int q = pr / THC, c = pr - q * THC;
      const int n = off[q + 1] - off[q];
      if (n <= 0) continue;
      const double x = lo + (hi - lo) * double(c + 1) / double(THC + 1);
      const int below = sturm(Ld + off[q], Le2 + off[q], n, x, piv[q]);
      atomicAdd(&cnt[c], n - below);
    }
    __syncthreads();
    if (tid == 0) {
      double nlo = lo, nhi = hi;
      for (int c = 0; c < THC; ++c) {
        const double x = lo + (hi - lo) * double(c + 1) / double(THC + 1);
        if (cnt[c] >= target) nlo = x;
        else { nhi = x; break; }
      }
      sx[0] = nlo;
      sx[1] = nhi;
    }
    __syncthreads();
  }
  const double thr = 0.999 * sx[0];
  if (T > target && thr > 0)
    for (int q = tid; q < np; q += THN) {
      EProb& P = probs[I.p0 + q];
      if (P.defer && tr[q] > 0) P.thr_rel = fmax(P.thr_rel, thr / tr[q]);
    }
}
__host__ __device__ constexpr int thresh_lds_bytes() { return 2 * kThrMaxT * 8; }

constexpr int BSN = 512;  // threads of k_heev_bisect
__global__ __launch_bounds__(BSN) void k_heev_bisect(const EProb* __restrict__ probs, const int* __restrict__ idx) {
  extern __shared__ __align__(16) char smem_bs[];
  const EProb P = probs[idx[blockIdx.x]];
  const int n = P.n, tid = threadIdx.x;
  double* Ld = reinterpret_cast<double*>(smem_bs);
  double* Le2 = Ld + n;
  double* lo = Le2 + n;
  double* hi = lo + n;
  int* cnt = reinterpret_cast<int*>(hi + n);
  for (int i = tid; i < n; i += BSN) {
    Ld[i] = P.d[i];
    Le2[i] = P.e[i] * P.e[i];
  }
  __syncthreads();
  bisect_all<BSN>(Ld, Le2, n, P.thr_rel, P.w, lo, hi, cnt, P.ks);
}
__host__ __device__ constexpr int bisect_lds_bytes(int n) { return 4 * n * 8 + 4 * BSN * 4 + 64; }

// ------------------------------------------------- split multisection (large blocks)
// A block's multisection inside k_heev_vals_any gives one thread (four shifts)
// to each eigenvalue once n > RNT / 2: 22 rounds of n-step Sturm sequences on
// one CU, 32 % of the kernel at n = 192, while the launch's other CUs have long
// finished their smaller blocks.  Blocks of order >= the split threshold are
// marked defer (the register kernel stops after the tridiagonal) and their
// eigenvalues are resolved here by ceil(n / spe) workgroups each: spe
// eigenvalues per workgroup, RNT / spe threads per eigenvalue (one shift each,
// EProb::ks = 1: RNT / spe + 1 sub-intervals per round).  Same bounds,
// tolerances and unresolved threshold as bisect_all (every workgroup of a block
// computes them identically).  The unresolved eigenvalues' mean needs all the
// resolved ones: the block's last workgroup to finish sets it (a per-block
// counter, zeroed by the host before the launch).
constexpr int SPE = 32;  // the largest chunk (split_spe: eigenvalues per workgroup, a divisor of RNT)
// bounds, tolerances and the number of resolved eigenvalues of (Ld, Le2) (uniform)
struct BisectBounds {
  double gl, gu, pivmin, atol, tr, thr;
  int nres;
};
template <int NTH>
__device__ __forceinline__ BisectBounds bisect_bounds(const double* Ld, const double* Le2, int n, double thr_rel) {
  const int tid = threadIdx.x;
  __shared__ double bb[4][NTH / 64];
  __shared__ int sres;
  double gl = 1e300, gu = -1e300, emax = 0, tr = 0;
  for (int i = tid; i < n; i += NTH) {
    const double el = i > 0 ? sqrt(Le2[i - 1]) : 0.0, er = i + 1 < n ? sqrt(Le2[i]) : 0.0;
    gl = fmin(gl, Ld[i] - el - er);
    gu = fmax(gu, Ld[i] + el + er);
    emax = fmax(emax, Le2[i]);
    tr += Ld[i];
  }
  for (int o = 32; o > 0; o >>= 1) {
    gl = fmin(gl, __shfl_xor(gl, o, 64));
    gu = fmax(gu, __shfl_xor(gu, o, 64));
    emax = fmax(emax, __shfl_xor(emax, o, 64));
    tr += __shfl_xor(tr, o, 64);
  }
  if ((tid & 63) == 0) { bb[0][tid >> 6] = gl; bb[1][tid >> 6] = gu; bb[2][tid >> 6] = emax; bb[3][tid >> 6] = tr; }
  __syncthreads();
  gl = bb[0][0]; gu = bb[1][0]; emax = bb[2][0]; tr = bb[3][0];
  for (int i = 1; i < NTH / 64; ++i) {
    gl = fmin(gl, bb[0][i]); gu = fmax(gu, bb[1][i]); emax = fmax(emax, bb[2][i]); tr += bb[3][i];
  }
  const double eps = 2.220446049250313e-16, safmin = 2.2250738585072014e-308;
  const double tnorm = fmax(fabs(gl), fabs(gu));
  BisectBounds B;
  B.pivmin = safmin * fmax(1.0, emax);
  B.gl = gl - (2.0 * eps * tnorm * n + 2.0 * B.pivmin);
  B.gu = gu + (2.0 * eps * tnorm * n + 2.0 * B.pivmin);
  B.atol = 4.0 * eps * tnorm;
  B.tr = tr;
  B.thr = thr_rel * tr;
  if (tid == 0) {
    int below = 0;
    if (B.thr > 0) {
      double x[4] = {B.thr, B.thr, B.thr, B.thr};
      int c4[4];
      sturm_count4(Ld, Le2, n, x, B.pivmin, c4);
      below = c4[0];
    }
    sres = n - below;
  }
  __syncthreads();
  B.nres = sres;
  return B;
}
// problem t.x, eigenvalues [SPE t.y, SPE t.y + SPE) of the resolved ones (descending)
__global__ __launch_bounds__(RNT) void k_heev_bisect_split(const EProb* __restrict__ probs,
                                                           const int2* __restrict__ tasks, int spe,
                                                           int* __restrict__ ctr) {
  extern __shared__ __align__(16) char smem_sp[];
  const int2 tk = tasks[blockIdx.x];
  const EProb P = probs[tk.x];
  const int n = P.n, tid = threadIdx.x;
  double* Ld = reinterpret_cast<double*>(smem_sp);
  double* Le2 = Ld + n;
  __shared__ double lo[SPE], hi[SPE];
  __shared__ int cnt[4 * RNT];
  for (int i = tid; i < n; i += RNT) {
    Ld[i] = P.d[i];
    Le2[i] = P.e[i] * P.e[i];
  }
  __syncthreads();
  const BisectBounds B = bisect_bounds<RNT>(Ld, Le2, n, P.thr_rel);
  const int t0 = spe * tk.y;
  if (t0 < B.nres) {  // uniform
    const int ne = B.nres - t0 < spe ? B.nres - t0 : spe;
    const double gl0 = B.nres < n ? fmax(B.gl, B.thr) : B.gl;
    // RNT / spe threads per eigenvalue (also when ne < spe: the same points)
    if (P.ks == 1) multisect<1, RNT>(Ld, Le2, n, gl0, B.gu, B.atol, B.pivmin, t0, ne, RNT / spe, P.w, lo, hi, cnt);
    else multisect<4, RNT>(Ld, Le2, n, gl0, B.gu, B.atol, B.pivmin, t0, ne, RNT / spe, P.w, lo, hi, cnt);
  }
  if (B.nres >= n) return;  // uniform: nothing unresolved, no count
  // every thread releases its eigenvalue stores, one lane counts; the block's
  // last workgroup acquires them and sets the unresolved ones to their mean
  __shared__ int last;
  __shared__ double bb[RNT / 64];
  __threadfence();
  __syncthreads();
  if (tid == 0) last = atomicAdd(ctr + tk.x, 1) == (n + spe - 1) / spe - 1;
  __syncthreads();
  if (!last) return;  // uniform
  __threadfence();
  double sr = 0;
  for (int t = tid; t < B.nres; t += RNT) sr += P.w[t];
  for (int o = 32; o > 0; o >>= 1) sr += __shfl_xor(sr, o, 64);
  if ((tid & 63) == 0) bb[tid >> 6] = sr;
  __syncthreads();
  sr = 0;
  for (int i = 0; i < RNT / 64; ++i) sr += bb[i];
  const double mean = fmin(fmax((B.tr - sr) / (n - B.nres), 0.0), B.thr);
  for (int t = B.nres + tid; t < n; t += RNT) P.w[t] = mean;
}
__host__ __device__ constexpr int bisect_split_lds_bytes(int n) { return 16 * n + 64; }
// One launch per decomposition: each workgroup picks the variant for its
// block's order (register slot grid 2 / 4 / 8 / 12 / 13, or the LDS / L2
// kernel for tiny and oversized blocks).  idx lists the problems, largest
// first.  Dynamic LDS: max over the variants present.
__global__ __launch_bounds__(RNT, 1) void k_heev_vals_any(const EProb* __restrict__ probs, const int* __restrict__ idx,
                                                          int reg_min) {
  extern __shared__ __align__(16) char smem_any[];
  const EProb P = probs[idx[blockIdx.x]];
  const int n = P.n;
  if (n >= reg_min && n <= RNMAX) {
    switch (reg_grid(n)) {
      case 2: heev_vals_reg_body<2>(P, smem_any); return;
      case 4: heev_vals_reg_body<4>(P, smem_any); return;
      case 8: heev_vals_reg_body<8>(P, smem_any); return;
      case 12: heev_vals_reg_body<12>(P, smem_any); return;
      default: heev_vals_reg_body<13>(P, smem_any); return;
    }
  }
  heev_vals_lds_body(P, smem_any);
}

// Gram blocks of order <= kSmallMax: the same bodies compiled apart, so that
// this launch's register and LDS footprint (slot grids 2 and 4, the LDS kernel)
// lets several workgroups share a CU instead of the 512 registers per lane
// the larger grids force on k_heev_vals_any.  Launched on the side stream
// beside k_heev_vals_any (Engine::decompose_eig).
constexpr int kSmallMax = 64;
__global__ __launch_bounds__(RNT, 2) void k_heev_vals_small(const EProb* __restrict__ probs,
                                                            const int* __restrict__ idx, int reg_min) {
  extern __shared__ __align__(16) char smem_small[];
  const EProb P = probs[idx[blockIdx.x]];
  const int n = P.n;
  if (n >= reg_min && n <= kSmallMax) {
    if (reg_grid(n) == 2) heev_vals_reg_body<2>(P, smem_small);
    else heev_vals_reg_body<4>(P, smem_small);
    return;
  }
  heev_vals_lds_body(P, smem_small);
}

// ------------------------------------------------------------------ vectors
// Kept eigenvectors U = Q D Z (n x k, ld k) of one problem per workgroup.
// Fast path (n <= RNMAX, k <= 64, Z fits LDS): inverse iteration on the real
// tridiagonal (one lane per eigenvalue), CholeskyQR2 of the k vectors with Z
// in LDS (classical Gram-Schmidt twice if a Cholesky pivot collapses), then
// U = D Z in registers (lane = column, rows i = 8a + wave) and the reflectors
// applied j = n-2 .. 0 from LDS blocks.  Other sizes: the same algorithm with
// Z in global memory (pivots in P.Dv) and U by k_heev_bt.
constexpr int kVecLds = 143360;  // bytes of the Z + pivot / Gram / reflector-block region
// Inverse iteration for eigenvalue lam into column jz of Z (ld ldz), one
// thread per eigenvalue, LDL^T pivots in column jd of Dv (ld ldd), LDS or
// global: pivots by a refined reciprocal, the forward and backward sweeps
// unrolled by 4 with their loads issued ahead of the dependent FMA chain (few
// threads carry the whole batch: nothing else hides the memory latency).
#ifndef INVIT_ITERS
#define INVIT_ITERS 2  // inverse-iteration sweeps per eigenvalue (3 until round 6: the same residuals, tools/gpu_invit.sh)
#endif
__device__ __forceinline__ void invit_fast(const double* __restrict__ Ld, const double* __restrict__ Le, int n,
                                           double lam, double tiny, double* __restrict__ Z, int ldz, int jz,
                                           double* __restrict__ Dv, int ldd, int jd, int jj) {
  // LDL^T of T - lam I; Dv keeps the pivots' reciprocals 1 / q_i (a refined
  // hardware reciprocal, computed once here), so neither sweep divides
  auto rcpr = [](double q) {
    double r = __builtin_amdgcn_rcp(q);
    return fma(r, fma(-q, r, 1.0), r);
  };
  double q = Ld[0] - lam;
  if (fabs(q) < tiny) q = q < 0 ? -tiny : tiny;
  for (int i = 1; i < n; ++i) {
    const double r = rcpr(q);
    Dv[(size_t)(i - 1) * ldd + jd] = r;
    q = fma(-Le[i - 1] * Le[i - 1], r, Ld[i] - lam);
    if (fabs(q) < tiny) q = q < 0 ? -tiny : tiny;
  }
  Dv[(size_t)(n - 1) * ldd + jd] = rcpr(q);
  for (int i = 0; i < n; ++i) Z[(size_t)i * ldz + jz] = hrand(i, jj);
  for (int it = 0; it < INVIT_ITERS; ++it) {
    // forward: y_i = b_i - (e_{i-1} / q_{i-1}) y_{i-1}
    double y = Z[jz];
    int i = 1;
    for (; i + 3 < n; i += 4) {
      double b[4], l[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        b[t] = Z[(size_t)(i + t) * ldz + jz];
        l[t] = Le[i + t - 1] * Dv[(size_t)(i + t - 1) * ldd + jd];
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        y = fma(-l[t], y, b[t]);
        Z[(size_t)(i + t) * ldz + jz] = y;
      }
    }
    for (; i < n; ++i) {
      y = fma(-Le[i - 1] * Dv[(size_t)(i - 1) * ldd + jd], y, Z[(size_t)i * ldz + jz]);
      Z[(size_t)i * ldz + jz] = y;
    }
    // backward: x_i = (y_i - e_i x_{i+1}) / q_i
    double xn = Z[(size_t)(n - 1) * ldz + jz] * Dv[(size_t)(n - 1) * ldd + jd];
    Z[(size_t)(n - 1) * ldz + jz] = xn;
    double ss = xn * xn;
    i = n - 2;
    for (; i - 3 >= 0; i -= 4) {
      double b[4], e[4], rq[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        b[t] = Z[(size_t)(i - t) * ldz + jz];
        e[t] = Le[i - t];
        rq[t] = Dv[(size_t)(i - t) * ldd + jd];
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        xn = fma(-e[t], xn, b[t]) * rq[t];
        Z[(size_t)(i - t) * ldz + jz] = xn;
        ss = fma(xn, xn, ss);
      }
    }
    for (; i >= 0; --i) {
      xn = (Z[(size_t)i * ldz + jz] - Le[i] * xn) * Dv[(size_t)i * ldd + jd];
      Z[(size_t)i * ldz + jz] = xn;
      ss = fma(xn, xn, ss);
    }
    const double inv = ss > 0 ? 1.0 / sqrt(ss) : 0.0;
    for (int t = 0; t < n; ++t) Z[(size_t)t * ldz + jz] *= inv;
  }
}

// problems whose eigenvectors the vecs kernel finishes itself (Z in LDS, U in registers)
__device__ __forceinline__ bool vecs_fast(int n, int k) {
  return n <= RNMAX && k <= 64 && (size_t(n) * (k + 1) + size_t(n) + 64 * 65) * 8 <= size_t(kVecLds);
}
// the others of order <= kBtRows leave Z (ld n) in P.Z for k_heev_bt
constexpr int kBtRows = 512;
constexpr int BNT = 256;  // threads of k_heev_bt (one wave per SIMD: 32 rows x 2 complex per lane in VGPRs)
constexpr int kBtBlk = 16;  // reflectors per LDS block (16 x 512 complex = 128 KB)
constexpr int kVecRows = (RNMAX + VNT / 64 - 1) / (VNT / 64);  // rows per thread (fast path)
constexpr int kRefBlk = 24;                   // reflectors per LDS block

template <class T>
__device__ __forceinline__ T block_sum_r(T v, T* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int tid = threadIdx.x;
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  T s = 0;
#pragma unroll
  for (int i = 0; i < VNT / 64; ++i) s += red[i];
  return s;
}


// Blocked right-looking Cholesky G = L L^T of the lower triangle of G
// (order k <= 128, ld ldg, LDS) by the workgroup, 16 columns per block: wave 0
// factors the block's panel (rows b0..k-1) in registers, a barrier, then the trailing lower triangle takes the block's
// rank-16 update on the matrix cores (16 x 16 tiles over the waves; lane l
// holds L[row 16 I + (l & 15)][b0 + kk] and L[col 16 J + (l & 15)][b0 + kk],
// kk = 4 s + (l >> 4)), a barrier.  false (uniform): a pivot <= 1e-10 (the
// columns are unit vectors: a near dependency).  Caller: barrier before (G
// written), none needed after.
__device__ __forceinline__ bool chol_wg(double* G, int ldg, int k) {
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int a16 = lane & 15, kq = lane >> 4;
  __shared__ int chol_bad;
  for (int b0 = 0; b0 < k; b0 += 16) {
    const int be = b0 + 16 < k ? b0 + 16 : k;
    if (wv == 0) {
      // the panel in registers: lane holds rows lane and lane + 64 of its 16 columns;
      // column c's pivot and the entries L[b0 + c2][b0 + c] come by readlane
      int bad = 0;
      double pr[2][16];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          const int row = lane + 64 * h;
          pr[h][c] = (row < k && b0 + c < be && b0 + c <= row) ? G[row * ldg + b0 + c] : 0.0;
        }
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const int cc = b0 + c;
        if (cc < be && !bad) {  // uniform; no break: every register index stays static
          const double dgg = rdl(cc < 64 ? pr[0][c] : pr[1][c], cc & 63);
          if (!(dgg > 1e-10)) {
            bad = 1;
          } else {
            const double dd = sqrt(dgg), inv = 1.0 / dd;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int row = lane + 64 * h;
              pr[h][c] = row > cc ? pr[h][c] * inv : (row == cc ? dd : pr[h][c]);
            }
#pragma unroll
            for (int c2 = c + 1; c2 < 16; ++c2) {
              const int j = b0 + c2;
              if (j < be) {
                const double ljc = rdl(j < 64 ? pr[0][c] : pr[1][c], j & 63);
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                  const int row = lane + 64 * h;
                  if (row >= j) pr[h][c2] = fma(-pr[h][c], ljc, pr[h][c2]);
                }
              }
            }
          }
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          const int row = lane + 64 * h;
          if (row < k && b0 + c < be && b0 + c <= row) G[row * ldg + b0 + c] = pr[h][c];
        }
      if (lane == 0) chol_bad = bad;
    }
    __syncthreads();
    if (chol_bad) return false;
    const int m = k - be;
    if (m > 0) {
      const int T = (m + 15) >> 4, ntile = T * (T + 1) / 2, nb = be - b0;
      for (int t = wv; t < ntile; t += VNT / 64) {
        int I = 0;
        while ((I + 1) * (I + 2) / 2 <= t) ++I;
        const int J = t - I * (I + 1) / 2;
        const int ra = be + 16 * I + a16, cb = be + 16 * J + a16;
        d4 acc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = be + 16 * I + kq + 4 * r;
          acc[r] = (row < k && cb < k) ? G[row * ldg + cb] : 0.0;
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int kk = 4 * s + kq;
          const double va = (ra < k && kk < nb) ? -G[ra * ldg + b0 + kk] : 0.0;
          const double vb = (cb < k && kk < nb) ? G[cb * ldg + b0 + kk] : 0.0;
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(va, vb, acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = be + 16 * I + kq + 4 * r;
          if (row < k && cb < k && cb <= row) G[row * ldg + cb] = acc[r];
        }
      }
      __syncthreads();
    }
  }
  return true;
}

// One CholeskyQR pass over the k columns of Z (n x k, ld ldz; LDS or global):
// G = Z^T Z (lower triangle, ld ldg, LDS), G = L L^T (chol_wg), Z <- Z L^-T.
// The Gram matrix and the solve's block updates run on the matrix cores
// (v_mfma_f64_16x16x4f64: lane l holds A[l & 15][kk] and B[kk][l & 15],
// kk = k-step + (l >> 4); the result C[(l >> 4) + 4 r][l & 15]), four
// k-steps' loads in flight per wave; the solve goes by 16-column blocks b0:
// Z_B -= Z_{<B} L_{B,<B}^T (waves over 16-row tiles), then every row's
// 16 x 16 forward substitution against L_BB by one thread.  false (uniform):
// a collapsed pivot (Z untouched by this pass).  Caller: barrier before.
#ifdef HBM_STAMP
__device__ unsigned long long g_cq_st[4];  // gram, chol, block updates, row substitutions (block 0, thread 0)
#define CQ_STAMP(slot)                                                               \
  do {                                                                               \
    __builtin_amdgcn_sched_barrier(0);                                               \
    unsigned long long t_;                                                           \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");       \
    __builtin_amdgcn_sched_barrier(0);                                               \
    if (threadIdx.x == 0 && blockIdx.x == 0) g_cq_st[slot] += t_ - cq_last;          \
    cq_last = t_;                                                                    \
  } while (0)
#else
#define CQ_STAMP(slot) do {} while (0)
#endif
__device__ __forceinline__ bool cholqr_pass(double* Z, int ldz, int n, int k, double* G, int ldg) {
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int a16 = lane & 15, kq = lane >> 4;
#ifdef HBM_STAMP
  unsigned long long cq_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(cq_last)::"memory");
#endif
  {
    const int T = (k + 15) >> 4, ntile = T * (T + 1) / 2;
    for (int t = wv; t < ntile; t += VNT / 64) {
      int I = 0;
      while ((I + 1) * (I + 2) / 2 <= t) ++I;
      const int J = t - I * (I + 1) / 2;
      const int ca = 16 * I + a16, cb = 16 * J + a16;
      d4 acc = {0, 0, 0, 0};
      for (int k0 = 0; k0 < n; k0 += 16) {
        double va[4], vb[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int rr = k0 + 4 * s + kq;
          va[s] = (rr < n && ca < k) ? Z[(size_t)rr * ldz + ca] : 0.0;
          vb[s] = (rr < n && cb < k) ? Z[(size_t)rr * ldz + cb] : 0.0;
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(va[s], vb[s], acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * I + kq + 4 * r;
        if (row < k && cb < k && cb <= row) G[row * ldg + cb] = acc[r];
      }
    }
  }
  __syncthreads();
  CQ_STAMP(0);
  const bool ok = chol_wg(G, ldg, k);
  CQ_STAMP(1);
  if (!ok) return false;
  for (int b0 = 0; b0 < k; b0 += 16) {
    const int nb = k - b0 < 16 ? k - b0 : 16;
    if (b0 > 0) {
      for (int R = wv; 16 * R < n; R += VNT / 64) {
        const int ra = 16 * R + a16, cb = b0 + a16;
        d4 acc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * R + kq + 4 * r;
          acc[r] = (row < n && cb < k) ? Z[(size_t)row * ldz + cb] : 0.0;
        }
        for (int k0 = 0; k0 < b0; k0 += 16) {
          double va[4], vb[4];
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const int kk = k0 + 4 * s + kq;
            va[s] = ra < n ? -Z[(size_t)ra * ldz + kk] : 0.0;
            vb[s] = cb < k ? G[cb * ldg + kk] : 0.0;
          }
#pragma unroll
          for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(va[s], vb[s], acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * R + kq + 4 * r;
          if (row < n && cb < k) Z[(size_t)row * ldz + cb] = acc[r];
        }
      }
      __syncthreads();
    }
    CQ_STAMP(2);
    for (int rr = tid; rr < n; rr += VNT) {
      double* zr = Z + (size_t)rr * ldz + b0;
      double x[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) x[t] = t < nb ? zr[t] : 0.0;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        if (t < nb) {
#pragma unroll
          for (int s2 = 0; s2 < t; ++s2) x[t] = fma(-x[s2], G[(b0 + t) * ldg + b0 + s2], x[t]);
          x[t] = x[t] / G[(b0 + t) * ldg + b0 + t];
        }
      }
#pragma unroll
      for (int t = 0; t < 16; ++t)
        if (t < nb) zr[t] = x[t];
    }
    __syncthreads();
    CQ_STAMP(3);
  }
  return true;
}

__global__ __launch_bounds__(VNT) void k_heev_vecs_reg(const EProb* __restrict__ probs, int nprob) {
  __shared__ __align__(16) char un[kVecLds];
  __shared__ double Ld[RNMAX], Le[RNMAX], Lc[64];
  __shared__ z part[VNT / 64][64];
  __shared__ double red[VNT / 64];
  const EProb P = probs[blockIdx.x];
  const int n = P.n, tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  if (n <= 0) return;
  const int k = *P.kept;
  if (k <= 0) return;
  if (n == 1) {
    if (tid == 0) P.U[0] = mk(1, 0);
    return;
  }
  const int ldz = k + 1;  // odd stride: row reads of Z by consecutive threads hit distinct banks
  const bool fast = vecs_fast(n, k);
  double* Zl = (double*)un;
  // generic path: the tridiagonal in global memory scratch (P.d / P.e), Z and U global
  const double* Gd = P.d;
  const double* Ge = P.e;
  if (fast) {
    for (int i = tid; i < n; i += VNT) { Ld[i] = P.d[i]; Le[i] = P.e[i]; }
    __syncthreads();
    Gd = Ld;
    Ge = Le;
  }
  double tn = 0;
  for (int i = tid; i < n; i += VNT) tn = fmax(tn, fabs(Gd[i]) + Ge[i] + (i > 0 ? Ge[i - 1] : 0.0));
  for (int o = 32; o > 0; o >>= 1) tn = fmax(tn, __shfl_xor(tn, o, 64));
  if (lane == 0) red[wv] = tn;
  __syncthreads();
  tn = red[0];
  for (int q = 1; q < VNT / 64; ++q) tn = fmax(tn, red[q]);
  __syncthreads();
  const double tiny = 2.220446049250313e-16 * fmax(tn, 1e-300);
#ifdef HBM_STAMP
  unsigned long long stamp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, stamp_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(stamp_last)::"memory");
#endif
  double* Z = fast ? Zl : P.Z;
  const int lz = fast ? ldz : n;
  if (fast) {
    // pivots in the region's tail after Z: as many eigenvectors per batch as fit (all of them when k <= 64
    // and n (k + 1 + k) doubles fit)
    double* piv = Zl + (size_t)n * ldz;
    const int room = int((size_t(kVecLds) / 8 - (size_t)n * ldz) / size_t(n));
    const int batch = room < k ? (room < 1 ? 1 : room) : k;
    for (int jb = 0; jb < k; jb += batch) {
      const int jj = jb + tid;
      if (tid < batch && jj < k) invit_fast(Ld, Le, n, P.w[jj], tiny, Zl, ldz, jj, piv, batch, tid, jj);
    }
  } else {
    for (int jj = tid; jj < k; jj += VNT) invit_fast(Gd, Ge, n, P.w[jj], tiny, Z, lz, jj, P.Dv, n, jj, jj);
  }
  __syncthreads();
  STAMP(0);
  // Orthonormalise the k inverse-iteration vectors.  Fast path: CholeskyQR2
  // (G = Z^T Z over all threads, G = L L^T by one wave, Z <- Z L^-T row by
  // row, twice); a collapsed Cholesky pivot (nearly dependent vectors) falls
  // back to classical Gram-Schmidt, twice, which any path can take.
  bool need_gs = !fast || k > 64;
  if (!need_gs) {
    // Z in LDS (ld k + 1), G (ld 65) after it (the pivots are no longer needed)
    for (int pass = 0; pass < 2 && !need_gs; ++pass)
      if (!cholqr_pass(Zl, ldz, n, k, Zl + (size_t)n * ldz, 65)) need_gs = true;
  }
  if (need_gs && !fast && k <= 128 && n <= kBtRows) {
    // Z (ld n) in global memory, G (ld k + 1) fills the LDS region
    need_gs = false;
    for (int pass = 0; pass < 2 && !need_gs; ++pass)
      if (!cholqr_pass(Z, n, n, k, (double*)un, k + 1)) need_gs = true;
  }
  if (need_gs) {
    // classical Gram-Schmidt, twice, descending; dots split over 8 row chunks
    for (int j = 0; j < k; ++j) {
      for (int pass = 0; pass < 2 && j > 0; ++pass) {
        // part[ch][i] = sum_{r = ch mod 8} Z[r][i] Z[r][j]
        for (int i0 = 0; i0 < j; i0 += 64) {
          const int i = i0 + lane;
          double pa = 0;
          if (i < j)
            for (int rr = wv; rr < n; rr += VNT / 64) pa += Z[(size_t)rr * lz + i] * Z[(size_t)rr * lz + j];
          part[wv][lane].x = pa;
          __syncthreads();
          if (tid < 64 && i < j) {
            double sc = 0;
#pragma unroll
            for (int q = 0; q < VNT / 64; ++q) sc += part[q][tid].x;
            part[0][tid].y = sc;
          }
          __syncthreads();
          // Z[r][j] -= sum_{i in this chunk} c_i Z[r][i]
          for (int rr = tid; rr < n; rr += VNT) {
            double s = 0;
            const int ie = j - i0 < 64 ? j - i0 : 64;
            for (int q = 0; q < ie; ++q) s += part[0][q].y * Z[(size_t)rr * lz + i0 + q];
            Z[(size_t)rr * lz + j] -= s;
          }
          __syncthreads();
        }
      }
      double ss = 0;
      for (int rr = tid; rr < n; rr += VNT) { const double v = Z[(size_t)rr * lz + j]; ss += v * v; }
      ss = block_sum_r(ss, red);
      const double inv = ss > 0 ? 1.0 / sqrt(ss) : 0.0;
      for (int rr = tid; rr < n; rr += VNT) Z[(size_t)rr * lz + j] *= inv;
      __syncthreads();
    }
  }
  STAMP(1);
  if (!fast && n <= kBtRows) {  // U = Q D Z by k_heev_bt
#ifdef HBM_STAMP
    if (tid == 0 && blockIdx.x == 0) printf("vecs slow n=%d k=%d stamps: invit %llu orth %llu (gram %llu chol %llu blk %llu subst %llu) gs %d\n", n, k, stamp_acc[0], stamp_acc[1], g_cq_st[0], g_cq_st[1], g_cq_st[2], g_cq_st[3], int(need_gs));
#endif
    return;
  }
  if (!fast) {
    // U = Q D Z in global memory, reflectors j = n-2 .. 0 (one column per thread)
    z* U = P.U;
    for (int e = tid; e < n * k; e += VNT) {
      const int rr = e / k, cc = e - rr * k;
      U[e] = zsc(P.ph[rr], Z[(size_t)rr * lz + cc]);
    }
    __syncthreads();
    for (int j = n - 2; j >= 0; --j) {
      const double t = P.tau[j];
      if (t == 0.0) continue;
      const z* u = P.A + j;
      for (int cc = tid; cc < k; cc += VNT) {
        z s = mk(0, 0);
        for (int rr = j + 1; rr < n; ++rr) s = zadd(s, zcjmul(u[(size_t)rr * n], U[(size_t)rr * k + cc]));
        s = zsc(s, t);
        for (int rr = j + 1; rr < n; ++rr) U[(size_t)rr * k + cc] = zsub(U[(size_t)rr * k + cc], zmul(u[(size_t)rr * n], s));
      }
      __syncthreads();
    }
    STAMP(4);
#ifdef HBM_STAMP
    if (tid == 0)
      for (int q = 0; q < 8; ++q) P.Z[q] = double(stamp_acc[q]);
#endif
    return;
  }
  // ---- fast path: U in registers.  Lane l of wave w: row chunk rc = l >> 2
  // (rows i = 16 t + rc), column cc = l & 3 of the wave's column groups
  // g = w, w + 8 (columns 4 g + cc); a reflector's dot products reduce over
  // the 16 row chunks inside the wave, so reflectors need no barrier.
  constexpr int TR = (RNMAX + 15) / 16;  // rows per lane (13)
  constexpr int NG = 2;                  // column groups per wave (k <= 64)
  const int rc = lane >> 2, cc = lane & 3;
  z Ur[NG][TR];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int col = 4 * (wv + 8 * g) + cc;
#pragma unroll
    for (int t = 0; t < TR; ++t) {
      const int i = 16 * t + rc;
      Ur[g][t] = (i < n && col < k) ? zsc(P.ph[i], Zl[(size_t)i * ldz + col]) : mk(0, 0);
    }
  }
  const bool g0 = 4 * wv < k, g1 = 4 * (wv + 8) < k;  // wave-uniform
  __syncthreads();  // Z no longer needed: the region now holds reflector blocks
  STAMP(2);
  z* Rb = (z*)un;   // [kRefBlk][RNMAX]: reflector jj of the block, rows 0..n-1 (zero at rows <= j)
  __shared__ double stau[kRefBlk];
  for (int jhi = n - 2; jhi >= 0; jhi -= kRefBlk) {
    const int jlo = jhi - kRefBlk + 1 > 0 ? jhi - kRefBlk + 1 : 0;
    const int nb = jhi - jlo + 1;
    __syncthreads();  // previous block consumed
    for (int e = tid; e < nb * n; e += VNT) {
      const int rr = e / nb, jj = e - rr * nb, j = jlo + jj;
      Rb[jj * RNMAX + rr] = rr > j ? P.A[(size_t)rr * n + j] : mk(0, 0);
    }
    for (int jj = tid; jj < nb; jj += VNT) stau[jj] = P.tau[jlo + jj];
    __syncthreads();
    STAMP(3);
    if (!g0) continue;
    for (int j = jhi; j >= jlo; --j) {
      const double t = stau[j - jlo];
      if (t == 0.0) continue;  // uniform
      const z* u = Rb + (j - jlo) * RNMAX;
      const int t0 = (j + 1) >> 4;  // first row slot holding rows > j (uniform)
      z uu[TR];
#pragma unroll
      for (int tt = 0; tt < TR; ++tt) uu[tt] = (tt >= t0 && 16 * tt + rc < n) ? u[16 * tt + rc] : mk(0, 0);
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        if (g == 1 && !g1) continue;
        z sacc = mk(0, 0);
#pragma unroll
        for (int tt = 0; tt < TR; ++tt) {
          if (tt < t0) continue;
          sacc.x = fma(uu[tt].x, Ur[g][tt].x, fma(uu[tt].y, Ur[g][tt].y, sacc.x));  // conj(u) U
          sacc.y = fma(uu[tt].x, Ur[g][tt].y, fma(-uu[tt].y, Ur[g][tt].x, sacc.y));
        }
#pragma unroll
        for (int o = 4; o < 64; o <<= 1) {
          sacc.x += __shfl_xor(sacc.x, o, 64);
          sacc.y += __shfl_xor(sacc.y, o, 64);
        }
        sacc = zsc(sacc, t);
#pragma unroll
        for (int tt = 0; tt < TR; ++tt) {
          if (tt < t0) continue;
          Ur[g][tt].x = fma(-uu[tt].x, sacc.x, fma(uu[tt].y, sacc.y, Ur[g][tt].x));
          Ur[g][tt].y = fma(-uu[tt].x, sacc.y, fma(-uu[tt].y, sacc.x, Ur[g][tt].y));
        }
      }
    }
    STAMP(4);
  }
#ifdef HBM_STAMP
  if (tid == 0)
    for (int q = 0; q < 8; ++q) P.Z[q] = double(stamp_acc[q]);
#endif
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int col = 4 * (wv + 8 * g) + cc;
    if (col >= k) continue;
#pragma unroll
    for (int t = 0; t < TR; ++t) {
      const int i = 16 * t + rc;
      if (i < n) P.U[(size_t)i * k + col] = Ur[g][t];
    }
  }
}

// ------------------------------------------------------------------ back-transformation
// U = Q D Z for the problems the vecs kernel left in global memory (order
// kBtRows at most, not vecs_fast): one workgroup per (problem, block of 16
// kept columns).  Lane l of wave w holds column 16 cb + 4 w + (l & 3), rows
// i = 16 t + (l >> 2) (t < 32) in registers; the reflectors j = n-2 .. 0 are
// staged through LDS kBtBlk at a time and applied with in-wave reductions over
// the 16 row chunks, as in the vecs kernel's fast path.  tasks: (problem,
// column block); blocks past the problem's kept count exit at once.
__global__ __launch_bounds__(BNT) void k_heev_bt(const EProb* __restrict__ probs, const int2* __restrict__ tasks) {
  __shared__ z Rb[kBtBlk * kBtRows];
  __shared__ double stau[kBtBlk];
  const int2 tk = tasks[blockIdx.x];
  const EProb P = probs[tk.x];
  const int n = P.n;
  if (n <= 1 || n > kBtRows) return;
  const int k = *P.kept;
  if (k <= 0 || vecs_fast(n, k)) return;
  const int c0 = 16 * tk.y;
  if (c0 >= k) return;  // workgroup-uniform
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int rc = lane >> 2, col = c0 + 4 * wv + (lane & 3);
  const bool wave_live = c0 + 4 * wv < k;  // wave-uniform
  constexpr int TR = kBtRows / 16;
  z Ur[TR];
#pragma unroll
  for (int t = 0; t < TR; ++t) {
    const int i = 16 * t + rc;
    Ur[t] = (i < n && col < k) ? zsc(P.ph[i], P.Z[(size_t)i * n + col]) : mk(0, 0);
  }
  for (int jhi = n - 2; jhi >= 0; jhi -= kBtBlk) {
    const int jlo = jhi - kBtBlk + 1 > 0 ? jhi - kBtBlk + 1 : 0;
    const int nb = jhi - jlo + 1;
    __syncthreads();  // previous block consumed
    for (int e = tid; e < nb * n; e += BNT) {
      const int rr = e / nb, jj = e - rr * nb, j = jlo + jj;
      Rb[jj * kBtRows + rr] = rr > j ? P.A[(size_t)rr * n + j] : mk(0, 0);
    }
    for (int jj = tid; jj < nb; jj += BNT) stau[jj] = P.tau[jlo + jj];
    __syncthreads();
    if (!wave_live) continue;
    for (int j = jhi; j >= jlo; --j) {
      const double t = stau[j - jlo];
      if (t == 0.0) continue;  // uniform
      const z* u = Rb + (j - jlo) * kBtRows;
      const int t0 = (j + 1) >> 4;  // first row slot holding rows > j (uniform)
      z uu[TR];
#pragma unroll
      for (int tt = 0; tt < TR; ++tt) uu[tt] = (tt >= t0 && 16 * tt + rc < n) ? u[16 * tt + rc] : mk(0, 0);
      z sacc = mk(0, 0);
#pragma unroll
      for (int tt = 0; tt < TR; ++tt) {
        if (tt < t0) continue;
        sacc.x = fma(uu[tt].x, Ur[tt].x, fma(uu[tt].y, Ur[tt].y, sacc.x));  // conj(u) U
        sacc.y = fma(uu[tt].x, Ur[tt].y, fma(-uu[tt].y, Ur[tt].x, sacc.y));
      }
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) {
        sacc.x += __shfl_xor(sacc.x, o, 64);
        sacc.y += __shfl_xor(sacc.y, o, 64);
      }
      sacc = zsc(sacc, t);
#pragma unroll
      for (int tt = 0; tt < TR; ++tt) {
        if (tt < t0) continue;
        Ur[tt].x = fma(-uu[tt].x, sacc.x, fma(uu[tt].y, sacc.y, Ur[tt].x));
        Ur[tt].y = fma(-uu[tt].x, sacc.y, fma(-uu[tt].y, sacc.x, Ur[tt].y));
      }
    }
  }
  if (col >= k) return;
#pragma unroll
  for (int t = 0; t < TR; ++t) {
    const int i = 16 * t + rc;
    if (i < n) P.U[(size_t)i * k + col] = Ur[t];
  }
}

// ------------------------------------------------------------------ large orders
// Eigenvalues of Gram blocks of order RNMAX < n <= kBigMax (config 5's sectors
// at chi = 512): the lower triangle no longer fits one CU's registers, and the
// eager L2 reduction (tridiag) reads and writes the trailing matrix three times
// per column.  Here the reduction is blocked like LAPACK's zhetrd / zlatrd:
// inside a panel of BNB columns the stored trailing matrix stays stale and its
// pending updates are carried by the panel vectors (A_j = A - U W^H - W U^H):
// thread r keeps row r of U and W in registers, so the pending updates of the
// column being reduced and of the matrix-vector product cost no memory
// traffic; one rank-2 BNB update of the trailing block (rows staged through
// the problem's Z / Dv scratch and LDS) closes the panel.  Per column the
// trailing matrix is read once (the product, 64 columns per wave, split over
// up to 8 row chunks).  Same reflector conventions as tridiag (vector j in
// column j of A, u[j+1] = u0, tau real), so the vecs / back-transformation
// kernels follow unchanged; all reductions in a fixed order.
// wave64 sum of a double: DPP within rows of 16 (xor 1, xor 2, half mirror,
// mirror), then the four row sums by readlane; fixed order, every lane the same
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, int(b), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, int(b >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double((long long)(unsigned)lo | ((long long)hi << 32));
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane(int(b), l), hi = __builtin_amdgcn_readlane(int(b >> 32), l);
  return __longlong_as_double((long long)(unsigned)lo | ((long long)hi << 32));
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);  // row_half_mirror
  v += dpp_f64<0x140>(v);  // row_mirror
  return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}
constexpr int VBG = 512;
constexpr int kBigMax = VBG;  // one row per thread
constexpr int BNB = 12;
__device__ __forceinline__ void vals_big_body(const EProb& P) {
  constexpr int NWV = VBG / 64;
  __shared__ z LU[kBigMax], LP[kBigMax], LB[kBigMax];
  __shared__ double Ld[kBigMax], Le2[kBigMax];
  __shared__ z rowU[BNB], rowW[BNB], dots[2 * BNB], dpart[NWV][2 * BNB];
  __shared__ double red[NWV], scal[4];
  __shared__ __align__(16) z ws[8 * kBigMax];  // product partials [8][kBigMax] | panel staging [4][64][BNB]
  static_assert(4 * 64 * BNB <= 8 * kBigMax, "panel staging fits the partials region");
  const int n = P.n, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (n < 2 || n > kBigMax) return;
  z* A = P.A;
  z* U = reinterpret_cast<z*>(P.Z);  // n x BNB (ld BNB): panel rows for the closing update
  z* W = reinterpret_cast<z*>(P.Dv);
  const int r = tid;  // this thread's row
  z pu[BNB], pw[BNB];  // row r of the panel's U and W
#ifdef HBM_STAMP
  unsigned long long stamp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, stamp_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(stamp_last)::"memory");
#endif
  auto bsum = [&](double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if (lane == 0) red[wv] = v;
    __syncthreads();
    double s = 0;
#pragma unroll
    for (int i = 0; i < NWV; ++i) s += red[i];
    return s;
  };
  for (int p0 = 0; p0 < n - 1; p0 += BNB) {
    const int pe = p0 + BNB < n - 1 ? p0 + BNB : n - 1;
#pragma unroll
    for (int q = 0; q < BNB; ++q) { pu[q] = mk(0, 0); pw[q] = mk(0, 0); }
    for (int j = p0; j < pe; ++j) {
      const int l = j - p0, m = n - j - 1;
      if (r == j) {
#pragma unroll
        for (int q = 0; q < BNB; ++q) { rowU[q] = pu[q]; rowW[q] = pw[q]; }
      }
      __syncthreads();
      // column j (rows j..n-1) with the panel's pending updates
      if (r >= j && r < n) {
        z x = A[(size_t)r * n + j];
#pragma unroll
        for (int q = 0; q < BNB; ++q)  // slots q >= l hold zeros: exact no-ops, no branches
          x = zsub(x, zadd(zmul(pu[q], zcj(rowW[q])), zmul(pw[q], zcj(rowU[q]))));
        if (r == j) Ld[j] = x.x;
        else LU[r - j - 1] = x;
      }
      __syncthreads();
      STAMP(0);
      // reflector H = I - t u u^H zeroing x[1..m)
      double s = 0;
      for (int i = 1 + tid; i < m; i += VBG) s += LU[i].x * LU[i].x + LU[i].y * LU[i].y;
      s = bsum(s);
      if (tid == 0) {
        const z a = LU[0];
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
        P.tau[j] = t;
        LB[j] = b;
        scal[0] = t;
        scal[1] = u0.x;
        scal[2] = u0.y;
      }
      __syncthreads();
      const double t = scal[0];
      if (t == 0.0) continue;  // column already reduced: H = I, panel slot l stays zero
      if (tid == 0) LU[0] = mk(scal[1], scal[2]);
      __syncthreads();
      STAMP(1);
      const bool mine = r > j && r < n;  // this thread's row is in the trailing block
      const z ur = mine ? LU[r - j - 1] : mk(0, 0);
      if (mine) A[(size_t)r * n + j] = ur;  // reflector j in column j
      // p = A_t u on the stored (panel-stale) trailing matrix: wave (ib, kc)
      // sums rows of chunk kc for columns 64 ib + lane; p_i = sum_k conj(A[k][i]) u_k
      const int nib = (m + 63) >> 6;
      const int kch = NWV / nib < 1 ? 1 : NWV / nib;
      for (int task = wv; task < nib * kch; task += NWV) {
        const int ib = task % nib, kc = task / nib;
        const int i = 64 * ib + lane;
        if (i < m) {
          const int klen = (m + kch - 1) / kch, k0 = kc * klen, k1 = k0 + klen < m ? k0 + klen : m;
          const z* col = A + (size_t)(j + 1) * n + (j + 1) + i;
          z acc = mk(0, 0);
          int k = k0;
          for (; k + 7 < k1; k += 8) {
            z av[8];
#pragma unroll
            for (int tt = 0; tt < 8; ++tt) av[tt] = col[(size_t)(k + tt) * n];
#pragma unroll
            for (int tt = 0; tt < 8; ++tt) {
              const z uk = LU[k + tt];
              acc.x += av[tt].x * uk.x + av[tt].y * uk.y;
              acc.y += av[tt].x * uk.y - av[tt].y * uk.x;
            }
          }
          for (; k < k1; ++k) {
            const z av = col[(size_t)k * n], uk = LU[k];
            acc.x += av.x * uk.x + av.y * uk.y;
            acc.y += av.x * uk.y - av.y * uk.x;
          }
          ws[kc * kBigMax + i] = acc;
        }
      }
      STAMP(2);
      // panel dots: dots[q] = W_q^H u, dots[BNB + q] = U_q^H u (rows j+1..n-1; zero rows elsewhere)
      {
        // the l filled slots: wave sums by DPP + readlane, no LDS traffic
#pragma unroll
        for (int q = 0; q < BNB; ++q) {
          if (q >= l) continue;  // uniform
          const z a = zcjmul(pw[q], ur), b = zcjmul(pu[q], ur);
          const double ax = wave_sum_dpp(a.x), ay = wave_sum_dpp(a.y);
          const double bx = wave_sum_dpp(b.x), by = wave_sum_dpp(b.y);
          if (lane == 0) {
            dpart[wv][q] = mk(ax, ay);
            dpart[wv][BNB + q] = mk(bx, by);
          }
        }
      }
      __syncthreads();
      if (tid < 2 * BNB) {
        z a = mk(0, 0);
        if ((tid < BNB ? tid : tid - BNB) < l)
#pragma unroll
          for (int w = 0; w < NWV; ++w) a = zadd(a, dpart[w][tid]);
        dots[tid] = a;  // slots past l: zero
      }
      __syncthreads();
      STAMP(3);
      // p = t (A u - U (W^H u) - W (U^H u));  K = t/2 Re(u^H p);  w = p - K u
      double kk = 0;
      z p = mk(0, 0);
      if (mine) {
        const int i = r - j - 1;
        p = ws[i];
        for (int c = 1; c < kch; ++c) p = zadd(p, ws[c * kBigMax + i]);
#pragma unroll
        for (int q = 0; q < BNB; ++q) p = zsub(p, zadd(zmul(pu[q], dots[q]), zmul(pw[q], dots[BNB + q])));
        p = zsc(p, t);
        kk = ur.x * p.x + ur.y * p.y;
      }
      kk = 0.5 * t * bsum(kk);
      const z wr = zsub(p, zsc(ur, kk));
#pragma unroll
      for (int q = 0; q < BNB; ++q)
        if (q == l && mine) { pu[q] = ur; pw[q] = wr; }
      // (the next step's first barrier orders the ws / LU reuse)
      STAMP(4);
    }
    // close the panel: A[pe.., pe..] -= U W^H + W U^H (64 x 64 tiles, panel rows staged in LDS)
    const int nl = pe - p0, mt = n - pe;
    if (r >= pe && r < n) {
#pragma unroll
      for (int q = 0; q < BNB; ++q) { U[(size_t)r * BNB + q] = pu[q]; W[(size_t)r * BNB + q] = pw[q]; }
    }
    z* S = ws;  // [4][64][BNB]: U rows r, W rows r, U rows c, W rows c
    // C -= [U_r W_r] [W_c U_c]^H on v_mfma_f64_16x16x4f64 (K = 2 BNB, zero-padded past nl):
    // wave w owns the 16 x 16 tiles (w >> 1, 2 (w & 1) + {0, 1}) of the 64 x 64 block
    const int tr = wv >> 1, tc0 = 2 * (wv & 1), ml = lane & 15, kl = lane >> 4;
    for (int r0 = 0; r0 < mt; r0 += 64)
      for (int c0 = 0; c0 < mt; c0 += 64) {
        __syncthreads();
        for (int e = tid; e < 4 * 64 * BNB; e += VBG) {
          const int which = e / (64 * BNB), rem = e - which * (64 * BNB), row_l = rem / BNB, q = rem - row_l * BNB;
          const int row = pe + (which < 2 ? r0 : c0) + row_l;
          S[e] = (q < nl && row < n) ? ((which & 1) ? W : U)[(size_t)row * BNB + q] : mk(0, 0);
        }
        __syncthreads();
        if (r0 + 16 * tr >= mt) continue;  // wave-uniform: tile rows past the block
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int tc = tc0 + h;
          if (c0 + 16 * tc >= mt) continue;  // wave-uniform
          d4 cr = {0, 0, 0, 0}, ci = {0, 0, 0, 0};
#pragma unroll
          for (int ks = 0; ks < 2 * BNB / 4; ++ks) {
            const int kap = 4 * ks + kl;  // this lane's k
            const int rowA = 16 * tr + ml, colB = 16 * tc + ml;
            const z av = kap < BNB ? S[rowA * BNB + kap] : S[(64 + rowA) * BNB + kap - BNB];
            const z bw = kap < BNB ? S[(192 + colB) * BNB + kap] : S[(128 + colB) * BNB + kap - BNB];
            const double bx = bw.x, by = -bw.y;  // B = conj(.)
            cr = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bx, cr, 0, 0, 0);
            cr = __builtin_amdgcn_mfma_f64_16x16x4f64(-av.y, by, cr, 0, 0, 0);
            ci = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, by, ci, 0, 0, 0);
            ci = __builtin_amdgcn_mfma_f64_16x16x4f64(av.y, bx, ci, 0, 0, 0);
          }
          const int c = pe + c0 + 16 * tc + ml;
          if (c < n) {
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
              const int rg = pe + r0 + 16 * tr + kl + 4 * rr;
              if (rg < n) {
                z* ap = A + (size_t)rg * n + c;
                const z v = *ap;
                *ap = mk(v.x - cr[rr], v.y - ci[rr]);
              }
            }
          }
        }
      }
    __syncthreads();
    STAMP(5);
  }
  if (tid == 0) Ld[n - 1] = A[(size_t)(n - 1) * n + (n - 1)].x;
  __syncthreads();
  // real tridiagonal (phases P.ph, d, e) and the eigenvalues by multisection,
  // unresolved below thr_rel * trace like the register kernels
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
  for (int j = tid; j < n; j += VBG) P.d[j] = Ld[j];
  __syncthreads();
  double* lo = reinterpret_cast<double*>(ws);
  double* hi = lo + kBigMax;
  int* cnt = reinterpret_cast<int*>(hi + kBigMax);
  bisect_all<VBG>(Ld, Le2, n, P.thr_rel, P.w, lo, hi, cnt, P.ks);
#ifdef HBM_STAMP
  __syncthreads();
  STAMP(6);
  if (tid == 0 && blockIdx.x == 0)
    printf("vals_big n=%d stamps: column %llu reflector %llu product %llu dots %llu p/w %llu panel %llu bisect %llu\n", n,
           stamp_acc[0], stamp_acc[1], stamp_acc[2], stamp_acc[3], stamp_acc[4], stamp_acc[5], stamp_acc[6]);
#endif
}
__global__ __launch_bounds__(VBG) void k_heev_vals_big(const EProb* __restrict__ probs, const int* __restrict__ idx) {
  vals_big_body(probs[idx[blockIdx.x]]);
}

}  // namespace hbm

#include "hbm_coop.hpp"
