// Multi-CU Hermitian eigenvalue stage of the HBM engine: one Gram block of
// order 64 < n <= 512 (by default the orders 209-512 the one-CU register
// kernels cannot hold: config 5's sectors at chi = 512) reduced by a GROUP of
// G workgroups on G CUs.
//
// The reference's truncation (ITensor denmatDecomp, src/BH_tDMRG.cpp:178,
// 191,209) diagonalises rho = Θ Θ^H per U(1) sector.  On one CU
// (k_heev_vals_any's register grids, k_heev_vals_big's blocked reduction) a
// block of order 512 takes ~19 ms: every Householder column reads the
// trailing matrix once (one CU's L2 bandwidth), every panel closes with a
// rank-2 BNB update of it, and all eigenvalues are bisected by 512 threads.
// Here the same blocked (zhetrd / zlatrd) reduction runs on G CUs:
//
//  * ownership: 16-column blocks of the trailing matrix are dealt
//    round-robin (block cb -> member cb mod G).  A member computes
//    p_i = (A u)_i for its own columns (rows in fixed 32-row chunks, the
//    chunks summed in order) and applies the panel's closing update to its
//    own columns; the matrix after the first panel lives in P.U (the
//    original block in P.A is never overwritten above the diagonal);
//  * everything else is computed redundantly, bit-identically, by every
//    member (thread r holds row r of the panel vectors U, W in registers):
//    the column with its pending panel updates, the reflector, the dots
//    W^H u / U^H u, w = p - K u.  Per column there is ONE exchange: the
//    members' slices of A u (and their u^H A u partials per column block)
//    through P.Dv, plus one per panel: the next panel's BNB columns through
//    P.Z;
//  * the exchange is the sc1 hand-off of MI355X_MICROARCH.md (§Workgroup
//    dispatch ..., table row 1): payload stored with agent-scope relaxed
//    atomics (global_store sc1) -> s_waitcnt vmcnt(0) -> workgroup barrier ->
//    one lane adds to the group's counter (agent-scope atomic); the consumer's
//    one lane polls the counter with sc1 loads -> workgroup barrier -> every
//    payload load is an sc1 load.  Counters and payload slots are double
//    buffered by column parity;
//  * every result is independent of G: each p_i, each u^H A u block partial
//    and each eigenvalue is computed by one member in an order fixed by
//    (n, column) alone, so the host may pick G per launch (CUs free) and
//    batched / pipelined / checkpointed runs still agree bit for bit;
//  * eigenvalues by multisection with 4 interior points per round (the
//    brackets depend only on the tridiagonal), the resolved eigenvalues
//    split into G contiguous ranges;
//  * progress: the members of a group are placed on one XCD (blocks b and
//    b + 8 share one, MI355X_MICROARCH.md) at consecutive positions of its
//    dispatch order; every wait is bounded (tmo, s_memrealtime ticks) and a
//    member that gives up raises the group's abort word, every member then
//    leaves, and k_heev_vals_coop_fix re-runs that block on one CU
//    (vals_big_body) after restoring its lower triangle from the untouched
//    upper one.
//
// Output conventions are those of tridiag / k_heev_vals_big (reflector j in
// column j of P.A, tau, real tridiagonal d / e with phases ph, eigenvalues
// descending in P.w, unresolved ones below thr_rel * trace set to their
// mean), so k_heev_vecs_reg / k_heev_bt follow unchanged.
#pragma once

namespace hbm {

constexpr int CPT = 512;      // threads per member: one row per thread, n <= CPT
constexpr int CNB = 12;       // panel width
constexpr int CMB = 8;        // own 16-column blocks per matvec pass
constexpr int kCoopCtl = 64;  // ints of control words per group: counter at 0, abort word at 32
constexpr int kCoopMaxG = 16;
#ifndef COOP_MV_UNROLL
#define COOP_MV_UNROLL 1  // 8-row load batches of a chunk unrolled (each batch one L2 round trip)
#endif
#ifndef COOP_MODEA_MIN
#define COOP_MODEA_MIN 24  // own 16-column blocks from which each wave sums whole column groups itself
#endif

// global-address-space views: the hand-off's loads and stores must be
// global_ (not flat_) sc1 instructions (MI355X_MICROARCH.md, Consumer bullet)
typedef __attribute__((address_space(1))) double gdouble;
typedef double dv2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) dv2 gdv2;
__device__ __forceinline__ gdouble* gd(const double* p) { return (gdouble*)(p); }
__device__ __forceinline__ double ldd_sc1(const double* p) {
  return __hip_atomic_load(gd(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ z ldz_sc1(const z* p) {
  const double* d = reinterpret_cast<const double*>(p);
  return mk(ldd_sc1(d), ldd_sc1(d + 1));
}
__device__ __forceinline__ void std_sc1(double* p, double v) {
  __hip_atomic_store(gd(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stz_sc1(z* p, z v) {
  double* d = reinterpret_cast<double*>(p);
  std_sc1(d, v.x);
  std_sc1(d + 1, v.y);
}
// plain global load / store of a complex
__device__ __forceinline__ z ldz_g(const z* p) {
  const dv2 v = *(const gdv2*)(p);
  return mk(v.x, v.y);
}
__device__ __forceinline__ void stz_g(z* p, z v) {
  dv2 w;
  w.x = v.x;
  w.y = v.y;
  *(gdv2*)(p) = w;
}
__device__ __forceinline__ z shfl_z(z v, int o) { return mk(__shfl_xor(v.x, o, 64), __shfl_xor(v.y, o, 64)); }

// the group's hand-off: every storing wave drains its sc1 stores, then one
// lane adds to the counter (caller: all threads)
__device__ __forceinline__ void coop_signal(int* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one lane polls until the counter reaches target (sc1 loads), then a
// workgroup barrier; false (uniform) when the group gave up
__device__ __forceinline__ bool coop_wait(int* cnt, int* abt, int target, long long tmo, int* sflag) {
  if (threadIdx.x == 0) {
    int bad = 0;
    if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      const long long t0 = wall_clock64();
      while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (__hip_atomic_load(abt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) { bad = 1; break; }
        if (wall_clock64() - t0 > tmo) {
          __hip_atomic_store(abt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          bad = 1;
          break;
        }
      }
    }
    *sflag = bad;
  }
  __syncthreads();
  return *sflag == 0;
}

// Sturm count of one shift (the loads of four steps ahead of the chain)
__device__ __forceinline__ int sturm_count1(const double* d, const double* e2, int n, double x, double pivmin) {
  double q = d[0] - x;
  if (fabs(q) < pivmin) q = -pivmin;
  int c = q < 0 ? 1 : 0;
  int i = 1;
  for (; i + 3 < n; i += 4) {
    double dv[4], ev[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { dv[u] = d[i + u]; ev[u] = e2[i + u - 1]; }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      q = sturm_next(dv[u] - x, ev[u], q);
      if (fabs(q) < pivmin) q = -pivmin;
      c += q < 0 ? 1 : 0;
    }
  }
  for (; i < n; ++i) {
    q = sturm_next(d[i] - x, e2[i - 1], q);
    if (fabs(q) < pivmin) q = -pivmin;
    c += q < 0 ? 1 : 0;
  }
  return c;
}

// cross-lane moves of a double without LDS: DPP within rows of 16 lanes, the
// gfx950 permlane swaps across rows / halves
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, int(b), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, int(b >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double((long long)(unsigned)lo | ((long long)hi << 32));
}
__device__ __forceinline__ double join_d(unsigned lo, unsigned hi) {
  return __longlong_as_double((long long)lo | ((long long)hi << 32));
}
// a' = [a lanes 0-31 | b lanes 0-31], b' = [a lanes 32-63 | b lanes 32-63]:
// lane L < 32 sees (a[L], a[L + 32]), lane L >= 32 sees (b[L - 32], b[L])
__device__ __forceinline__ void swap32(double& a, double& b) {
#ifdef COOP_DBG_NOSWAP
  { const double pa = __shfl_xor(a, 32, 64), pb = __shfl_xor(b, 32, 64); const bool up = (threadIdx.x & 32) != 0; const double na = up ? pb : a, nb = up ? b : pa; a = na; b = nb; return; }
#endif
  const long long ia = __double_as_longlong(a), ib = __double_as_longlong(b);
  const auto lo = __builtin_amdgcn_permlane32_swap(unsigned(ia), unsigned(ib), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(unsigned(ia >> 32), unsigned(ib >> 32), false, false);
  a = join_d(lo[0], hi[0]);
  b = join_d(lo[1], hi[1]);
}
// the same between rows 0/1 and 2/3 (lane L and L ^ 16)
__device__ __forceinline__ void swap16(double& a, double& b) {
#ifdef COOP_DBG_NOSWAP
  { const double pa = __shfl_xor(a, 16, 64), pb = __shfl_xor(b, 16, 64); const bool up = (threadIdx.x & 16) != 0; const double na = up ? pb : a, nb = up ? b : pa; a = na; b = nb; return; }
#endif
  const long long ia = __double_as_longlong(a), ib = __double_as_longlong(b);
  const auto lo = __builtin_amdgcn_permlane16_swap(unsigned(ia), unsigned(ib), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(unsigned(ia >> 32), unsigned(ib >> 32), false, false);
  a = join_d(lo[0], hi[0]);
  b = join_d(lo[1], hi[1]);
}
// wave sum, the same bits in every lane (every pairwise step is commutative)
__device__ __forceinline__ double wave_allsum(double v) {
  v += dpp_d<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_d<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_d<0x141>(v);  // row_half_mirror
  v += dpp_d<0x140>(v);  // row_mirror: the row's sum in its 16 lanes
  double a = v, b = v;
  swap16(a, b);
  v = a + b;
  a = v;
  b = v;
  swap32(a, b);
  return a + b;
}
// reduce-scatter step: lanes with the step's bit clear keep the sum of value
// lo, the others of value hi (each lane adds its partner's)
__device__ __forceinline__ double rs32(double lo, double hi) {
  swap32(lo, hi);
  return lo + hi;
}
__device__ __forceinline__ double rs16(double lo, double hi) {
  swap16(lo, hi);
  return lo + hi;
}
__device__ __forceinline__ double rs8(double lo, double hi, int lane) {
  const bool up = (lane & 8) != 0;
  const double keep = up ? hi : lo, send = up ? lo : hi;
  return keep + dpp_d<0x128>(send);  // row_ror:8 = lane ^ 8 within the row
}
// sum over the 8 lanes of a half-row, the same bits in all 8
__device__ __forceinline__ double sum8(double v) {
  v += dpp_d<0xB1>(v);
  v += dpp_d<0x4E>(v);
  v += dpp_d<0x141>(v);
  return v;
}

// conj(A[k][col]) u_k summed over the 32 rows of chunk c in row order (explicit
// fma: the same bits wherever it is called; rows <= j and invalid columns are
// zeros).  Loads in batches of 8 (one L2 round trip each).
// Branch-free: every lane loads a valid (clamped) address and the rows or
// columns outside the trailing block are selected to zero afterwards (an
// exec-masked load per element cost ~15 instructions of mask bookkeeping).
__device__ __forceinline__ z zsel0(bool keep, z v) { return mk(keep ? v.x : 0.0, keep ? v.y : 0.0); }
typedef unsigned u4v __attribute__((ext_vector_type(4)));
// buffer resource over an n x n complex block: 32-bit offsets, and loads past
// its end return zeros (rows >= n)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t zblock_rsrc(const z* S, int n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<z*>(S), (short)0, unsigned(n) * unsigned(n) * 16u, 0x00020000);
}
__device__ __forceinline__ z ldz_buf(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const u4v v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return mk(__builtin_bit_cast(double, (unsigned long long)v.x | ((unsigned long long)v.y << 32)),
            __builtin_bit_cast(double, (unsigned long long)v.z | ((unsigned long long)v.w << 32)));
}
__device__ __forceinline__ z chunk_acc(const z* __restrict__ S, int n, int col, bool cok, int j, int c, z u0,
                                       const z* LU) {
  z acc = mk(0, 0);
  const __amdgpu_buffer_rsrc_t rs = zblock_rsrc(S, n);
  const unsigned cb = 16u * unsigned(col < n ? col : n - 1), rb = 16u * unsigned(n);
#pragma unroll COOP_MV_UNROLL
  for (int hh = 0; hh < 4; ++hh) {
    z av[8];
    const unsigned k0 = unsigned(32 * c + 8 * hh);
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) av[s8] = ldz_buf(rs, cb + (k0 + s8) * rb);
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) {
      const int k = 32 * c + 8 * hh + s8;
      av[s8] = zsel0(cok && k > j && k < n, av[s8]);
      const z lk = LU[k];
      const z uk = k == j + 1 ? u0 : lk;
      acc.x = fma(av[s8].x, uk.x, fma(av[s8].y, uk.y, acc.x));
      acc.y = fma(av[s8].x, uk.y, fma(-av[s8].y, uk.x, acc.y));
    }
  }
  return acc;
}

// grid: 8 * G * ceil(ngroup / 8) workgroups of CPT threads; block b is member
// (b >> 3) % G of group 8 ((b >> 3) / G) + (b & 7).  ctl: kCoopCtl zeroed ints
// per group.  probs[idx[g]]: the block of group g (64 < n <= CPT).
__global__ __launch_bounds__(CPT, 1) void k_heev_vals_coop(const EProb* __restrict__ probs,
                                                           const int* __restrict__ idx, int ngroup, int G,
                                                           int* __restrict__ ctl, long long tmo) {
  // XCD-local groups: members at consecutive dispatch positions of one XCD
  // (blocks b, b + 8, ...), which measured ~3 % faster than spreading a group
  // over the XCDs (gi = b / G)
  const int bid = blockIdx.x, slot = bid >> 3, gi = (slot / G) * 8 + (bid & 7), me = slot - (slot / G) * G;
  if (gi >= ngroup) return;
  const EProb P = probs[idx[gi]];
  const int n = P.n, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (n < 2 || n > CPT) return;
  int* cnt = ctl + kCoopCtl * gi;
  int* abt = cnt + 32;
  z* A0 = P.A;                                   // the block (upper triangle never written)
  z* Ab = P.U;                                   // trailing matrix after the first panel (ld n)
  z* xc = reinterpret_cast<z*>(P.Z);             // [2][CNB][n]: the next panel's columns
  z* pb = reinterpret_cast<z*>(P.Dv);            // [2][n]: A u of the column being reduced
  z* bp = pb + 2 * n;                            // [2][32]: u^H A u per own 16-column block

  __shared__ z LU[CPT];
  __shared__ double Ld[CPT], Le2[CPT], Ltau[CPT];
  __shared__ z LB[CPT];
  __shared__ z Nx[2][2][CNB];     // [parity of the row][U / W][q]: row j+1's panel entries
  __shared__ z X1;                // x_{j+1}
  __shared__ double red1[8];
  __shared__ double red2[8][48];
  __shared__ double fin[48];
  __shared__ int sflag;
  __shared__ __align__(16) z ws[4 * 64 * CNB];  // matvec partials [chunks][CMB * 16] | panel staging [4][64][CNB]
  static_assert((CPT / 32) * CMB * 16 <= 4 * 64 * CNB, "matvec partials fit the staging region");

  const int r = tid;
  if (tid < 4 * CNB) (&Nx[0][0][0])[tid] = mk(0, 0);
  __syncthreads();
  z pu[CNB], pw[CNB];
  z ru = mk(0, 0), rw = mk(0, 0);  // row j's panel slot l - 1 (computed by every thread)
#ifdef HBM_STAMP
  unsigned long long stamp_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, stamp_last;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(stamp_last)::"memory");
#endif
  int hop = 0;
  int panel = 0;
  const int nblk = (n + 15) >> 4;
  for (int p0 = 0; p0 < n - 1; p0 += CNB, ++panel) {
    const int pe = p0 + CNB < n - 1 ? p0 + CNB : n - 1;
    const z* S = panel == 0 ? A0 : Ab;
#pragma unroll
    for (int q = 0; q < CNB; ++q) { pu[q] = mk(0, 0); pw[q] = mk(0, 0); }
    z xnext = mk(0, 0);  // the panel's first column
    if (r >= p0 && r < n)
      xnext = panel == 0 ? ldz_g(A0 + (size_t)r * n + p0) : ldz_sc1(xc + (size_t)((panel & 1) * CNB) * n + r);
    for (int j = p0; j < pe; ++j) {
      const int l = j - p0;
      // (a) column j with the panel's pending updates: x = A_j - U W^H - W U^H
      // (its stored value was loaded during the previous column)
      z x = xnext;
      if (j + 1 < pe && r >= j + 1 && r < n)
        xnext = panel == 0 ? ldz_g(A0 + (size_t)r * n + j + 1)
                           : ldz_sc1(xc + (size_t)((panel & 1) * CNB + l + 1) * n + r);
      if (r >= j && r < n) {
#pragma unroll
        for (int q = 0; q < CNB; ++q) {
          if (q < l) {  // slots l.. are zero (uniform branch)
            const z rU = q == l - 1 ? ru : Nx[j & 1][0][q], rW = q == l - 1 ? rw : Nx[j & 1][1][q];
            x = zsub(x, zadd(zmul(pu[q], zcj(rW)), zmul(pw[q], zcj(rU))));
          }
        }
      }
      if (r == j) Ld[j] = x.x;
      if (r == j + 1) {
        X1 = x;
#pragma unroll
        for (int q = 0; q < CNB; ++q) { Nx[(j + 1) & 1][0][q] = pu[q]; Nx[(j + 1) & 1][1][q] = pw[q]; }
      }
      LU[r] = x;
      const double v = wave_allsum((r >= j + 2 && r < n) ? x.x * x.x + x.y * x.y : 0.0);
      if (lane == 0) red1[wv] = v;
      __syncthreads();
      double s = 0;
#pragma unroll
      for (int w = 0; w < 8; ++w) s += red1[w];
      STAMP(0);
      // (b) reflector H = I - t u u^H zeroing x[j+2..n) (every thread)
      const z a = X1;
      const double aa = sqrt(a.x * a.x + a.y * a.y), xn = sqrt(aa * aa + s);
      double t = 0;
      z bb = mk(0, 0), u0 = a;
      if (xn > 0) {
        const z ph = aa > 0 ? mk(a.x / aa, a.y / aa) : mk(1, 0);
        bb = mk(-ph.x * xn, -ph.y * xn);
        u0 = mk(a.x + ph.x * xn, a.y + ph.y * xn);
        const double ua = aa + xn;
        t = 2.0 / (ua * ua + s);
      }
      if (tid == 0) { Ltau[j] = t; LB[j] = bb; }
      if (t == 0.0) {  // column already reduced: H = I, slot l stays zero (uniform)
        ru = mk(0, 0);
        rw = mk(0, 0);
        continue;
      }
      const bool live = r > j && r < n;
      const z ur = r == j + 1 ? u0 : (live ? x : mk(0, 0));
      STAMP(1);
      // (c) p = A u on this member's columns (the panel-start matrix)
      const int hb = hop & 1;
      {
        const int cb_lo = (j + 1) >> 4;
        const int k0 = cb_lo <= me ? 0 : (cb_lo - me + G - 1) / G;
        const int nown = me + G * k0 < nblk ? (nblk - 1 - me) / G - k0 + 1 : 0;
        const int c_lo = (j + 1) >> 5, nch = ((n - 1) >> 5) - c_lo + 1;
        // this member's column p_i and the u^H A u partial of its block (lanes of one
        // 16-lane row = one block), handed off with sc1 stores
        auto finish = [&](z p, int cb, int i) {
          const bool li = i > j && i < n;
          const z ui = li ? (i == j + 1 ? u0 : LU[i]) : mk(0, 0);
          z e = li ? zcjmul(ui, p) : mk(0, 0);
          // the block's sum over its 16 lanes (one DPP row), the same bits in each
          e.x += dpp_d<0xB1>(e.x); e.y += dpp_d<0xB1>(e.y);
          e.x += dpp_d<0x4E>(e.x); e.y += dpp_d<0x4E>(e.y);
          e.x += dpp_d<0x141>(e.x); e.y += dpp_d<0x141>(e.y);
          e.x += dpp_d<0x140>(e.x); e.y += dpp_d<0x140>(e.y);
          if (li) stz_sc1(pb + hb * n + i, p);
          if ((i & 15) == 0) stz_sc1(bp + hb * 32 + cb, e);
        };
        if (nown >= COOP_MODEA_MIN) {
          // every wave busy with whole 64-column groups: each lane sums its column's
          // chunks in order itself (the same bits as the partials below)
          for (int g4 = wv; 4 * g4 < nown; g4 += 8) {
            const int bi = 4 * g4 + (lane >> 4), cb = me + G * (k0 + bi), col = 16 * cb + (lane & 15);
            const bool cok = bi < nown && col > j && col < n;
            z p = mk(0, 0);
            for (int c = c_lo; c < c_lo + nch; ++c) {
              const z acc = chunk_acc(S, n, col, cok, j, c, u0, LU);
              p = c == c_lo ? acc : zadd(p, acc);
            }
            if (bi < nown) finish(p, cb, col);
          }
        } else
        for (int b0 = 0; b0 < nown; b0 += CMB) {
          const int nb = nown - b0 < CMB ? nown - b0 : CMB;
          // items (64-column group, 32-row chunk): lane = column, the chunk's rows summed in order
          const int ncg = (nb + 3) >> 2;
          for (int it = wv; it < ncg * nch; it += 8) {
            const int cgl = it % ncg, c = c_lo + it / ncg;
            const int bi = cgl * 4 + (lane >> 4);
            const int col = 16 * (me + G * (k0 + b0 + bi)) + (lane & 15);
            const bool cok = bi < nb && col > j && col < n;
            ws[(c - c_lo) * (CMB * 16) + cgl * 64 + lane] = chunk_acc(S, n, col, cok, j, c, u0, LU);
          }
          __syncthreads();
          if (tid < nb * 16) {
            const int cb = me + G * (k0 + b0 + (tid >> 4)), i = 16 * cb + (tid & 15);
            z p = ws[tid];
            for (int c = 1; c < nch; ++c) p = zadd(p, ws[c * (CMB * 16) + tid]);
            finish(p, cb, i);
          }
          if (b0 + CMB < nown) __syncthreads();  // the partials are reused
        }
      }
      STAMP(2);
      if (G > 1) coop_signal(cnt);
      else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      STAMP(3);
      // (d) dots W^H u, U^H u over rows j+1.. (while the other members finish)
      {
        // values 2q, 2q+1 (W_q^H u) and 24+2q, 24+2q+1 (U_q^H u): halved by xor 32,
        // 16, 8 (permlane swaps, DPP), then summed over the remaining 8 lanes
        double d24[24];
#pragma unroll
        for (int q = 0; q < CNB; ++q) {
          if (q < l) {  // uniform: slots l.. are zero
            const z a1 = zcjmul(pw[q], ur), b1 = zcjmul(pu[q], ur);
            d24[2 * q] = rs32(a1.x, b1.x);
            d24[2 * q + 1] = rs32(a1.y, b1.y);
          } else {
            d24[2 * q] = 0.0;
            d24[2 * q + 1] = 0.0;
          }
        }
        double d12[12], d6[6];
#pragma unroll
        for (int i = 0; i < 12; ++i) d12[i] = (i >> 1) < l || 6 + (i >> 1) < l ? rs16(d24[i], d24[12 + i]) : 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i)
          d6[i] = (i >> 1) < l || 3 + (i >> 1) < l || 6 + (i >> 1) < l || 9 + (i >> 1) < l
                      ? sum8(rs8(d12[i], d12[6 + i], lane)) : 0.0;
        if ((lane & 7) == 0) {
          const int b = 24 * (lane >> 5) + 12 * ((lane >> 4) & 1) + 6 * ((lane >> 3) & 1);
#pragma unroll
          for (int i = 0; i < 6; ++i) red2[wv][b + i] = d6[i];
        }
      }
      __syncthreads();
      if (tid < 48) {
        double f = 0;
#pragma unroll
        for (int w = 0; w < 8; ++w) f += red2[w][tid];
        fin[tid] = f;
      }
      STAMP(4);
      ++hop;
      if (G > 1) {
        if (!coop_wait(cnt, abt, G * hop, tmo, &sflag)) return;
      } else {
        __syncthreads();
      }
      // reflector j into column j of the block, by its owner, once every member has read column j
      STAMP(5);
      if (live && ((j >> 4) - me) % G == 0) stz_g(A0 + (size_t)r * n + j, ur);
      // (e) p = t (A u - U (W^H u) - W (U^H u)), K = t/2 Re(u^H p), w = p - K u
      // dots from LDS where used: W_q^H u = fin[2q..], U_q^H u = fin[24 + 2q..]
#define DW(q) mk(fin[2 * (q)], fin[2 * (q) + 1])
#define DU(q) mk(fin[24 + 2 * (q)], fin[24 + 2 * (q) + 1])
      // the hand-off's loads first (independent, one latency): this row's and
      // row j+1's A u, the u^H A u partials of the column blocks
      const int cbl = (j + 1) >> 4;
      z p1 = ldz_sc1(pb + hb * n + j + 1);
      z p = live ? ldz_sc1(pb + hb * n + r) : mk(0, 0);
      const z eb = lane < nblk - cbl ? ldz_sc1(bp + hb * 32 + cbl + lane) : mk(0, 0);
      const z uau = mk(wave_allsum(eb.x), wave_allsum(eb.y));
      // one pass over the panel slots (each dot read once from LDS): Re sum
      // conj(dU) dW for K, row j+1's p (every thread the same way), this row's p
      double sd = 0;
#pragma unroll
      for (int q = 0; q < CNB; ++q) {
        if (q < l) {  // uniform: slots l.. are zero
          const z dw = DW(q), du = DU(q);
          sd += du.x * dw.x + du.y * dw.y;  // Re(conj(dU) dW)
          p1 = zsub(p1, zadd(zmul(Nx[(j + 1) & 1][0][q], dw), zmul(Nx[(j + 1) & 1][1][q], du)));
          p = zsub(p, zadd(zmul(pu[q], dw), zmul(pw[q], du)));
        }
      }
      const double K = 0.5 * t * t * (uau.x - 2.0 * sd);
      rw = zsub(zsc(p1, t), zsc(u0, K));
      ru = u0;
      if (live) {
        const z wr = r == j + 1 ? rw : zsub(zsc(p, t), zsc(ur, K));
#pragma unroll
        for (int q = 0; q < CNB; ++q)
          if (q == l) { pu[q] = ur; pw[q] = wr; }
      }
      STAMP(6);
#undef DW
#undef DU
    }
    // close the panel on this member's columns: C -= U W^H + W U^H, rows and
    // columns pe..n-1 (64 x 64 tiles on v_mfma_f64_16x16x4f64, panel rows
    // staged in LDS from the registers of the threads holding them); the next
    // panel's columns go to the hand-off buffer as well
    {
      const int cb_lo = pe >> 4;
      const int k0 = cb_lo <= me ? 0 : (cb_lo - me + G - 1) / G;
      const int nown = me + G * k0 < nblk ? (nblk - 1 - me) / G - k0 + 1 : 0;
      const int nxp = (panel + 1) & 1;
      z* Sg = ws;  // [4][64][CNB]: U rows, W rows, U cols, W cols
      const int tr = wv >> 1, tc0 = 2 * (wv & 1), ml = lane & 15, kl = lane >> 4;
      for (int b0 = 0; b0 < nown; b0 += 4) {
        const int nb = nown - b0 < 4 ? nown - b0 : 4;
        for (int r0 = pe; r0 < n; r0 += 64) {
          // this wave's outputs of the tile: the stored values first (in flight
          // while the panel rows are staged and the MFMAs run)
          z v0[2][4];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int c = 16 * (me + G * (k0 + b0 + tc0 + h)) + ml;
            const bool cok = tc0 + h < nb && c >= pe && c < n;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {  // clamped address, unconditional load (used only where valid)
              const int rg = r0 + 16 * tr + kl + 4 * rr;
              v0[h][rr] = ldz_g(S + (size_t)(rg < n ? rg : n - 1) * n + (c < n ? c : n - 1));
            }
            (void)cok;
          }
          __syncthreads();
          if (r >= r0 && r < r0 + 64) {
#pragma unroll
            for (int q = 0; q < CNB; ++q) { Sg[(r - r0) * CNB + q] = pu[q]; Sg[(64 + r - r0) * CNB + q] = pw[q]; }
          }
          if (r0 == pe) {  // the batch's columns: staged once
            const int cbr = r >> 4;
            const int kk = (cbr - me) / G - k0 - b0;
            if (cbr >= me && (cbr - me) % G == 0 && kk >= 0 && kk < nb) {
              const int cl = 16 * kk + (r & 15);
#pragma unroll
              for (int q = 0; q < CNB; ++q) { Sg[(128 + cl) * CNB + q] = pu[q]; Sg[(192 + cl) * CNB + q] = pw[q]; }
            }
          }
          __syncthreads();
          if (r0 + 16 * tr >= n) continue;  // wave-uniform
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int tc = tc0 + h;
            if (tc >= nb) continue;  // wave-uniform
            d4 cr = {0, 0, 0, 0}, ci = {0, 0, 0, 0};
#pragma unroll
            for (int ks = 0; ks < 2 * CNB / 4; ++ks) {
              const int kap = 4 * ks + kl;
              const int rowA = 16 * tr + ml, colB = 16 * tc + ml;
              const z av = kap < CNB ? Sg[rowA * CNB + kap] : Sg[(64 + rowA) * CNB + kap - CNB];
              const z bw = kap < CNB ? Sg[(192 + colB) * CNB + kap] : Sg[(128 + colB) * CNB + kap - CNB];
              const double bx = bw.x, by = -bw.y;
              cr = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, bx, cr, 0, 0, 0);
              cr = __builtin_amdgcn_mfma_f64_16x16x4f64(-av.y, by, cr, 0, 0, 0);
              ci = __builtin_amdgcn_mfma_f64_16x16x4f64(av.x, by, ci, 0, 0, 0);
              ci = __builtin_amdgcn_mfma_f64_16x16x4f64(av.y, bx, ci, 0, 0, 0);
            }
            const int c = 16 * (me + G * (k0 + b0 + tc)) + ml;
            if (c >= pe && c < n) {
#pragma unroll
              for (int rr = 0; rr < 4; ++rr) {
                const int rg = r0 + 16 * tr + kl + 4 * rr;
                if (rg < n) {
                  const z v = mk(v0[h][rr].x - cr[rr], v0[h][rr].y - ci[rr]);
                  stz_g(Ab + (size_t)rg * n + c, v);
                  if (c - pe < CNB) stz_sc1(xc + (size_t)(nxp * CNB + c - pe) * n + rg, v);
                }
              }
            }
          }
        }
      }
      ++hop;
      if (G > 1) {
        coop_signal(cnt);
        if (!coop_wait(cnt, abt, G * hop, tmo, &sflag)) return;
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      STAMP(7);
    }
  }
  // the last diagonal element (after the last panel's update)
  if (tid == 0) Ld[n - 1] = n > 1 ? ldz_sc1(xc + (size_t)((panel & 1) * CNB) * n + n - 1).x : A0[0].x;
  for (int j = tid; j < n - 1; j += CPT) Le2[j] = LB[j].x * LB[j].x + LB[j].y * LB[j].y;
  if (tid == 0) Le2[n - 1] = 0;
  __syncthreads();
  if (me == 0) {
    for (int j = tid; j < n; j += CPT) {
      P.d[j] = Ld[j];
      if (j < n - 1) {
        P.e[j] = sqrt(Le2[j]);
        P.tau[j] = Ltau[j];
      }
    }
    if (tid == 0) {
      P.e[n - 1] = 0;
      z dl = mk(1, 0);
      P.ph[0] = dl;
      for (int j = 0; j + 1 < n; ++j) {
        const z b = LB[j];
        const double ab = sqrt(b.x * b.x + b.y * b.y);
        if (ab > 0) dl = zmul(dl, mk(b.x / ab, b.y / ab));
        P.ph[j + 1] = dl;
      }
    }
  }
  // eigenvalues: multisection, 4 interior points per round (LAPACK dstebz
  // bounds and tolerances, as bisect_all), this member's range of the
  // resolved ones (the nres largest; the rest below thr_rel * trace)
  double gl = 1e300, gu = -1e300, emax = 0, tr = 0;
  for (int i = tid; i < n; i += CPT) {
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
  __shared__ double bb4[4][8];
  __shared__ int sres;
  if (lane == 0) { bb4[0][wv] = gl; bb4[1][wv] = gu; bb4[2][wv] = emax; bb4[3][wv] = tr; }
  __syncthreads();
  gl = bb4[0][0]; gu = bb4[1][0]; emax = bb4[2][0]; tr = bb4[3][0];
  for (int i = 1; i < 8; ++i) { gl = fmin(gl, bb4[0][i]); gu = fmax(gu, bb4[1][i]); emax = fmax(emax, bb4[2][i]); tr += bb4[3][i]; }
  const double eps = 2.220446049250313e-16, safmin = 2.2250738585072014e-308;
  const double tnorm = fmax(fabs(gl), fabs(gu));
  const double pivmin = safmin * fmax(1.0, emax);
  gl -= 2.0 * eps * tnorm * n + 2.0 * pivmin;
  gu += 2.0 * eps * tnorm * n + 2.0 * pivmin;
  const double atol = 4.0 * eps * tnorm;
  const double thr = P.thr_rel * tr;
  if (tid == 0) {
    int below = 0;
    if (thr > 0) below = sturm_count1(Ld, Le2, n, thr, pivmin);
    sres = n - below;
  }
  __syncthreads();
  const int nres = sres;
  const int per = (nres + G - 1) / G, e0 = me * per, e1 = e0 + per < nres ? e0 + per : nres;
  const int ne = e1 > e0 ? e1 - e0 : 0;
  double* lo = reinterpret_cast<double*>(ws);
  double* hi = lo + CPT;
  int* cntl = reinterpret_cast<int*>(hi + CPT);  // [ne][4]
  constexpr int NP = 5;                          // sub-intervals per round
  if (ne > 0) {
    for (int tt = tid; tt < ne; tt += CPT) { lo[tt] = nres < n ? fmax(gl, thr) : gl; hi[tt] = gu; }
    __syncthreads();
    const bool one = ne <= CPT / 4;  // one shift per thread (4 threads per eigenvalue), else 4 per thread
    for (int it = 0; it < 128; ++it) {
      bool active = false;
      if (one) {
        const int t = tid >> 2, q = tid & 3;
        if (t < ne) {
          const double l = lo[t], h = hi[t];
          active = h - l > atol + 2.0 * eps * fmax(fabs(l), fabs(h));
          if (active) cntl[4 * t + q] = sturm_count1(Ld, Le2, n, l + (h - l) * double(q + 1) / NP, pivmin);
        }
      } else if (tid < ne) {
        const double l = lo[tid], h = hi[tid];
        active = h - l > atol + 2.0 * eps * fmax(fabs(l), fabs(h));
        if (active) {
          double xs[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) xs[q] = l + (h - l) * double(q + 1) / NP;
          sturm_count4(Ld, Le2, n, xs, pivmin, cntl + 4 * tid);
        }
      }
      if (!__syncthreads_or(active)) break;
      if (tid < ne) {
        const double l = lo[tid], h = hi[tid];
        if (h - l > atol + 2.0 * eps * fmax(fabs(l), fabs(h))) {
          const int idxa = n - 1 - (e0 + tid);  // ascending index of the (e0 + tid)-th largest
          double nl = l, nh = h;
          for (int q = 1; q < NP; ++q) {
            const double xq = l + (h - l) * double(q) / NP;
            if (cntl[4 * tid + q - 1] > idxa) { nh = xq; break; }
            nl = xq;
          }
          lo[tid] = nl;
          hi[tid] = nh;
        }
      }
      __syncthreads();
    }
  }
#ifdef HBM_STAMP
  __syncthreads();
  STAMP(8);
  if (tid == 0 && gi == 0)
    printf("vals_coop n=%d G=%d member %d stamps: column %llu reflector %llu matvec %llu signal %llu dots %llu wait %llu "
           "p/w %llu panel %llu bisect %llu\n", n, G, me, stamp_acc[0], stamp_acc[1], stamp_acc[2], stamp_acc[3],
           stamp_acc[4], stamp_acc[5], stamp_acc[6], stamp_acc[7], stamp_acc[8]);
#endif
  if (nres == n) {
    for (int tt = tid; tt < ne; tt += CPT) P.w[e0 + tt] = 0.5 * (lo[tt] + hi[tt]);
    return;
  }
  // unresolved eigenvalues: their mean (trace minus the resolved ones), by member 0
  for (int tt = tid; tt < ne; tt += CPT) std_sc1(P.w + e0 + tt, 0.5 * (lo[tt] + hi[tt]));
  ++hop;
  if (G > 1) {
    coop_signal(cnt);
    if (me != 0) return;
    if (!coop_wait(cnt, abt, G * hop, tmo, &sflag)) return;
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  double sr = 0;
  for (int t = tid; t < nres; t += CPT) sr += ldd_sc1(P.w + t);
  for (int o = 32; o > 0; o >>= 1) sr += __shfl_xor(sr, o, 64);
  if (lane == 0) red1[wv] = sr;
  __syncthreads();
  sr = 0;
  for (int i = 0; i < 8; ++i) sr += red1[i];
  const double mean = fmin(fmax((tr - sr) / (n - nres), 0.0), thr);
  for (int t = nres + tid; t < n; t += CPT) P.w[t] = mean;
}

// groups that gave up: the block again on one CU (k_heev_vals_big's body),
// its lower triangle first restored from the untouched upper one
// (nfb: count of the groups re-run, or null)
__global__ __launch_bounds__(VBG) void k_heev_vals_coop_fix(const EProb* __restrict__ probs,
                                                            const int* __restrict__ idx, const int* __restrict__ ctl,
                                                            int* __restrict__ nfb) {
  const int gi = blockIdx.x;
  if (__hip_atomic_load(const_cast<int*>(ctl) + kCoopCtl * gi + 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
    return;
  if (nfb && threadIdx.x == 0) __hip_atomic_fetch_add(nfb, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const EProb P = probs[idx[gi]];
  const int n = P.n;
  for (size_t e = threadIdx.x; e < (size_t)n * n; e += VBG) {
    const int rr = int(e / n), c = int(e - (size_t)rr * n);
    if (rr > c) P.A[e] = zcj(P.A[(size_t)c * n + rr]);
  }
  __syncthreads();
  vals_big_body(P);
}

}  // namespace hbm
