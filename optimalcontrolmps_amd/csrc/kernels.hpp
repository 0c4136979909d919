// Kernel bodies of liboptimalcontrolmps_amd (device code, gfx950).  The
// __global__ entry points in ocmps.hip only declare the dynamic LDS and call
// these; one workgroup = one MPS chain (engine_device.hpp).
#pragma once

#include "engine_device.hpp"
#include "fast_chain.hpp"
#include "fast_overlap.hpp"

namespace ocg {

// LDS arrays of the general chain as flat pointers (the one-wave chain's
// load / store take either global or LDS memory)
__device__ __forceinline__ int* flat(LDS int* p) { return (int*)p; }
__device__ __forceinline__ zc* flat(lzp p) { return (zc*)(double*)p.p; }
// the one-wave padded chain steps this launch (fast_chain.hpp)
__device__ __forceinline__ bool fast_on(const OcgParams& P) { return P.fplan != nullptr && !P.imag; }
// a publishing fast chain's write-through stores have all completed (wave 0; the
// other waves store nothing), so the flag that follows can be a plain relaxed
// agent-scope store: no L2 write-back fence.  This relies on the gfx950
// hand-off rule of MI355X_MICROARCH.md (§Workgroup dispatch ..., "Valid forms"
// and the hand-off table, row 1): every payload store is an agent-scope
// (sc1, write-through) atomic store, the storing wave waits s_waitcnt vmcnt(0)
// before the one lane that signals, and every consumer polls relaxed, then
// takes one agent-scope acquire before its plain loads (wait_flag).  Under the
// HIP memory model alone the relaxed flag store is not a release; the CPU
// emulation (OCG_EMU: tests/emu/hip/hip_runtime.h maps every HIP atomic to a
// seq_cst one, payload stores included) therefore runs a correctly
// synchronised protocol, which its TSan run checks.
__device__ __forceinline__ void publish_flag_wt(int* flag, int epoch, int* progress) {
  if (threadIdx.x < 64) {
#ifndef OCG_EMU
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    if (threadIdx.x == 0) {
      __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(progress, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// --------------------------------------------------------------------------
// device statistics: [kind][0] = alg bytes, [1] = alg flops, [2] = steps
struct StatAcc {
  double bytes = 0, flops = 0, steps = 0;
};

#ifdef OCG_PROFILE
__device__ double g_ocg_prof[32];
#endif

template <class CH>
__device__ inline void flush_stats(CH& c, double* stats, double bytes, double flops, double steps) {
#ifdef OCG_PROFILE
  c.pf(12);
  if (threadIdx.x == 0)
    for (int i = 0; i < 32; ++i) atomicAdd(&g_ocg_prof[i], c.PROF[i]);
#endif
  if (threadIdx.x == 0 && stats) {
    atomicAdd(stats + 0, bytes);
    atomicAdd(stats + 1, flops);
    atomicAdd(stats + 2, steps);
  }
}

struct Pool {
  int* dims;       // [nslots][nsq]
  zc* data;   // [nslots][cap]
};

#define SLOT_D(pool, P, s) ((pool).dims + (size_t)(s) * (P).nsq)
#define SLOT_X(pool, P, s) ((pool).data + (size_t)(s) * (P).cap)

// --------------------------------------------------------------------------
template <int NT>
__device__ OCG_INLINE void body_trajectory(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md,
                                                   Pool pool, int slot_init, int slot_target, int psi_base0,
                                                   int xi_base0, const double* u0, int N, int which, double* stats,
                                                   int cs) {
  Chain<NT> c(P, smem);
  c.load_tables(gf, gb, md);
  // which == 3: workgroup 2k + {0, 1} = control k's psi / xi chain (ocg_gradient_multi:
  // control k's slots cs after control k-1's, its controls N after)
  int chain = (which == 3) ? (blockIdx.x & 1) : (which == 1 ? 0 : 1);
  const int kc = (which == 3) ? (blockIdx.x >> 1) : 0;
  const int psi_base = psi_base0 + kc * cs, xi_base = xi_base0 + kc * cs;
  const double* u = u0 + (size_t)kc * N;
  // chain 0: psi_t forward from psi_init (calcPsi, src/OptimalControl.cpp:375-390)
  // chain 1: xi_t backward from psi_target (calcXi, :392-407)
  const int fwd = (chain == 0) ? 1 : 0;
  const int base = fwd ? psi_base : xi_base;
  const int src = fwd ? slot_init : slot_target;
  double bytes = 0, flops = 0;
  int t = fwd ? 0 : N - 1;
  if (fast_on(P)) {
    FastChain f(P, smem + P.fast_off, P.fplan, c.PROF);
    __syncthreads();  // load_tables' writes first: the region may alias them (P.fast_off = 0)
    f.init(P.fplan, gf, gb);
    f.load(SLOT_D(pool, P, src), SLOT_X(pool, P, src));
    f.store(SLOT_D(pool, P, base + t), SLOT_X(pool, P, base + t));
    for (int s = 0; s + 1 < N; ++s) {
      const int tn = fwd ? t + 1 : t - 1;
      f.step(u[t], u[tn], fwd, s + 2 == N);
      f.store(SLOT_D(pool, P, base + tn), SLOT_X(pool, P, base + tn));
      t = tn;
    }
    f.model_totals(bytes, flops);
    __syncthreads();
  } else {
    c.load(SLOT_D(pool, P, src), SLOT_X(pool, P, src));
    c.store(SLOT_D(pool, P, base + t), SLOT_X(pool, P, base + t));
    for (int s = 0; s + 1 < N; ++s) {
      const int tn = fwd ? t + 1 : t - 1;
      c.step(u[t], u[tn], fwd, s + 2 == N);  // closing gauge move on the last step only (Chain::step)
      c.store(SLOT_D(pool, P, base + tn), SLOT_X(pool, P, base + tn));
      t = tn;
    }
    c.model_totals(bytes, flops);
  }
  flush_stats(c, stats, bytes, flops, double(N - 1));
}

// out[i] = <x_i|y_i> or <x_i|dH|y_i>
template <int NT>
__device__ OCG_INLINE void body_overlaps(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md,
                                                 Pool pool, const int* xs, const int* ys, int npairs, int with_dH,
                                                 zc* out, double* stats) {
  Chain<NT, true> c(P, smem);
  c.load_tables(gf, gb, md);
  int i = blockIdx.x;
  if (i >= npairs) return;
  c.load(SLOT_D(pool, P, ys[i]), SLOT_X(pool, P, ys[i]));
  zc r = c.overlap(SLOT_D(pool, P, xs[i]), SLOT_X(pool, P, xs[i]), with_dH);
  const double b = 32.0 * c.mps_used();
  if (threadIdx.x == 0) out[i] = r;
  flush_stats(c, stats, b, 8.0 * b / 16.0 * 4.0, 0.0);
}

// body_overlaps on the padded layout (fast_overlap.hpp, P.oplan set): one wave
// per pair, grid-stride
__device__ inline OCG_INLINE void body_overlaps_pad(char* smem, OcgParams P, Pool pool, const int* xs, const int* ys,
                                                    int npairs, int with_dH, zc* out, double* stats) {
  FastOverlap o(P, smem, P.oplan, true);
  o.init(P.oplan);
  double b = 0;
  for (int i = blockIdx.x; i < npairs; i += gridDim.x) {
    const int ny = o.load(SLOT_D(pool, P, xs[i]), SLOT_X(pool, P, xs[i]), SLOT_D(pool, P, ys[i]),
                          SLOT_X(pool, P, ys[i]));
    const zc r = with_dH ? o.contract_dH(o.YP, P.dH) : o.contract(o.YP);
    b += 32.0 * ny;
    if (threadIdx.x == 0) out[i] = r;
    o.wsync();  // LDS reuse by the next pair
  }
  if (threadIdx.x == 0 && stats) {
    atomicAdd(stats + 0, b);
    atomicAdd(stats + 1, 8.0 * b / 16.0 * 4.0);
  }
}

template <int NT>
__device__ OCG_INLINE void body_apply_dH(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md,
                                                 Pool pool, const int* in, const int* outs, int n, double* norms,
                                                 double* stats) {
  Chain<NT> c(P, smem);
  c.load_tables(gf, gb, md);
  int i = blockIdx.x;
  if (i >= n) return;
  c.load(SLOT_D(pool, P, in[i]), SLOT_X(pool, P, in[i]));
  const double b0 = 16.0 * c.mps_used();
  c.apply_dH();
  double n2 = c.site_norm2(1);
  c.store(SLOT_D(pool, P, outs[i]), SLOT_X(pool, P, outs[i]));
  const double b = b0 + 16.0 * c.mps_used();
  if (threadIdx.x == 0 && norms) norms[i] = sqrt(n2);
  flush_stats(c, stats, b, 8.0 * b, 0.0);
}

// calcHessianRow (src/OptimalControl.cpp:251-279).  psiH_i =
// exactApplyMPO(propDeriv, psi_t[i]) and its norm normiH come from a preceding
// batched body_apply_dH launch (slots psih_base + i, norms[i]).
template <int NT>
__device__ OCG_INLINE void body_hessian_rows(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md, Pool pool,
                                  int psih_base, int xih_base, const int* rows, int nrows, const double* norms,
                                  const double* u, int N, const zc* divT, zc F, double* H, double* stats) {
  Chain<NT> c(P, smem);
  c.load_tables(gf, gb, md);
  int r = blockIdx.x;
  if (r >= nrows) return;
  const int i = rows[r];
  const double dt2 = P.dt * P.dt;
  const double normiH = norms[i];
  c.load(SLOT_D(pool, P, psih_base + i), SLOT_X(pool, P, psih_base + i));
  double bytes = 0, flops = 0;
  const bool fo = fast_on(P);
  FastChain f(P, smem + P.fast_off, P.fplan, c.PROF);
  // the padded overlap (fast_overlap.hpp) in the general chain's region, which
  // the one-wave chain leaves unused: the arithmetic of k_row_overlaps_pad, so
  // fused == unfused stays bitwise
  const bool po = fo && P.oplan != nullptr;
  FastOverlap o(P, smem, po ? P.oplan : nullptr);
  if (fo) {
    if (po) {
      __syncthreads();  // load_tables' writes into the region first
      o.init(P.oplan);
    }
    f.init(P.fplan, gf, gb);
    f.load(SLOT_D(pool, P, psih_base + i), SLOT_X(pool, P, psih_base + i));
  }
  // j = i: diagonal entry (:259-264); j > i: step psiH once, then overlap (:266-278)
  for (int j = i; j + 1 < N; ++j) {
    if (j > i) {
      if (fo) {
        f.step(u[j - 1], u[j], 1, false);
        if (!po) {
          // the general overlap: the state goes through the general chain's LDS
          // copy (compact layout, offsets rebuilt by load)
          f.store(flat(c.DIMS), flat(c.A));
          __syncthreads();
          c.load(flat(c.DIMS), flat(c.A));
        }
      } else {
        c.step(u[j - 1], u[j], 1, false);  // row: no closing gauge move (Chain::step)
      }
    }
    zc ov;
    double used;
    if (po) {
      o.load(SLOT_D(pool, P, xih_base + j), SLOT_X(pool, P, xih_base + j), nullptr, nullptr);
      ov = o.contract(f.MP);
      used = o.compact_size(f.DIM);
    } else {
      ov = c.overlap(SLOT_D(pool, P, xih_base + j), SLOT_X(pool, P, xih_base + j), 0);
      used = c.mps_used();
    }
    if (threadIdx.x == 0) {
      zc di = divT[i], dj = divT[j];
      double v1 = (F.x * ov.x - F.y * ov.y) * (j > i ? normiH : 1.0);  // Re(F <xiH_j|psiH> n_i)
      double v2 = -(di.x * dj.x + di.y * dj.y);                        // -Re(divT_i conj(divT_j))
      double res = dt2 * (v1 + v2);
      H[(size_t)i * N + j] = res;
      if (j > i) H[(size_t)j * N + i] = res;
      bytes += 32.0 * used;
    }
  }
  double mb, mf;
  if (fo) f.model_totals(mb, mf);
  else c.model_totals(mb, mf);
  bytes += mb;
  flops += mf;
  flush_stats(c, stats, bytes, flops, double(N - 2 - i > 0 ? N - 2 - i : 0));
}

// --------------------------------------------------------------------------
// Fused getHessian pipeline (ocg_hessian).  Rows start as soon as their psi_i
// exists instead of after both trajectory sweeps, and the <xiH_j|psiH_i(j)>
// overlaps move to a second, fully parallel kernel:
//   k_pipeline   grid [0] psi chain, [1] xi chain (each publishes state t via
//                flags[t] / flags[N+t]), [2, 2+nxw) xiH_t = dH xi_t workers,
//                [2+nxw, 2+nxw+nrows) row r: wait psi_i, psiH = dH psi_i, store
//                psiH_i(i..N-2) (the states calcHessianRow overlaps, :251-279)
//   k_row_overlaps  one workgroup per stored psiH_i(j): overlap with xiH_j, H_ij
// Producers and consumers live in one grid.  Roles are taken by ticket (the
// order in which workgroups start running, flags[2N+1], zeroed per launch),
// not by blockIdx: every role only ever waits on roles with lower tickets,
// which are already running, so progress holds whatever the dispatch order
// and however few workgroups fit the device (long horizons: N_t = 801 has
// 799 rows > CUs).  Every publication also bumps a progress counter
// (flags[2N]); a waiter gives up (err |= OCG_ERR_WATCHDOG) only after ~2^24
// polls (~15 s) during which no producer published anything, so a slow but
// live pipeline (long horizons, large chains, several shards per GPU) never
// trips it.
__device__ __forceinline__ void publish_flag(int* flag, int epoch, int* progress) {
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(flag, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(progress, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
template <int NT>
__device__ OCG_INLINE bool await_flag(Chain<NT>& c, const int* flag, int epoch, int* err, const int* progress) {
  if (threadIdx.x == 0) {
    int ok = 1;
    long spins = 0;
    int seen = __hip_atomic_load(progress, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // relaxed polls (no L2 invalidate per poll), one acquire fence on success
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch) {
      __builtin_amdgcn_s_sleep(32);  // ~2k cycles between polls: a waiting row is idle, not a poller
      const int now = __hip_atomic_load(progress, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (now != seen) {
        seen = now;
        spins = 0;
      }
      if (++spins > (1L << 24) || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        ok = 0;
        atomicOr(err, OCG_ERR_WATCHDOG);
        break;
      }
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);  // once per wait (system scope)
    c.ISCAL[15] = ok;
  }
  __syncthreads();
  const int ok = c.ISCAL[15];
  __syncthreads();
  return ok != 0;
}

// K control vectors in one launch (ocg_hessian_multi): control k's trajectory
// slots start k * cs after control 0's, its flags k * (2N + 2) after, its u
// k * N after; the role ticket counter follows the K flag blocks.  Tickets:
// [0, 2K) the K psi / xi chain pairs, [2K, 2K + K nxw) the xiH workers, then
// the rows of all controls interleaved (row r of control k: 2K + K nxw + r K
// + k), so every waiter still waits only on lower tickets.
template <int NT>
__device__ OCG_INLINE void body_pipeline(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md,
                                         Pool pool, int slot_init, int slot_target, int psi_base0, int xi_base0,
                                         int xih_base0, const double* u0, int N, const int* rows, int nrows,
                                         const int* rbase, Pool rs, double* rnorm0, int* flags0, int epoch, int* err,
                                         int nxw, double* stats, int K, int cs) {
  Chain<NT> c(P, smem);
  if (threadIdx.x == 0)
    c.ISCAL[14] = __hip_atomic_fetch_add(flags0 + K * (2 * N + 2), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int tk = c.ISCAL[14];  // this workgroup's ticket
  __syncthreads();
  // ticket -> (control kc, role b of the single-control numbering)
  int kc, b;
  if (tk < 2 * K) { kc = tk >> 1; b = tk & 1; }
  else if (tk < 2 * K + K * nxw) { kc = (tk - 2 * K) / nxw; b = 2 + (tk - 2 * K) % nxw; }
  else { const int t = tk - 2 * K - K * nxw; kc = t % K; b = 2 + nxw + t / K; }
  const int psi_base = psi_base0 + kc * cs, xi_base = xi_base0 + kc * cs, xih_base = xih_base0 + kc * cs;
  const double* u = u0 + (size_t)kc * N;
  int* const flags = flags0 + (size_t)kc * (2 * N + 2);
  c.load_tables(gf, gb, md);
  int* const progress = flags + 2 * N;
  double bytes = 0, flops = 0, nsteps = 0;
  const bool fo = fast_on(P);
  FastChain f(P, smem + P.fast_off, P.fplan, c.PROF);
  // (the region may alias the general chain's LDS, P.fast_off = 0: a row worker
  // initialises it only after its exactApplyMPO, below)
  if (fo && b < 2) {
    __syncthreads();  // load_tables' writes first (uniform: b is the workgroup's role)
    f.init(P.fplan, gf, gb);
  }
  if (b < 2 && fo) {
    // calcPsi / calcXi on the one-wave chain: every state stored write-through;
    // state t's flag is raised after step t+1 has been computed, when its
    // stores have long completed (the wait costs nothing on the chain's path)
    const int fwd = (b == 0) ? 1 : 0;
    const int base = fwd ? psi_base : xi_base;
    int* fl = flags + (fwd ? 0 : N);
    const int src = fwd ? slot_init : slot_target;
    f.load(SLOT_D(pool, P, src), SLOT_X(pool, P, src));
    int t = fwd ? 0 : N - 1;
    f.store(SLOT_D(pool, P, base + t), SLOT_X(pool, P, base + t), true);
    for (int s = 0; s + 1 < N; ++s) {
      const int tn = fwd ? t + 1 : t - 1;
      f.step(u[t], u[tn], fwd, s + 2 == N);
      publish_flag_wt(fl + t, epoch, progress);
      f.store(SLOT_D(pool, P, base + tn), SLOT_X(pool, P, base + tn), true);
      t = tn;
    }
    publish_flag_wt(fl + t, epoch, progress);
    nsteps = N - 1;
    f.model_totals(bytes, flops);
    __syncthreads();
    flush_stats(c, stats, bytes, flops, nsteps);
    return;
  }
  if (b < 2) {
    // calcPsi / calcXi (src/OptimalControl.cpp:375-407), every state published
    const int fwd = (b == 0) ? 1 : 0;
    const int base = fwd ? psi_base : xi_base;
    int* fl = flags + (fwd ? 0 : N);
    const int src = fwd ? slot_init : slot_target;
    c.load(SLOT_D(pool, P, src), SLOT_X(pool, P, src));
    int t = fwd ? 0 : N - 1;
    c.store(SLOT_D(pool, P, base + t), SLOT_X(pool, P, base + t));
    publish_flag(fl + t, epoch, progress);
    for (int s = 0; s + 1 < N; ++s) {
      const int tn = fwd ? t + 1 : t - 1;
      c.step(u[t], u[tn], fwd, s + 2 == N);  // closing gauge move on the last step only (Chain::step)
      c.store(SLOT_D(pool, P, base + tn), SLOT_X(pool, P, base + tn));
      publish_flag(fl + tn, epoch, progress);
      t = tn;
    }
    nsteps = N - 1;
  } else if (b < 2 + nxw) {
    // xiHlist[t] = exactApplyMPO(propDeriv, xi_t[t]) (:300-303): nxw workers
    // take t = N-1-w, N-1-w-nxw, ... in the order the xi chain publishes
    // them, so few workgroups keep up with it and every row keeps a CU
    for (int t = N - 1 - (b - 2); t >= 0; t -= nxw) {
      if (!await_flag(c, flags + N + t, epoch, err, progress)) return;
      c.load(SLOT_D(pool, P, xi_base + t), SLOT_X(pool, P, xi_base + t));
      c.apply_dH();
      c.store(SLOT_D(pool, P, xih_base + t), SLOT_X(pool, P, xih_base + t));
    }
  } else {
    const int r = b - 2 - nxw;
    if (r >= nrows) return;
    const int i = rows[r];
    if (!await_flag(c, flags + i, epoch, err, progress)) return;
    // psiH = exactApplyMPO(propDeriv, psi_t[i]); normiH = norm(psiH) (:256-257)
    c.load(SLOT_D(pool, P, psi_base + i), SLOT_X(pool, P, psi_base + i));
    c.apply_dH();
    const double n2 = c.site_norm2(1);
    if (threadIdx.x == 0) rnorm0[(size_t)kc * nrows + r] = sqrt(n2);
    int k = kc * rbase[nrows] + rbase[r];  // control kc's row states follow control kc-1's
    c.store(SLOT_D(rs, P, k), SLOT_X(rs, P, k));
    if (fo) {  // the row's steps on the one-wave chain, from the stored psiH_i
      __syncthreads();  // every wave's stores of psiH_i before the one-wave chain reads them
      f.init(P.fplan, gf, gb);
      f.load(SLOT_D(rs, P, k), SLOT_X(rs, P, k));
      for (int j = i + 1; j + 1 < N; ++j) {
        f.step(u[j - 1], u[j], 1, false);
        ++k;
        f.store(SLOT_D(rs, P, k), SLOT_X(rs, P, k));
      }
      double fb, ff;
      f.model_totals(fb, ff);
      bytes += fb;
      flops += ff;
      __syncthreads();
    } else {
      for (int j = i + 1; j + 1 < N; ++j) {  // timeStepper.step(psiH, u[j-1], u[j]) (:269)
        c.step(u[j - 1], u[j], 1, false);  // row: no closing gauge move (Chain::step)
        ++k;
        c.store(SLOT_D(rs, P, k), SLOT_X(rs, P, k));
      }
    }
    nsteps = N - 2 - i;
  }
  double mb, mf;
  c.model_totals(mb, mf);
  flush_stats(c, stats, bytes + mb, flops + mf, nsteps);
}

// H_ij from the stored psiH_i(j) (calcHessianRow's two terms, :259-277)
// K controls (ocg_hessian_multi): pair g of control k = g / total; control
// k's xiH slots k * cs after control 0's, its divT k * N after, its F at Fp[k],
// its row norms k * nrows after, its Hessian k * N^2 after.
template <int NT>
__device__ OCG_INLINE void body_row_overlaps(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md,
                                             Pool pool, int xih_base0, const int* rows, int nrows, const int* rbase,
                                             Pool rs, const double* rnorm0, const zc* divT0, const zc* Fp, int N,
                                             double* H0, double* stats, int K, int cs) {
  Chain<NT, true> c(P, smem);
  c.load_tables(gf, gb, md);
  // grid-stride over the (row, column) pairs: a few thousand resident
  // workgroups each take several pairs (one pair per workgroup is bound by
  // the dispatch rate, not by the work)
  const int total = rbase[nrows];
  double b = 0;
  for (int g = blockIdx.x; g < K * total; g += gridDim.x) {
    const int kc = g / total, gl = g - kc * total;
    int lo = 0, hi = nrows - 1;  // row r with rbase[r] <= gl < rbase[r+1]
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (rbase[mid] <= gl) lo = mid;
      else hi = mid - 1;
    }
    const int r = lo, i = rows[r], j = i + (gl - rbase[r]);
    const int xih_base = xih_base0 + kc * cs;
    c.load(SLOT_D(rs, P, g), SLOT_X(rs, P, g));
    const zc ov = c.overlap(SLOT_D(pool, P, xih_base + j), SLOT_X(pool, P, xih_base + j), 0);
    b += 32.0 * c.mps_used();
    if (threadIdx.x == 0) {
      const zc* divT = divT0 + (size_t)kc * N;
      double* H = H0 + (size_t)kc * N * N;
      const zc F = Fp[kc], di = divT[i], dj = divT[j];
      const double v1 = (F.x * ov.x - F.y * ov.y) * (j > i ? rnorm0[(size_t)kc * nrows + r] : 1.0);  // Re(F <xiH_j|psiH> normiH)
      const double v2 = -(di.x * dj.x + di.y * dj.y);                          // -Re(divT_i conj(divT_j))
      const double res = P.dt * P.dt * (v1 + v2);
      H[(size_t)i * N + j] = res;
      if (j > i) H[(size_t)j * N + i] = res;
    }
    c.sync();  // LDS reuse by the next pair
  }
  flush_stats(c, stats, b, 8.0 * b / 16.0 * 4.0, 0.0);
}

// body_row_overlaps on the padded layout (fast_overlap.hpp, P.oplan set): one
// wave per workgroup, the same pairs, the same H_ij assembly
__device__ inline OCG_INLINE void body_row_overlaps_pad(char* smem, OcgParams P, Pool pool, int xih_base0,
                                                        const int* rows, int nrows, const int* rbase, Pool rs,
                                                        const double* rnorm0, const zc* divT0, const zc* Fp, int N,
                                                        double* H0, double* stats, int K, int cs) {
  FastOverlap o(P, smem, P.oplan);
  // the row table after the overlap's region: the (row, column) search of every
  // pair runs on LDS instead of ~log2(rows) dependent global loads
  LDS int* RB = (LDS int*)(smem + P.ovl_bytes);
  LDS int* RW = RB + nrows + 1;
  o.init(P.oplan);
  for (int x = threadIdx.x; x <= nrows; x += 64) {
    RB[x] = rbase[x];
    if (x < nrows) RW[x] = rows[x];
  }
  o.wsync();
  const int total = RB[nrows];
  double b = 0;
  for (int g = blockIdx.x; g < K * total; g += gridDim.x) {
    const int kc = g / total, gl = g - kc * total;
    int lo = 0, hi = nrows - 1;  // row r with rbase[r] <= gl < rbase[r+1]
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (RB[mid] <= gl) lo = mid;
      else hi = mid - 1;
    }
    const int r = lo, i = RW[r], j = i + (gl - RB[r]);
    const int xih_base = xih_base0 + kc * cs;
    // the assembly's operands first: their loads overlap the contraction
    const zc* divT = divT0 + (size_t)kc * N;
    const zc F = Fp[kc], di = divT[i], dj = divT[j];
    const double rn = rnorm0[(size_t)kc * nrows + r];
    const int ny = o.load(SLOT_D(pool, P, xih_base + j), SLOT_X(pool, P, xih_base + j), SLOT_D(rs, P, g),
                          SLOT_X(rs, P, g));
    const zc ov = o.contract(o.YP);
    b += 32.0 * ny;
    if (threadIdx.x == 0) {
      double* H = H0 + (size_t)kc * N * N;
      const double v1 = (F.x * ov.x - F.y * ov.y) * (j > i ? rn : 1.0);  // Re(F <xiH_j|psiH> normiH)
      const double v2 = -(di.x * dj.x + di.y * dj.y);                  // -Re(divT_i conj(divT_j))
      const double res = P.dt * P.dt * (v1 + v2);
      H[(size_t)i * N + j] = res;
      if (j > i) H[(size_t)j * N + i] = res;
    }
    o.wsync();  // LDS reuse by the next pair
  }
  if (threadIdx.x == 0 && stats) {
    atomicAdd(stats + 0, b);
    atomicAdd(stats + 1, 8.0 * b / 16.0 * 4.0);
  }
}

// nsteps steps per state; u holds nsteps+1 controls per state (u_stride apart)
template <int NT>
__device__ OCG_INLINE void body_steps(char* smem, OcgParams P, const zc* gf, const zc* gb, const int* md,
                                              Pool pool, const int* slots, int n, const double* u, int u_stride,
                                              int nsteps, int forward, double* stats) {
  Chain<NT> c(P, smem);
  c.load_tables(gf, gb, md);
  int i = blockIdx.x;
  if (i >= n) return;
  double bytes = 0, flops = 0;
  const double* ui = u + (size_t)i * u_stride;
  if (fast_on(P)) {
    FastChain f(P, smem + P.fast_off, P.fplan, c.PROF);
    __syncthreads();  // load_tables' writes first: the region may alias them (P.fast_off = 0)
    f.init(P.fplan, gf, gb);
    f.load(SLOT_D(pool, P, slots[i]), SLOT_X(pool, P, slots[i]));
    for (int s = 0; s < nsteps; ++s) f.step(ui[s], ui[s + 1], forward);
    f.store(SLOT_D(pool, P, slots[i]), SLOT_X(pool, P, slots[i]));
    f.model_totals(bytes, flops);
    __syncthreads();
    flush_stats(c, stats, bytes, flops, double(nsteps));
    return;
  }
  c.load(SLOT_D(pool, P, slots[i]), SLOT_X(pool, P, slots[i]));
  for (int s = 0; s < nsteps; ++s) {
    c.step(ui[s], ui[s + 1], forward);
  }
  c.store(SLOT_D(pool, P, slots[i]), SLOT_X(pool, P, slots[i]));
  c.model_totals(bytes, flops);
  flush_stats(c, stats, bytes, flops, double(nsteps));
}


}  // namespace ocg
